/* copy_host_probe.c -- the host side of the per-object bounce copies: how
 * fast T threads copy 4 MiB blocks from a large pageable source (Go-heap
 * pages the caller owns) into a 4 MiB staging buffer of their own, with
 * glibc memcpy, with AVX2 non-temporal stores and with AVX-512 non-temporal
 * stores.  Prints GB/s per thread and in total, and CPU seconds per GB copied
 * (getrusage), per method and thread count.  Host only (no GPU).
 * build: cc -O2 -o tools/copy_host_probe tools/copy_host_probe.c -lpthread */
#define _GNU_SOURCE
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>

static const size_t kBlk = 4 << 20;
static size_t g_src_blocks = 512;  // 2 GiB of source per thread group
static uint8_t *g_src;
static int g_method, g_T;
static double g_seconds = 2.0;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static double cpu_s(void) {
    struct rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

__attribute__((target("avx2"))) static void copy_nt_avx2(uint8_t *d, const uint8_t *s, size_t n) {
    for (size_t i = 0; i < n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i *)(s + i));
        __m256i b = _mm256_loadu_si256((const __m256i *)(s + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i *)(s + i + 64));
        __m256i e = _mm256_loadu_si256((const __m256i *)(s + i + 96));
        _mm256_stream_si256((__m256i *)(d + i), a);
        _mm256_stream_si256((__m256i *)(d + i + 32), b);
        _mm256_stream_si256((__m256i *)(d + i + 64), c);
        _mm256_stream_si256((__m256i *)(d + i + 96), e);
    }
    _mm_sfence();
}

__attribute__((target("avx512f"))) static void copy_nt_avx512(uint8_t *d, const uint8_t *s, size_t n) {
    for (size_t i = 0; i < n; i += 256) {
        __m512i a = _mm512_loadu_si512((const void *)(s + i));
        __m512i b = _mm512_loadu_si512((const void *)(s + i + 64));
        __m512i c = _mm512_loadu_si512((const void *)(s + i + 128));
        __m512i e = _mm512_loadu_si512((const void *)(s + i + 192));
        _mm512_stream_si512((void *)(d + i), a);
        _mm512_stream_si512((void *)(d + i + 64), b);
        _mm512_stream_si512((void *)(d + i + 128), c);
        _mm512_stream_si512((void *)(d + i + 192), e);
    }
    _mm_sfence();
}

static double g_bytes[256];

static void *worker(void *vp) {
    const int t = (int)(intptr_t)vp;
    uint8_t *dst = aligned_alloc(4096, kBlk);
    memset(dst, 0, kBlk);
    double bytes = 0;
    size_t k = (size_t)t * 7;
    for (const double t0 = now(); now() - t0 < g_seconds;) {
        const uint8_t *src = g_src + (k++ % g_src_blocks) * kBlk;
        if (g_method == 0) memcpy(dst, src, kBlk);
        else if (g_method == 1) copy_nt_avx2(dst, src, kBlk);
        else copy_nt_avx512(dst, src, kBlk);
        bytes += kBlk;
    }
    g_bytes[t] = bytes;
    free(dst);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc > 1) g_seconds = atof(argv[1]);
    g_src = aligned_alloc(4096, g_src_blocks * kBlk);
    for (size_t i = 0; i < g_src_blocks * kBlk; i += 8) *(uint64_t *)(g_src + i) = i * 0x9E3779B97F4A7C15ull;
    const char *names[] = {"memcpy", "nt_avx2", "nt_avx512"};
    const int ts[] = {1, 4, 10, 20};
    for (int m = 0; m < 3; m++) {
        if (m == 2 && !__builtin_cpu_supports("avx512f")) continue;
        if (m == 1 && !__builtin_cpu_supports("avx2")) continue;
        for (unsigned ti = 0; ti < sizeof ts / sizeof ts[0]; ti++) {
            g_method = m;
            g_T = ts[ti];
            pthread_t th[256];
            const double c0 = cpu_s(), w0 = now();
            for (int t = 0; t < g_T; t++) pthread_create(&th[t], NULL, worker, (void *)(intptr_t)t);
            for (int t = 0; t < g_T; t++) pthread_join(th[t], NULL);
            const double wall = now() - w0, cpu = cpu_s() - c0;
            double b = 0;
            for (int t = 0; t < g_T; t++) b += g_bytes[t];
            printf("{\"method\": \"%s\", \"threads\": %d, \"GBs_total\": %.2f, \"GBs_per_thread\": %.2f, "
                   "\"cpu_s_per_GB\": %.4f}\n",
                   names[m], g_T, b / wall / 1e9, b / wall / 1e9 / g_T, cpu / (b / 1e9));
            fflush(stdout);
        }
    }
    return 0;
}

/* agg_bench.c -- the per-object call shape from C threads (no Python): T
 * threads each seal one 4 MiB block of pinned host memory per call through
 * the aggregator (jfsx_agg_seal), as the Go shim's upload goroutines do
 * (pkg/chunk/cached_store.go:415-472, max-uploads at cmd/flags.go:124-128).
 * Reports GB/s of plaintext for the aggregator and for direct one-block
 * jfsx_seal_batch calls, to separate the engine from the Python harness.
 *
 * usage: agg_bench [threads=20] [blocks=512] [passes=4] [max_mb=16] [window_us=500] [numa=0] [layout=0] [heap=0]
 * numa=1 binds the pinned blocks to the GPU's NUMA node and runs the threads
 * on that node's CPUs (as bench.py's host ingest does).
 * layout=0: thread t seals blocks t, t + T, ... of one pinned arena, so the
 * blocks in flight together are neighbours (a shim that hands out pages of
 * one pinned pool in order); layout=1: thread t owns a contiguous range of
 * blocks, so no two blocks in flight are adjacent (every caller with its own
 * buffers).
 * heap=1: the blocks live in ordinary pageable memory (malloc, as a Go-heap
 * slice), so the engine stages them through its pinned bounce buffers.
 * The aggregator run also reports the process's CPU time (getrusage) per GB
 * and the cores it kept busy: the host cost of the GPU path without Python.
 * build: cc -O2 -o tools/agg_bench tools/agg_bench.c -Iinclude -Ljuicefs_amd -ljfsx -lpthread \
 *        -Wl,-rpath,'$ORIGIN/../juicefs_amd' */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <time.h>

#include "jfsx.h"

static int T = 20, NB = 512, PASSES = 4;
static const uint64_t L = 4 << 20;
static uint8_t *hin, *hout, *hcrc;
static jfsx_ctx *ctx;
static jfsx_agg *agg;
static int use_agg, layout;

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *worker(void *vp) {
    const int t = (int)(intptr_t)vp;
    jfsx_blk *b = calloc(1, sizeof(jfsx_blk));
    const int per = NB / T;
    for (int pass = 0; pass < PASSES; pass++)
        for (int k = 0; layout ? k < per : t + k * T < NB; k++) {
            const int i = layout ? t * per + k : t + k * T;
            memset(b, 0, sizeof(*b));
            jfsx_gen_key(7, (uint64_t)i, b->key, b->nonce);
            b->src = hin + (uint64_t)i * L;
            b->dst = hout + (uint64_t)i * L;
            b->len = L;
            b->crc = hcrc + (uint64_t)i * 512;
            const int rc = use_agg ? jfsx_agg_seal(agg, JFSX_AES256GCM, b, JFSX_CRC_GEN, JFSX_MEM_HOST)
                                   : jfsx_seal_batch(ctx, JFSX_AES256GCM, 1, b, JFSX_CRC_GEN, JFSX_MEM_HOST);
            if (rc || b->status) {
                fprintf(stderr, "seal failed: rc %d status %d\n", rc, b->status);
                exit(1);
            }
        }
    free(b);
    return NULL;
}

static double cpu_s(void) {
    struct rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    return ru.ru_utime.tv_sec + ru.ru_utime.tv_usec * 1e-6 + ru.ru_stime.tv_sec + ru.ru_stime.tv_usec * 1e-6;
}

static double run(void) {
    pthread_t th[256];
    const double t0 = now();
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, (void *)(intptr_t)t);
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    const double blocks = layout ? (double)(NB / T) * T : (double)NB;
    return blocks * L * PASSES / (now() - t0) / 1e9;
}

int main(int argc, char **argv) {
    if (argc > 1) T = atoi(argv[1]);
    if (argc > 2) NB = atoi(argv[2]);
    if (argc > 3) PASSES = atoi(argv[3]);
    const uint64_t max_mb = argc > 4 ? strtoull(argv[4], 0, 10) : 16;
    const uint32_t window = argc > 5 ? (uint32_t)atoi(argv[5]) : 500;
    const int numa = argc > 6 ? atoi(argv[6]) : 0;
    layout = argc > 7 ? atoi(argv[7]) : 0;
    const int heap = argc > 8 ? atoi(argv[8]) : 0;
    int node = -1;
    if (numa && jfsx_device_numa_node(0, &node) == 0 && node >= 0) {
        char path[96], list[4096];
        snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
        FILE *f = fopen(path, "r");
        if (f && fgets(list, sizeof list, f)) {
            cpu_set_t set;
            CPU_ZERO(&set);
            for (char *p = list; *p && *p != '\n';) {
                const long a = strtol(p, &p, 10);
                const long b = *p == '-' ? strtol(p + 1, &p, 10) : a;
                for (long c = a; c <= b; c++) CPU_SET((int)c, &set);
                if (*p == ',') p++;
            }
            cpu_set_t cur;
            sched_getaffinity(0, sizeof cur, &cur);
            CPU_AND(&set, &set, &cur);
            if (CPU_COUNT(&set)) sched_setaffinity(0, sizeof set, &set);
        }
        if (f) fclose(f);
    }
    if (jfsx_ctx_open(0, 0, &ctx)) return 1;
    if (heap) {
        hin = aligned_alloc(4096, NB * L);
        hout = aligned_alloc(4096, NB * L);
        hcrc = aligned_alloc(4096, NB * 512);
        if (!hin || !hout || !hcrc) return 1;
        memset(hout, 0, NB * L);
    } else if (node >= 0) {
        if (jfsx_alloc_pinned_node(ctx, NB * L, node, (void **)&hin) ||
            jfsx_alloc_pinned_node(ctx, NB * L, node, (void **)&hout) ||
            jfsx_alloc_pinned_node(ctx, NB * 512, node, (void **)&hcrc))
            return 1;
    } else if (jfsx_alloc_pinned(ctx, NB * L, (void **)&hin) || jfsx_alloc_pinned(ctx, NB * L, (void **)&hout) ||
               jfsx_alloc_pinned(ctx, NB * 512, (void **)&hcrc))
        return 1;
    for (uint64_t i = 0; i < NB * L; i += 8) *(uint64_t *)(hin + i) = i * 0x9E3779B97F4A7C15ull;
    use_agg = 0;
    PASSES = 1;
    // warm the copy path up first: a cold box's D2H rate ramps up over the
    // first seconds of traffic (tools/pin_probe.hip)
    for (const double w0 = now(); now() - w0 < 8.0;) run();
    const int passes = argc > 3 ? atoi(argv[3]) : 4;
    PASSES = passes;
    const double direct = run();
    if (jfsx_agg_new(ctx, 0, max_mb << 20, window, &agg)) return 1;
    use_agg = 1;
    PASSES = 1;
    run();
    PASSES = passes;
    const double c0 = cpu_s(), w0 = now();
    const double aggr = run();
    const double cpu = cpu_s() - c0, wall = now() - w0;
    const double gb = aggr * wall;
    uint64_t calls, batches, blocks;
    jfsx_agg_stats(agg, &calls, &batches, &blocks);
    printf("{\"threads\": %d, \"blocks\": %d, \"passes\": %d, \"max_mb\": %llu, \"window_us\": %u, "
           "\"numa_node\": %d, \"layout\": %d, \"direct_GBs\": %.2f, \"agg_GBs\": %.2f, \"agg_batches\": %llu, \"agg_calls\": %llu, "
           "\"heap\": %d, \"agg_cpu_s_per_GB\": %.4f, \"agg_cores_busy\": %.2f}\n",
           T, NB, passes, (unsigned long long)max_mb, window, node, layout, direct, aggr, (unsigned long long)batches,
           (unsigned long long)calls, heap, cpu / gb, cpu / wall);
    jfsx_agg_free(agg);
    if (heap) {
        free(hin);
        free(hout);
        free(hcrc);
    } else {
        jfsx_free_pinned(ctx, hin);
        jfsx_free_pinned(ctx, hout);
        jfsx_free_pinned(ctx, hcrc);
    }
    jfsx_ctx_close(ctx);
    return 0;
}

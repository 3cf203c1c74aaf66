// pin_probe.hip -- does the page size behind pinned host memory change the
// copy rates the host pipeline sees?  (round 5: some processes saw one-block
// D2H-heavy calls 2.4x slower than others on the same box.)
// Compares, for 1 GiB of pinned memory:
//   A. hipHostMalloc (hipHostMallocPortable, as jfsx_alloc_pinned)
//   B. 2 MiB-aligned anonymous memory with madvise(MADV_HUGEPAGE), touched,
//      then hipHostRegister (transparent huge pages behind the DMA mappings)
// and reports the huge-page share of each region (/proc/self/smaps) and the
// H2D, D2H and duplex rates of 4 MiB copies.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/pin_probe tools/pin_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

static const size_t kTotal = (size_t)1 << 30, kChunk = (size_t)4 << 20;

// kB of AnonHugePages in the smaps entries overlapping [p, p + n)
static long huge_kb(const void *p, size_t n) {
    FILE *f = fopen("/proc/self/smaps", "r");
    if (!f) return -1;
    char line[512];
    unsigned long lo = 0, hi = 0;
    bool in = false;
    long kb = 0;
    const unsigned long a = (unsigned long)p, b = a + n;
    while (fgets(line, sizeof line, f)) {
        unsigned long x, y;
        if (sscanf(line, "%lx-%lx ", &x, &y) == 2 && strchr(line, '-') == line + strcspn(line, "-")) {
            lo = x;
            hi = y;
            in = hi > a && lo < b;
            continue;
        }
        long v;
        if (in && sscanf(line, "AnonHugePages: %ld kB", &v) == 1) kb += v;
    }
    fclose(f);
    return kb;
}

static void cat(const char *path) {
    FILE *f = fopen(path, "r");
    char buf[256] = "?";
    if (f) {
        if (!fgets(buf, sizeof buf, f)) strcpy(buf, "?\n");
        fclose(f);
    }
    printf("%s: %s", path, buf);
}

static double rate(char *h, char *d, int mode, hipStream_t a, hipStream_t b) {
    // mode 0: H2D, 1: D2H, 2: duplex (H2D first half of h, D2H second half)
    const int m = (int)(kTotal / kChunk);
    double best = 1e30;
    for (int rep = 0; rep < 3; rep++) {
        CK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < m; i++) {
            char *hp = h + (size_t)i * kChunk, *dp = d + (size_t)i * kChunk;
            if (mode == 0) CK(hipMemcpyAsync(dp, hp, kChunk, hipMemcpyHostToDevice, a));
            else if (mode == 1) CK(hipMemcpyAsync(hp, dp, kChunk, hipMemcpyDeviceToHost, b));
            else if (i < m / 2) {
                CK(hipMemcpyAsync(dp, hp, kChunk, hipMemcpyHostToDevice, a));
                CK(hipMemcpyAsync(hp + kTotal / 2, dp + kTotal / 2, kChunk, hipMemcpyDeviceToHost, b));
            }
        }
        CK(hipDeviceSynchronize());
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (ms < best) best = ms;
    }
    const double bytes = mode == 2 ? (double)kTotal / 2 : (double)kTotal;
    return bytes / best / 1e6;
}

int main() {
    cat("/sys/kernel/mm/transparent_hugepage/enabled");
    cat("/sys/kernel/mm/transparent_hugepage/defrag");
    CK(hipSetDevice(0));
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    char *d = nullptr;
    CK(hipMalloc((void **)&d, kTotal));
    CK(hipMemset(d, 1, kTotal));
    for (int kind = 0; kind < 2; kind++) {
        char *h = nullptr;
        if (kind == 0) {
            CK(hipHostMalloc((void **)&h, kTotal, hipHostMallocPortable));
            memset(h, 2, kTotal);
        } else {
            if (posix_memalign((void **)&h, (size_t)2 << 20, kTotal)) return 1;
            if (madvise(h, kTotal, MADV_HUGEPAGE)) perror("madvise");
            memset(h, 2, kTotal);
            CK(hipHostRegister(h, kTotal, hipHostRegisterPortable));
        }
        const long kb = huge_kb(h, kTotal);
        const double h2d = rate(h, d, 0, a, b), d2h = rate(h, d, 1, a, b), dup = rate(h, d, 2, a, b);
        printf("%-38s huge pages %5.1f %%  4 MiB copies: H2D %6.2f  D2H %6.2f  duplex %6.2f GB/s per direction\n",
               kind == 0 ? "hipHostMalloc" : "madvise(MADV_HUGEPAGE) + hipHostRegister",
               kb < 0 ? -1.0 : 100.0 * kb / (kTotal >> 10), h2d, d2h, dup);
        if (kind == 0) CK(hipHostFree(h));
        else {
            CK(hipHostUnregister(h));
            free(h);
        }
    }
    CK(hipFree(d));
    printf("pin probe ok\n");
    return 0;
}

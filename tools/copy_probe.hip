// copy_probe.hip -- how the host pipeline's copies behave by size and source
// (round 5, for the per-object path).  Times, on one GPU:
//   1. hipMemcpyAsync H2D / D2H in chunks of 256 KiB .. 64 MiB, back to back on
//      one stream, pinned host memory (hipHostMallocPortable, as the engine's)
//   2. the same D2H right after a kernel wrote the device source
//   3. zero-copy: a kernel that streams device -> pinned host (global stores
//      over PCIe) and host -> device (global loads over PCIe), 4 MiB per block
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/copy_probe tools/copy_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void fill_k(uint4 *p, size_t n16, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_uint4(v, v + 1, v + 2, (uint32_t)i);
}

// dst[i] = src[i] for n16 16-byte words; either side may be pinned host memory
__global__ void stream_k(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double elapsed_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main() {
    const size_t total = (size_t)256 << 20;
    void *h = nullptr, *d = nullptr;
    CK(hipSetDevice(0));
    CK(hipHostMalloc(&h, total, hipHostMallocPortable));
    CK(hipMalloc(&d, total));
    memset(h, 1, total);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t chunks[] = {256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20};
    printf("# hipMemcpyAsync, %zu MiB per pass, back to back on one stream\n", total >> 20);
    printf("%-8s %10s %10s %12s %12s %14s\n", "chunk", "H2D GB/s", "D2H GB/s", "H2D us/copy", "D2H us/copy",
           "D2H-after-k us");
    for (size_t ch : chunks) {
        const int n = (int)(total / ch);
        double t[3];
        for (int dir = 0; dir < 3; dir++) {
            double best = 1e30;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < n; i++) {
                    char *dp = (char *)d + i * ch, *hp = (char *)h + i * ch;
                    if (dir == 2) hipLaunchKernelGGL(fill_k, dim3(256), dim3(256), 0, s, (uint4 *)dp, ch / 16, i);
                    if (dir == 0) CK(hipMemcpyAsync(dp, hp, ch, hipMemcpyHostToDevice, s));
                    else CK(hipMemcpyAsync(hp, dp, ch, hipMemcpyDeviceToHost, s));
                }
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                const double ms = elapsed_ms(e0, e1);
                if (ms < best) best = ms;
            }
            t[dir] = best;
        }
        printf("%-8zu %10.2f %10.2f %12.1f %12.1f %14.1f\n", ch >> 10, total / t[0] / 1e6, total / t[1] / 1e6,
               t[0] * 1e3 / n, t[1] * 1e3 / n, t[2] * 1e3 / n);
    }
    printf("# zero-copy kernel streams (4 MiB per launch, 64 launches), grid x 256 threads\n");
    const size_t ch = 4 << 20;
    const int n = (int)(total / ch);
    for (int grid : {64, 256, 1024, 4096}) {
        double best[2] = {1e30, 1e30};
        for (int dir = 0; dir < 2; dir++)
            for (int rep = 0; rep < 3; rep++) {
                CK(hipStreamSynchronize(s));
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < n; i++) {
                    char *dp = (char *)d + i * ch, *hp = (char *)h + i * ch;
                    if (dir == 0)
                        hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, s, (const uint4 *)hp, (uint4 *)dp, ch / 16);
                    else
                        hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, s, (const uint4 *)dp, (uint4 *)hp, ch / 16);
                }
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                const double ms = elapsed_ms(e0, e1);
                if (ms < best[dir]) best[dir] = ms;
            }
        CK(hipGetLastError());
        printf("grid %5d   host->dev %8.2f GB/s   dev->host %8.2f GB/s\n", grid, total / best[0] / 1e6,
               total / best[1] / 1e6);
    }
    // both directions at once on two streams (kernel reads host, kernel writes host)
    {
        hipStream_t s2;
        CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        void *h2 = nullptr, *d2 = nullptr;
        CK(hipHostMalloc(&h2, total, hipHostMallocPortable));
        CK(hipMalloc(&d2, total));
        double best = 1e30;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, s));
            CK(hipStreamWaitEvent(s2, e0, 0));
            for (int i = 0; i < n; i++) {
                hipLaunchKernelGGL(stream_k, dim3(1024), dim3(256), 0, s, (const uint4 *)((char *)h + i * ch),
                                   (uint4 *)((char *)d + i * ch), ch / 16);
                hipLaunchKernelGGL(stream_k, dim3(1024), dim3(256), 0, s2, (const uint4 *)((char *)d2 + i * ch),
                                   (uint4 *)((char *)h2 + i * ch), ch / 16);
            }
            hipEvent_t e2;
            CK(hipEventCreate(&e2));
            CK(hipEventRecord(e2, s2));
            CK(hipStreamWaitEvent(s, e2, 0));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            const double ms = elapsed_ms(e0, e1);
            if (ms < best) best = ms;
            CK(hipEventDestroy(e2));
        }
        printf("zero-copy duplex (grid 1024 each way): %8.2f GB/s per direction\n", total / best / 1e6);
    }
    // SDMA duplex with 4 MiB chunks (the pipeline's copy size)
    {
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        void *h2 = nullptr, *d2 = nullptr;
        CK(hipHostMalloc(&h2, total, hipHostMallocPortable));
        CK(hipMalloc(&d2, total));
        for (size_t c2 : {(size_t)4 << 20, (size_t)16 << 20, (size_t)64 << 20}) {
            const int m = (int)(total / c2);
            double best = 1e30;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, a));
                CK(hipStreamWaitEvent(b, e0, 0));
                for (int i = 0; i < m; i++) {
                    CK(hipMemcpyAsync((char *)d + i * c2, (char *)h + i * c2, c2, hipMemcpyHostToDevice, a));
                    CK(hipMemcpyAsync((char *)h2 + i * c2, (char *)d2 + i * c2, c2, hipMemcpyDeviceToHost, b));
                }
                hipEvent_t e2;
                CK(hipEventCreate(&e2));
                CK(hipEventRecord(e2, b));
                CK(hipStreamWaitEvent(a, e2, 0));
                CK(hipEventRecord(e1, a));
                CK(hipEventSynchronize(e1));
                const double ms = elapsed_ms(e0, e1);
                if (ms < best) best = ms;
                CK(hipEventDestroy(e2));
            }
            printf("SDMA duplex, %3zu MiB copies: %8.2f GB/s per direction\n", c2 >> 20, total / best / 1e6);
        }
    }
    // mixed duplex: SDMA one way, a streaming kernel the other; and one kernel
    // that reads pinned host memory and writes pinned host memory (a fused
    // zero-copy transform's traffic), 4 MiB per launch
    {
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        void *h2 = nullptr, *d2 = nullptr;
        CK(hipHostMalloc(&h2, total, hipHostMallocPortable));
        CK(hipMalloc(&d2, total));
        const size_t c2 = 4 << 20;
        const int m = (int)(total / c2);
        for (int mode = 0; mode < 4; mode++) {
            for (int grid : {64, 256, 1024}) {
                double best = 1e30;
                for (int rep = 0; rep < 3; rep++) {
                    CK(hipDeviceSynchronize());
                    CK(hipEventRecord(e0, a));
                    CK(hipStreamWaitEvent(b, e0, 0));
                    for (int i = 0; i < m; i++) {
                        char *hp = (char *)h + i * c2, *dp = (char *)d + i * c2, *hp2 = (char *)h2 + i * c2,
                             *dp2 = (char *)d2 + i * c2;
                        if (mode == 0) {  // SDMA H2D + kernel D2H
                            CK(hipMemcpyAsync(dp, hp, c2, hipMemcpyHostToDevice, a));
                            hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, b, (const uint4 *)dp2, (uint4 *)hp2, c2 / 16);
                        } else if (mode == 1) {  // kernel H2D + SDMA D2H
                            hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, a, (const uint4 *)hp, (uint4 *)dp, c2 / 16);
                            CK(hipMemcpyAsync(hp2, dp2, c2, hipMemcpyDeviceToHost, b));
                        } else if (mode == 2) {  // kernel H2D + kernel D2H, both at `grid`
                            hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, a, (const uint4 *)hp, (uint4 *)dp, c2 / 16);
                            hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, b, (const uint4 *)dp2, (uint4 *)hp2, c2 / 16);
                        } else {  // one kernel: host -> host
                            hipLaunchKernelGGL(stream_k, dim3(grid), dim3(256), 0, a, (const uint4 *)hp, (uint4 *)hp2, c2 / 16);
                        }
                    }
                    hipEvent_t e2;
                    CK(hipEventCreate(&e2));
                    CK(hipEventRecord(e2, b));
                    CK(hipStreamWaitEvent(a, e2, 0));
                    CK(hipEventRecord(e1, a));
                    CK(hipEventSynchronize(e1));
                    const double ms = elapsed_ms(e0, e1);
                    if (ms < best) best = ms;
                    CK(hipEventDestroy(e2));
                }
                static const char *names[] = {"SDMA H2D + kernel D2H", "kernel H2D + SDMA D2H",
                                              "kernel H2D + kernel D2H", "one kernel host -> host"};
                printf("%-26s grid %5d: %8.2f GB/s per direction\n", names[mode], grid, total / best / 1e6);
            }
        }
        for (size_t c3 : {(size_t)128 << 20, (size_t)256 << 20}) {  // SDMA duplex at the ring's slot sizes
            const int k = (int)(total / c3);
            double best = 1e30;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, a));
                CK(hipStreamWaitEvent(b, e0, 0));
                for (int i = 0; i < k; i++) {
                    CK(hipMemcpyAsync((char *)d + i * c3, (char *)h + i * c3, c3, hipMemcpyHostToDevice, a));
                    CK(hipMemcpyAsync((char *)h2 + i * c3, (char *)d2 + i * c3, c3, hipMemcpyDeviceToHost, b));
                }
                hipEvent_t e2;
                CK(hipEventCreate(&e2));
                CK(hipEventRecord(e2, b));
                CK(hipStreamWaitEvent(a, e2, 0));
                CK(hipEventRecord(e1, a));
                CK(hipEventSynchronize(e1));
                const double ms = elapsed_ms(e0, e1);
                if (ms < best) best = ms;
                CK(hipEventDestroy(e2));
            }
            printf("SDMA duplex, %3zu MiB copies: %8.2f GB/s per direction\n", c3 >> 20, total / best / 1e6);
        }
    }
    // SDMA duplex with 4 MiB copies spread round-robin over k streams per
    // direction (more copy engines / queues in flight per direction?)
    for (int k : {1, 2, 4}) {
        hipStream_t a[4], b[4];
        for (int j = 0; j < k; j++) {
            CK(hipStreamCreateWithFlags(&a[j], hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&b[j], hipStreamNonBlocking));
        }
        void *h2 = nullptr, *d2 = nullptr;
        CK(hipHostMalloc(&h2, total, hipHostMallocPortable));
        CK(hipMalloc(&d2, total));
        const size_t c2 = 4 << 20;
        const int m = (int)(total / c2);
        double best = 1e30;
        for (int rep = 0; rep < 3; rep++) {
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < m; i++) {
                CK(hipMemcpyAsync((char *)d + i * c2, (char *)h + i * c2, c2, hipMemcpyHostToDevice, a[i % k]));
                CK(hipMemcpyAsync((char *)h2 + i * c2, (char *)d2 + i * c2, c2, hipMemcpyDeviceToHost, b[i % k]));
            }
            CK(hipDeviceSynchronize());
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (ms < best) best = ms;
        }
        printf("SDMA duplex, 4 MiB copies over %d stream(s) per direction: %8.2f GB/s per direction\n", k,
               total / best / 1e6);
        for (int j = 0; j < k; j++) {
            CK(hipStreamDestroy(a[j]));
            CK(hipStreamDestroy(b[j]));
        }
        CK(hipHostFree(h2));
        CK(hipFree(d2));
    }
    // SDMA duplex, 4 MiB copies submitted g at a time through
    // hipMemcpyBatchAsync (one call per group of g scattered blocks)
    {
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        void *h2 = nullptr, *d2 = nullptr;
        CK(hipHostMalloc(&h2, total, hipHostMallocPortable));
        CK(hipMalloc(&d2, total));
        const size_t c2 = 4 << 20;
        const int m = (int)(total / c2);
        for (int g : {1, 3, 8}) {
            double best = 1e30;
            for (int rep = 0; rep < 3; rep++) {
                CK(hipDeviceSynchronize());
                const auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < m; i += g) {
                    const int k = i + g <= m ? g : m - i;
                    void *di[8], *si[8], *dd[8], *sd[8];
                    size_t sz[8];
                    for (int j = 0; j < k; j++) {
                        // scattered: every other 4 MiB block, wrapping
                        const size_t o = (size_t)((2 * (i + j)) % m + ((2 * (i + j)) / m) % 2) * c2;
                        di[j] = (char *)d + o;
                        si[j] = (char *)h + o;
                        dd[j] = (char *)h2 + o;
                        sd[j] = (char *)d2 + o;
                        sz[j] = c2;
                    }
                    size_t fail = 0;
                    CK(hipMemcpyBatchAsync(di, si, sz, (size_t)k, nullptr, nullptr, 0, &fail, a));
                    CK(hipMemcpyBatchAsync(dd, sd, sz, (size_t)k, nullptr, nullptr, 0, &fail, b));
                }
                CK(hipDeviceSynchronize());
                const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                if (ms < best) best = ms;
            }
            printf("SDMA duplex, 4 MiB copies via hipMemcpyBatchAsync, %d per call: %8.2f GB/s per direction\n", g,
                   total / best / 1e6);
        }
        CK(hipHostFree(h2));
        CK(hipFree(d2));
    }
    printf("copy probe ok\n");
    return 0;
}

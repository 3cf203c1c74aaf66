// PCIe duplex probe (measurement tool): H2D and D2H alone and together, by
// SDMA (hipMemcpyAsync on two streams) and by shader copies that read / write
// pinned host memory directly (zero-copy), one kernel per direction.
// Usage: pcie_duplex [MiB per copy] [chunks]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void copy16(uint4 *__restrict__ dst, const uint4 *__restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main(int argc, char **argv) {
    size_t mib = argc > 1 ? atoi(argv[1]) : 256;
    int chunks = argc > 2 ? atoi(argv[2]) : 8;
    size_t bytes = mib << 20, ch = bytes / chunks;
    char *hA, *hB, *dA, *dB;
    CK(hipHostMalloc((void **)&hA, bytes, 0));
    CK(hipHostMalloc((void **)&hB, bytes, 0));
    CK(hipMalloc((void **)&dA, bytes));
    CK(hipMalloc((void **)&dB, bytes));
    memset(hA, 1, bytes); memset(hB, 2, bytes);
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto run = [&](bool h2d, bool d2h, bool kern, int grid) {
        double best = 1e9;
        for (int it = 0; it < 5; it++) {
            CK(hipDeviceSynchronize());
            double t0 = now();
            for (int c = 0; c < chunks; c++) {
                if (kern) {
                    if (h2d) hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s1, (uint4 *)(dA + c * ch), (const uint4 *)(hA + c * ch), ch / 16);
                    if (d2h) hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s2, (uint4 *)(hB + c * ch), (const uint4 *)(dB + c * ch), ch / 16);
                } else {
                    if (h2d) CK(hipMemcpyAsync(dA + c * ch, hA + c * ch, ch, hipMemcpyHostToDevice, s1));
                    if (d2h) CK(hipMemcpyAsync(hB + c * ch, dB + c * ch, ch, hipMemcpyDeviceToHost, s2));
                }
            }
            CK(hipStreamSynchronize(s1));
            CK(hipStreamSynchronize(s2));
            double t = now() - t0;
            if (t < best) best = t;
        }
        double gb = (double)bytes * ((int)h2d + (int)d2h) / 1e9;
        printf("%-5s %-4s %-4s grid %4d %8.2f GB/s total  (%.3f ms)\n", kern ? "kern" : "sdma", h2d ? "H2D" : "",
               d2h ? "D2H" : "", kern ? grid : 0, gb / best, best * 1e3);
    };
    run(true, false, false, 0);
    run(false, true, false, 0);
    run(true, true, false, 0);
    for (int grid : {64, 256, 1024}) {
        run(true, false, true, grid);
        run(false, true, true, grid);
        run(true, true, true, grid);
    }
    return 0;
}

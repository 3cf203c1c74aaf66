// Table-lookup throughput probe (measurement tool, not product code).
// T-table AES-256 is bound by LDS lookups (2 LDS cycles per wave64
// ds_read_b32): this measures how many random 32-bit lookups per clock per CU
// the other paths deliver -- global loads that hit the vector L1 (a 1 or 4 KiB
// table), and mixes of LDS and L1 lookups in one wave -- so the GCM kernel
// can decide whether moving part of its lookups to the L1 pays.
// Each lane runs CH independent chains x <- rotl8(x) ^ T[byte(x)] (the shape
// of an AES column), 16 waves per CU, one workgroup per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH 8
#define WAVES 16
typedef __attribute__((address_space(1))) const uint32_t gu32;
typedef __attribute__((address_space(3))) const uint32_t lu32;

__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }

// MODE 0: LDS only (replicated, conflict-free); 1: L1 only, 1 KiB table;
// 2: L1 only, 4 KiB table (byte k of x picks sub-table k);
// 3: 2 LDS : 1 L1; 4: 1 LDS : 1 L1; 5: 3 LDS : 1 L1; 6: L1 only, 16 KiB
template <int MODE>
__global__ __launch_bounds__(WAVES * 64) void probe(const uint32_t *__restrict__ gtab, uint32_t *out, uint32_t seed,
                                                    int iters) {
    __shared__ uint32_t lds[256 * 64];  // entry idx at byte idx*256 + 4*replica (as the GCM kernel's T0|T2)
    for (uint32_t i = threadIdx.x; i < 256 * 64; i += blockDim.x) lds[i] = gtab[i >> 6];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t loff = (lane & 31) << 2;
    gu32 *g = (gu32 *)gtab;
    lu32 *l = (lu32 *)lds;
    uint32_t x[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) x[i] = seed * (threadIdx.x + 1 + 64 * blockIdx.x) + i * 0x9e3779b9u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < CH; i++) {
            // byte 0 of x as the index; the LDS address (idx << 7) | replica
            const uint32_t la = __builtin_amdgcn_perm(x[i], loff, 0x0c0c0400u);  // (b0 << 8) | loff
            const uint32_t ga = (x[i] & 0xffu) << 2;
            uint32_t v;
            if constexpr (MODE == 0) v = *(const lu32 *)((const __attribute__((address_space(3))) char *)l + la);
            else if constexpr (MODE == 1) v = *(gu32 *)((__attribute__((address_space(1))) const char *)g + ga);
            else if constexpr (MODE == 2) v = *(gu32 *)((__attribute__((address_space(1))) const char *)g + ga + ((i & 3) << 10));
            else if constexpr (MODE == 6) v = *(gu32 *)((__attribute__((address_space(1))) const char *)g + ga + ((i & 15) << 10));
            else {
                constexpr int per = MODE == 3 ? 3 : (MODE == 4 ? 2 : 4);  // one L1 lookup per `per`
                if (i % per == per - 1) v = *(gu32 *)((__attribute__((address_space(1))) const char *)g + ga);
                else v = *(const lu32 *)((const __attribute__((address_space(3))) char *)l + la);
            }
            x[i] = rotl8(x[i]) ^ v;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) r ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kfn)(const uint32_t *, uint32_t *, uint32_t, int);

int main() {
    kfn fns[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>};
    const char *names[] = {"LDS ds_read_b32 (32 replicas)", "L1 global_load_dword, 1 KiB table",
                           "L1 global_load_dword, 4 KiB table", "2 LDS : 1 L1", "1 LDS : 1 L1", "3 LDS : 1 L1",
                           "L1 global_load_dword, 16 KiB table"};
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    uint32_t *tab, *out;
    hipMalloc(&tab, 16384 * 4);
    hipMalloc(&out, (size_t)cus * 4 * WAVES * 64 * 4);
    uint32_t h[16384];
    for (int i = 0; i < 16384; i++) h[i] = 0x9e3779b9u * (i + 1) ^ (i << 13);
    hipMemcpy(tab, h, sizeof h, hipMemcpyHostToDevice);
    const int iters = 4096;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    printf("CUs %d, clock %d kHz; lookups per clock per CU at 2.4 GHz\n", cus, prop.clockRate);
    for (int m = 0; m < 7; m++) {
        for (int grid_mul = 1; grid_mul <= 2; grid_mul++) {
            const int grid = cus * grid_mul;
            hipLaunchKernelGGL(fns[m], dim3(grid), dim3(WAVES * 64), 0, 0, tab, out, 7u, 64);
            hipEventRecord(a);
            hipLaunchKernelGGL(fns[m], dim3(grid), dim3(WAVES * 64), 0, 0, tab, out, 7u, iters);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double lookups = (double)grid * WAVES * 64 * CH * iters;
            printf("%-36s grid %4d: %8.3f ms  %.2f lookups/clk/CU (%.1f G lookups/s)\n", names[m], grid, ms,
                   lookups / (ms * 1e-3) / cus / 2.4e9, lookups / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}

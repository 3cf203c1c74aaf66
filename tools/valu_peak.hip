// VALU issue-rate probe for the bitsliced AES (measurement tool, not product code):
// independent v_bitop3_b32 / v_xor_b32 / add+alignbit / v_mad_u64_u32 streams
// at 2 and 4 waves per SIMD (rates in wave-instructions of the loop body; mode
// 3 is two instructions per element, mode 4 is one mad plus one xor).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int MODE>
__global__ __launch_bounds__(1024) void probe(uint32_t *out, uint32_t seed, int iters) {
    uint32_t r[32];
#pragma unroll
    for (int i = 0; i < 32; i++) r[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 32; i++) {
            const uint32_t a = r[(i + 5) & 31], b = r[(i + 11) & 31];
            if (MODE == 0) r[i] = __builtin_amdgcn_bitop3_b32(r[i], a, b, 0x96);       // 3 VGPR sources
            else if (MODE == 1) r[i] = r[i] ^ a;                                        // v_xor_b32
            else if (MODE == 2) r[i] = __builtin_amdgcn_bitop3_b32(r[i], a, seed, 0x96); // 2 VGPR + SGPR
            else if (MODE == 3) r[i] = __builtin_amdgcn_alignbit(r[i] + a, r[i] + a, 16);  // v_add + v_alignbit
            else {  // v_mad_u64_u32 (Poly1305 limb products)
                const uint64_t m = (uint64_t)r[i] * a + b;
                r[i] = (uint32_t)m ^ (uint32_t)(m >> 32);
            }
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) x ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

int main() {
    uint32_t *out;
    hipMalloc(&out, 1024 * 1024 * 4 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    for (int mode = 0; mode < 5; mode++) {
        for (int wps : {2, 4}) {  // waves per SIMD: 256 CUs x 4 SIMDs
            const int threads = 256 * wps;  // per workgroup: 4*wps waves -> one WG per CU
            const int blocks = 256;
            float best = 1e9;
            for (int rep = 0; rep < 3; rep++) {
                hipEventRecord(e0);
                if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(blocks), dim3(threads), 0, 0, out, 7u, iters);
                if (mode == 1) hipLaunchKernelGGL(probe<1>, dim3(blocks), dim3(threads), 0, 0, out, 7u, iters);
                if (mode == 2) hipLaunchKernelGGL(probe<2>, dim3(blocks), dim3(threads), 0, 0, out, 7u, iters);
                if (mode == 3) hipLaunchKernelGGL(probe<3>, dim3(blocks), dim3(threads), 0, 0, out, 7u, iters);
                if (mode == 4) hipLaunchKernelGGL(probe<4>, dim3(blocks), dim3(threads), 0, 0, out, 7u, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            const double winstr = (double)blocks * threads / 64 * iters * 32;  // wave-instructions
            const double per_simd_per_ns = winstr / 1024 / (best * 1e6);
            printf("mode %d waves/SIMD %d: %.3f ms, %.3f wave-instr/ns/SIMD (%.3f per cycle @2.4GHz)\n", mode, wps, best,
                   per_simd_per_ns, per_simd_per_ns / 2.4);
        }
    }
    return 0;
}

// VALU issue-rate probe (measurement tool, not product code): wave64 issue
// cost of the instructions the ChaCha20-Poly1305 and GCM kernels lean on,
// and of the candidates for a cheaper Poly1305 multiply.  Each mode runs 8
// independent dependency chains of one instruction per lane (inline asm, so
// the compiler cannot fold them), one 1024-thread workgroup per CU (4 waves
// per SIMD).  Prints cycles per wave-instruction per SIMD at the measured
// clock-free rate (ns) and at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CH 8
template <int MODE>
__global__ __launch_bounds__(1024) void probe(uint32_t *out, uint32_t seed, int iters) {
    uint32_t r[CH], s[CH];
    double f[CH];
    uint64_t q[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) {
        r[i] = seed * (threadIdx.x + 1) + i * 0x9e3779b9u;
        s[i] = r[i] ^ 0x5bd1e995u;
        f[i] = (double)(r[i] & 0xfffff);
        q[i] = ((uint64_t)s[i] << 32) | r[i];
    }
    const uint32_t k = seed | 1u;
    const double fk = 1.0000001;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < CH; i++) {
            if constexpr (MODE == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(s[i]));
            else if constexpr (MODE == 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(s[i]));
            else if constexpr (MODE == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(r[i]));
            else if constexpr (MODE == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(s[i]), "v"(k));
            else if constexpr (MODE == 4) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(q[i]) : "v"(r[i]), "v"(s[i]));
            else if constexpr (MODE == 5) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(r[i]) : "v"(s[i]));
            else if constexpr (MODE == 6) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(r[i]) : "v"(s[i]));
            else if constexpr (MODE == 7) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(r[i]) : "v"(s[i]));
            else if constexpr (MODE == 8) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(r[i]) : "v"(s[i]));
            else if constexpr (MODE == 9) asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(f[i]) : "v"(fk));
            else if constexpr (MODE == 10) asm volatile("v_add_f64 %0, %0, %1" : "+v"(f[i]) : "v"(fk));
            else if constexpr (MODE == 11) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r[i]) : "v"(s[i]), "v"(k));
            else if constexpr (MODE == 12) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(s[i]), "v"(k));
            else if constexpr (MODE == 13) asm volatile("v_lshl_add_u64 %0, %0, 2, %1" : "+v"(q[i]) : "v"(q[(i + 1) % CH]));
            else if constexpr (MODE == 14) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(s[i]), "v"(k));
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) x ^= r[i] ^ (uint32_t)q[i] ^ (uint32_t)(q[i] >> 32) ^ (uint32_t)f[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

typedef void (*kfn)(uint32_t *, uint32_t, int);
static const char *names[] = {"v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_perm_b32", "v_mad_u64_u32",
                              "v_mad_u32_u24", "v_mul_hi_u32_u24", "v_mul_lo_u32", "v_mul_hi_u32", "v_fma_f64",
                              "v_add_f64", "v_bitop3_b32", "v_add3_u32", "v_lshl_add_u64", "v_xad_u32"};

int main() {
    kfn fns[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>, probe<6>, probe<7>,
                 probe<8>, probe<9>, probe<10>, probe<11>, probe<12>, probe<13>, probe<14>};
    uint32_t *out;
    if (hipMalloc(&out, 256 * 1024 * 4) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    for (int m = 0; m < 15; m++) {
        float best = 1e9;
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(fns[m], dim3(256), dim3(1024), 0, 0, out, 7u, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        // 256 WGs x 16 waves x iters x CH wave-instructions, over 1024 SIMDs
        const double per_simd = 16.0 * iters * CH / 4;  // wave-instructions per SIMD
        const double ns_each = best * 1e6 / per_simd;
        printf("%-18s %.3f ms  %.3f ns/wave-instr/SIMD  = %.2f cycles @2.4GHz\n", names[m], best, ns_each,
               ns_each * 2.4);
    }
    return 0;
}

// LDS probe (measurement tool, not product code): does a byte-misaligned
// ds_read_b32 return the right bytes on gfx950, and what does it cost next to
// an aligned ds_read_b32 / ds_read_b64, with the T-table replica layouts the
// GCM kernel would use?
//   mode 0: aligned b32, row 256 B, lane l -> dword (l & 31)      (current T0 layout)
//   mode 1: unaligned b32, row 256 B, lane l -> byte 8 (l & 31) + k, k = 1..3
//   mode 2: aligned b32 at byte 8 (l & 31) (k = 0 of mode 1's layout)
//   mode 3: aligned b64 at byte 8 (l & 31)
//   mode 4: unaligned b32, row 256 B, lane l -> byte 4 (l & 31) + k (4-B stride)
// Each lane walks 8 independent chains: row = (previous value) & 255.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(1024) void probe(uint32_t *out, int iters) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[65536 + 64];
    for (uint32_t i = threadIdx.x; i < 65536 / 4; i += 1024)
        reinterpret_cast<uint32_t *>(lds)[i] = i * 0x9e3779b9u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint32_t v[8];
#pragma unroll
    for (int c = 0; c < 8; c++) v[c] = (lane * 7 + c * 13) & 255;
    uint64_t acc64 = 0;
    for (int it = 0; it < iters; it++) {
        uint32_t r[8];
        uint64_t q[8];
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const uint32_t row = (v[c] & 255u) << 8;
            uint32_t a;
            if (MODE == 0) a = row | ((lane & 31) << 2);
            else if (MODE == 1) a = row | ((lane & 31) << 3) | (1 + (c % 3));
            else if (MODE == 2 || MODE == 3) a = row | ((lane & 31) << 3);
            else a = row | ((lane & 31) << 2) | (1 + (c % 3));
            if (MODE == 3) asm volatile("ds_read_b64 %0, %1" : "=v"(q[c]) : "v"(a));
            else asm volatile("ds_read_b32 %0, %1" : "=v"(r[c]) : "v"(a));
        }
        if (MODE == 3) {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]), "+v"(q[4]),
                         "+v"(q[5]), "+v"(q[6]), "+v"(q[7]));
#pragma unroll
            for (int c = 0; c < 8; c++) v[c] = (uint32_t)q[c] ^ (uint32_t)(q[c] >> 32) ^ (v[c] >> 8);
        } else {
            asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]),
                         "+v"(r[5]), "+v"(r[6]), "+v"(r[7]));
#pragma unroll
            for (int c = 0; c < 8; c++) v[c] = r[c] ^ (v[c] >> 8);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < 8; c++) x ^= v[c];
    out[blockIdx.x * 1024 + threadIdx.x] = x ^ (uint32_t)acc64;
}

// correctness: unaligned reads against the byte image
__global__ void check(uint32_t *bad) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4096];
    for (uint32_t i = threadIdx.x; i < 4096; i += 64) lds[i] = (unsigned char)(i * 37 + 11);
    __syncthreads();
    uint32_t errs = 0;
    for (uint32_t off = threadIdx.x; off < 4000; off += 64) {
        uint32_t r;
        asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(off));
        uint32_t want = 0;
        for (int b = 0; b < 4; b++) want |= (uint32_t)(unsigned char)((off + b) * 37 + 11) << (8 * b);
        errs += r != want;
    }
    atomicAdd(bad, errs);
}

typedef void (*kfn)(uint32_t *, int);

int main() {
    uint32_t *out, *bad;
    if (hipMalloc(&out, 256 * 1024 * 4) != hipSuccess || hipMalloc(&bad, 4) != hipSuccess) return 1;
    (void)hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, bad);
    uint32_t nb = 0;
    (void)hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
    printf("unaligned ds_read_b32 mismatches: %u of 4000\n", nb);
    kfn fns[] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>};
    const char *names[] = {"aligned b32 4-B replica stride", "UNALIGNED b32 8-B replica stride",
                           "aligned b32 8-B replica stride", "aligned b64 8-B replica stride",
                           "UNALIGNED b32 4-B replica stride"};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 4000;
    for (int m = 0; m < 5; m++) {
        float best = 1e9;
        for (int rep = 0; rep < 3; rep++) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(fns[m], dim3(256), dim3(1024), 0, 0, out, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double per_cu = 16.0 * iters * 8;  // wave-instructions per CU
        printf("%-36s %.3f ms  %.3f ns per wave-read per CU (%.2f cycles @2.4GHz)\n", names[m], best,
               best * 1e6 / per_cu, best * 1e6 / per_cu * 2.4);
    }
    return 0;
}

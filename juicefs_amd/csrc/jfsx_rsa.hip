// jfsx_rsa.hip -- batched RSA-OAEP key unwrap on the GPU.
//
// rsaEncryptor.Decrypt (pkg/object/encrypt.go:124-134) runs once per object
// the reference opens (encrypt.go:207-210): an RSA-2048 private operation of
// ~0.35 ms per core, which caps end-to-end Decrypt far below the Open kernel.
// Here one batch unwraps every object key of a read window on the GPU:
//   * rsa_half_k: one thread per (object, CRT half): c mod p_h, then
//     c^d_h mod p_h by a fixed-window Montgomery exponentiation (32-limb CIOS,
//     jfsx_rsa.h), constant time in the exponent.
//   * rsa_finish_k: one thread per object: c < n check, CRT recombination,
//     EME-OAEP decoding (SHA-256, MGF1, label hash), message out.
// Bit-exact to rsa.DecryptOAEP(sha256, ..., "keys") and, like it, constant
// time with respect to the private key and the decrypted data (jfsx_rsa.h):
// no branch and no memory address depends on the exponent, the CRT values or
// the OAEP checks; the one branch on secret-derived data is the final valid /
// invalid outcome, which Go's decryptOAEP also returns as an error.
#include "jfsx_internal.h"

#define JFSX_HD __device__ __forceinline__
#include "jfsx_rsa.h"

namespace jfsx {

using jfsx_rsa::kLimbs;
using jfsx_rsa::kModBytes;

// x^e mod m on jfsx_rsa.h's constant-time schedule (kDigits fixed 4-bit
// digits over the full prime length, four squarings and one multiply per
// digit, the window entry picked by a masked scan of all 16), with one
// Montgomery multiply site: the unrolled CIOS is ~6K instructions, and one
// copy keeps the loop inside the instruction cache.  The step sequence is a
// function of the step counter alone; the exponent only feeds the masks,
// which pass through a register barrier so the compiler cannot turn them
// back into a secret-dependent branch or a secret-indexed load.
__device__ __forceinline__ void mod_exp_ct(const uint32_t *x, const uint32_t *e, const uint32_t *m, uint32_t minv,
                                           const uint32_t *r2, uint32_t *out) {
    using jfsx_rsa::kDigits;
    uint32_t tab[16][kLimbs];  // tab[j] = x^j R mod m
    uint32_t acc[kLimbs], b[kLimbs];
    constexpr int kTab = 16, kMain = kTab + 5 * kDigits;  // steps: table, digits, leave the domain
#pragma unroll 1
    for (int st = 0; st <= kMain; st++) {
        if (st == 0) {  // R mod m = r2 * 1
#pragma unroll
            for (int j = 0; j < kLimbs; j++) acc[j] = r2[j], b[j] = j == 0;
        } else if (st == 1) {  // x R mod m
#pragma unroll
            for (int j = 0; j < kLimbs; j++) acc[j] = x[j], b[j] = r2[j];
        } else if (st < kTab) {  // tab[st] = tab[st - 1] * x R
#pragma unroll
            for (int j = 0; j < kLimbs; j++) b[j] = tab[1][j];
        } else if (st < kMain) {
            const int r = st - kTab;
            if (r % 5 < 4) {
#pragma unroll
                for (int j = 0; j < kLimbs; j++) b[j] = acc[j];
            } else {
                uint32_t idx = jfsx_rsa::exp_digit(e, kDigits - 1 - r / 5);
                asm volatile("" : "+v"(idx));
#pragma unroll
                for (int j = 0; j < kLimbs; j++) b[j] = 0;
#pragma unroll
                for (uint32_t w = 0; w < 16; w++) {
                    uint32_t msk = ~jfsx_rsa::ct_nz(w ^ idx);
                    asm volatile("" : "+v"(msk));
#pragma unroll
                    for (int j = 0; j < kLimbs; j++) b[j] |= tab[w][j] & msk;
                }
            }
        } else {  // out of the Montgomery domain
#pragma unroll
            for (int j = 0; j < kLimbs; j++) b[j] = j == 0;
        }
        jfsx_rsa::mont_mul(acc, b, m, minv, acc);
        if (st < kTab) {
#pragma unroll
            for (int j = 0; j < kLimbs; j++) tab[st][j] = acc[j];
            if (st == kTab - 1) {
#pragma unroll
                for (int j = 0; j < kLimbs; j++) acc[j] = tab[0][j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kLimbs; j++) out[j] = acc[j];
}

__global__ __launch_bounds__(64) void rsa_half_k(const jfsx_rsa::Key *__restrict__ key, int n,
                                                 const uint8_t *__restrict__ ct, uint32_t *__restrict__ mh) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    const int half = blockIdx.y;  // 0: p, 1: q
    if (i >= n) return;
    const jfsx_rsa::Key &k = *key;
    uint32_t c[2 * kLimbs], x[kLimbs], r[kLimbs];
    jfsx_rsa::from_be(ct + (size_t)kModBytes * i, kModBytes, c, 2 * kLimbs);
    if (half == 0) {
        jfsx_rsa::reduce_2048(c, k.p, k.pinv, k.r2p, x);
        mod_exp_ct(x, k.dp, k.p, k.pinv, k.r2p, r);
    } else {
        jfsx_rsa::reduce_2048(c, k.q, k.qinv32, k.r2q, x);
        mod_exp_ct(x, k.dq, k.q, k.qinv32, k.r2q, r);
    }
    uint32_t *o = mh + ((size_t)half * n + i) * kLimbs;
#pragma unroll
    for (int j = 0; j < kLimbs; j++) o[j] = r[j];
}

__global__ __launch_bounds__(64) void rsa_finish_k(const jfsx_rsa::Key *__restrict__ key, int n,
                                                   const uint8_t *__restrict__ ct, const uint32_t *__restrict__ mh,
                                                   uint8_t *__restrict__ em_out, int32_t *__restrict__ len_out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= n) return;
    const jfsx_rsa::Key &k = *key;
    uint32_t c[2 * kLimbs], m1[kLimbs], m2[kLimbs], m[2 * kLimbs];
    jfsx_rsa::from_be(ct + (size_t)kModBytes * i, kModBytes, c, 2 * kLimbs);
    uint8_t *em = em_out + (size_t)kModBytes * i;
    if (jfsx_rsa::geq(c, k.n, 2 * kLimbs)) {  // rsa.decrypt: c >= n is a decryption error
        len_out[i] = -1;
        return;
    }
    for (int j = 0; j < kLimbs; j++) {
        m1[j] = mh[(size_t)i * kLimbs + j];
        m2[j] = mh[((size_t)n + i) * kLimbs + j];
    }
    jfsx_rsa::crt(k, m1, m2, m);
    uint8_t buf[kModBytes];
    jfsx_rsa::to_be(m, 2 * kLimbs, buf, kModBytes);
    const int len = jfsx_rsa::oaep_decode(buf, kModBytes, k.lhash);
    for (int j = 0; j < (len > 0 ? len : 0); j++) em[j] = buf[j];
    len_out[i] = len;
}

void launch_rsa_unwrap(hipStream_t s, const void *key, int n, const uint8_t *ct, uint32_t *mh, uint8_t *em,
                       int32_t *len) {
    if (n <= 0) return;
    const int g = (n + 63) / 64;
    hipLaunchKernelGGL(rsa_half_k, dim3(g, 2), dim3(64), 0, s, (const jfsx_rsa::Key *)key, n, ct, mh);
    hipLaunchKernelGGL(rsa_finish_k, dim3(g), dim3(64), 0, s, (const jfsx_rsa::Key *)key, n, ct, mh, em, len);
}

}  // namespace jfsx

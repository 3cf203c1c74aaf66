// jfsx_rsa.hip -- batched RSA-OAEP key unwrap on the GPU.
//
// rsaEncryptor.Decrypt (pkg/object/encrypt.go:124-134) runs once per object
// the reference opens (encrypt.go:207-210): an RSA-2048 private operation of
// ~0.35 ms per core, which caps end-to-end Decrypt far below the Open kernel.
// Here one batch unwraps every object key of a read window on the GPU:
//   * rsa_half_k: one thread per (object, CRT half): c mod p_h, then
//     c^d_h mod p_h by left-to-right Montgomery exponentiation (32-limb CIOS,
//     jfsx_rsa.h).  The key is wave-uniform (scalar loads); the exponent bits
//     are uniform branches.
//   * rsa_finish_k: one thread per object: c < n check, CRT recombination,
//     EME-OAEP decoding (SHA-256, MGF1, label hash), message out.
// Bit-exact to rsa.DecryptOAEP(sha256, ..., "keys"); not constant-time (the
// data-dependent OAEP checks branch) -- the batch runs on the GPU the key
// owner controls, as the host path does.
#include "jfsx_internal.h"

#define JFSX_HD __device__ __forceinline__
#include "jfsx_rsa.h"

namespace jfsx {

using jfsx_rsa::kLimbs;
using jfsx_rsa::kModBytes;

// x^e mod m, left to right with a fixed 4-bit window: x^1..x^15 (Montgomery
// domain) in private memory, then per digit four squarings and one multiply
// by the digit's power (none for a zero digit) -- about 1275 products for a
// 1024-bit exponent instead of 1535 bit by bit.  One Montgomery multiply site
// in the loop: the unrolled CIOS is ~6K instructions, and one copy keeps the
// loop inside the instruction cache.  The exponent (the key's) is wave-uniform,
// so every branch is.
#ifndef JFSX_RSA_WIN
#define JFSX_RSA_WIN 1  // 0: bit by bit (A/B)
#endif
__device__ __forceinline__ uint32_t exp_digit(const uint32_t *e, int d) { return (e[d >> 3] >> (4 * (d & 7))) & 15u; }

__device__ __forceinline__ void mod_exp_1site(const uint32_t *x, const uint32_t *e, int e_bits, const uint32_t *m,
                                              uint32_t minv, const uint32_t *r2, uint32_t *out) {
#if JFSX_RSA_WIN
    uint32_t tab[16][kLimbs];  // tab[j] = x^j R mod m, j >= 1
    uint32_t acc[kLimbs], b[kLimbs];
    jfsx_rsa::mont_mul(x, r2, m, minv, acc);  // to the Montgomery domain
#pragma unroll
    for (int j = 0; j < kLimbs; j++) tab[1][j] = acc[j];
    const int ndig = (e_bits + 3) / 4;  // the top digit holds the top set bit: nonzero
    int k = 2;                          // phase 0: tab[k] = tab[k - 1] * x
    int d = ndig - 1, phase = 0, nsq = 0;
    for (;;) {
        const uint32_t bi = phase == 0 ? 1u : phase == 2 ? exp_digit(e, d) : 0u;
        if (phase == 1) {
#pragma unroll
            for (int j = 0; j < kLimbs; j++) b[j] = acc[j];
        } else {
#pragma unroll
            for (int j = 0; j < kLimbs; j++) b[j] = tab[bi][j];
        }
        jfsx_rsa::mont_mul(acc, b, m, minv, acc);
        if (phase == 0) {
#pragma unroll
            for (int j = 0; j < kLimbs; j++) tab[k][j] = acc[j];
            if (++k < 16) continue;
            const uint32_t top = exp_digit(e, ndig - 1);
#pragma unroll
            for (int j = 0; j < kLimbs; j++) acc[j] = tab[top][j];
            if (--d < 0) break;
            phase = 1, nsq = 4;
        } else if (phase == 1) {
            if (--nsq) continue;
            if (exp_digit(e, d)) {
                phase = 2;
            } else {
                if (--d < 0) break;
                nsq = 4;
            }
        } else {
            if (--d < 0) break;
            phase = 1, nsq = 4;
        }
    }
#else
    uint32_t xm[kLimbs], acc[kLimbs], b[kLimbs];
    jfsx_rsa::mont_mul(x, r2, m, minv, xm);  // to the Montgomery domain
#pragma unroll
    for (int j = 0; j < kLimbs; j++) acc[j] = xm[j];
    int bit = e_bits - 2;
    bool mul = false;  // a multiply by x is pending for the bit just squared in
    while (bit >= 0 || mul) {
        const bool do_mul = mul;  // wave-uniform
#pragma unroll
        for (int j = 0; j < kLimbs; j++) b[j] = do_mul ? xm[j] : acc[j];
        jfsx_rsa::mont_mul(acc, b, m, minv, acc);
        if (do_mul) {
            mul = false;
        } else {
            mul = (e[bit >> 5] >> (bit & 31)) & 1u;
            bit--;
        }
    }
#endif
#pragma unroll
    for (int j = 0; j < kLimbs; j++) b[j] = j == 0;
    jfsx_rsa::mont_mul(acc, b, m, minv, out);  // out of the Montgomery domain
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
        mod_exp_1site(x, k.dp, k.dp_bits, k.p, k.pinv, k.r2p, r);
    } else {
        jfsx_rsa::reduce_2048(c, k.q, k.qinv32, k.r2q, x);
        mod_exp_1site(x, k.dq, k.dq_bits, k.q, k.qinv32, k.r2q, r);
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

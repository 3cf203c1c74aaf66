// jfsx_rsa.hip -- batched RSA-OAEP key unwrap on the GPU.
//
// rsaEncryptor.Decrypt (pkg/object/encrypt.go:124-134) runs once per object
// the reference opens (encrypt.go:207-210): an RSA-2048 private operation of
// ~0.35 ms per core, which caps end-to-end Decrypt far below the Open kernel.
// Here one batch unwraps every object key of a read window on the GPU:
//   * rsa_pair_k: two lanes per (object, CRT half): c mod p_h, then
//     c^d_h mod p_h by a fixed-window Montgomery exponentiation in 28-bit
//     limbs with lazy carries, each product split by columns over the lane
//     pair with DPP exchanges (jfsx_rsa.h: mod_exp28_pair), constant time in
//     the exponent.  rsa_half_k (JFSX_RSA_PAIR=0) is the one-lane form
//     (mod_exp28): half the waves, each issuing the whole product.
//   * rsa_finish_k: one thread per object: c < n check, CRT recombination,
//     EME-OAEP decoding (SHA-256, MGF1, label hash), message out.
// Bit-exact to rsa.DecryptOAEP(sha256, ..., "keys") and, like it, constant
// time with respect to the private key and the decrypted data (jfsx_rsa.h):
// no branch and no memory address depends on the exponent, the CRT values or
// the OAEP checks; the one branch on secret-derived data is the final valid /
// invalid outcome, which Go's decryptOAEP also returns as an error.
#include <stdlib.h>
#include <string.h>

#include "jfsx_internal.h"

#define JFSX_HD __device__ __forceinline__
#define JFSX_RSA_OPAQUE(x) asm volatile("" : "+v"(x))
#include "jfsx_rsa.h"

namespace jfsx {

using jfsx_rsa::kLimbs;
using jfsx_rsa::kModBytes;

// threads per workgroup of rsa_half_k
#ifndef JFSX_RSA_LANES
#define JFSX_RSA_LANES 64
#endif
constexpr int kRsaLanes = JFSX_RSA_LANES;

__global__ __launch_bounds__(kRsaLanes) void rsa_half_k(const jfsx_rsa::Key *__restrict__ key, int n,
                                                        const uint8_t *__restrict__ ct, uint32_t *__restrict__ mh) {
    const int i = blockIdx.x * kRsaLanes + threadIdx.x;
    const int half = blockIdx.y;  // 0: p, 1: q
    if (i >= n) return;
    const jfsx_rsa::Key &k = *key;
    uint32_t c[2 * kLimbs], x[kLimbs], r[kLimbs];
    jfsx_rsa::from_be(ct + (size_t)kModBytes * i, kModBytes, c, 2 * kLimbs);
    if (half == 0) {
        jfsx_rsa::reduce_2048(c, k.p, k.pinv, k.r2p, x);
        jfsx_rsa::mod_exp28(x, k.dp, k.p, k.pinv, k.r2p28, r);
    } else {
        jfsx_rsa::reduce_2048(c, k.q, k.qinv32, k.r2q, x);
        jfsx_rsa::mod_exp28(x, k.dq, k.q, k.qinv32, k.r2q28, r);
    }
    uint32_t *o = mh + ((size_t)half * n + i) * kLimbs;
#pragma unroll
    for (int j = 0; j < kLimbs; j++) o[j] = r[j];
}

// the lane exchange of mod_exp28_pair: the pair is lanes (2k, 2k+1); DPP
// quad_perm moves (0,0,2,2) / (1,1,3,3) / (1,0,3,2)
struct PairDpp {
    uint32_t hi;
    __device__ __forceinline__ static constexpr bool tracing() { return false; }
    __device__ __forceinline__ uint32_t lo(uint32_t v) const {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xA0, 0xF, 0xF, true);
    }
    __device__ __forceinline__ uint32_t up(uint32_t v) const {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xF5, 0xF, 0xF, true);
    }
    __device__ __forceinline__ uint32_t other(uint32_t v) const {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
    }
};

// threads 2i, 2i+1 of the grid: object i; blockIdx.y: the CRT half.  Pairs
// never straddle a bound: both lanes of a pair see the same i.
__global__ __launch_bounds__(64) void rsa_pair_k(const jfsx_rsa::Key *__restrict__ key, int n,
                                                 const uint8_t *__restrict__ ct, uint32_t *__restrict__ mh) {
    const int t = blockIdx.x * 64 + threadIdx.x, i = t >> 1;
    const int half = blockIdx.y;
    if (i >= n) return;
    const PairDpp x{(uint32_t)(t & 1)};
    const jfsx_rsa::Key &k = *key;
    uint32_t c[2 * kLimbs], v[kLimbs], r[kLimbs];
    jfsx_rsa::from_be(ct + (size_t)kModBytes * i, kModBytes, c, 2 * kLimbs);
    if (half == 0) {
        jfsx_rsa::reduce_2048(c, k.p, k.pinv, k.r2p, v);
        jfsx_rsa::mod_exp28_pair(x, v, k.dp, k.p, k.pinv, k.r2p28, r);
    } else {
        jfsx_rsa::reduce_2048(c, k.q, k.qinv32, k.r2q, v);
        jfsx_rsa::mod_exp28_pair(x, v, k.dq, k.q, k.qinv32, k.r2q28, r);
    }
    // each lane stores half of the result
    uint32_t *o = mh + ((size_t)half * n + i) * kLimbs + (t & 1) * (kLimbs / 2);
#pragma unroll
    for (int j = 0; j < kLimbs / 2; j++) o[j] = (t & 1) ? r[kLimbs / 2 + j] : r[j];
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
    static const bool pair = [] {  // JFSX_RSA_PAIR=0: the one-lane kernel (A/B)
        const char *e = getenv("JFSX_RSA_PAIR");
        return !(e && !strcmp(e, "0"));
    }();
    const int g = (n + 63) / 64, gh = (n + kRsaLanes - 1) / kRsaLanes;
    if (pair)
        hipLaunchKernelGGL(rsa_pair_k, dim3((2 * n + 63) / 64, 2), dim3(64), 0, s, (const jfsx_rsa::Key *)key, n, ct,
                           mh);
    else
        hipLaunchKernelGGL(rsa_half_k, dim3(gh, 2), dim3(kRsaLanes), 0, s, (const jfsx_rsa::Key *)key, n, ct, mh);
    hipLaunchKernelGGL(rsa_finish_k, dim3(g), dim3(64), 0, s, (const jfsx_rsa::Key *)key, n, ct, mh, em, len);
}

}  // namespace jfsx

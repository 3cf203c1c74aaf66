// jfsx_gf.h -- GF(2^128) product for GHASH from integer multiplies, for a
// per-lane x and a per-lane y (no table, no LDS, no barrier).
//
// The kernels' g128 keeps GCM's reflected bit order (w[0] bit 31 is the
// coefficient of x^0, w[3] bit 0 that of x^127; SP 800-38D 6.3).  Reversing
// the bits of each word gives the plain order (word k bit b = coefficient
// 32k + b), in which the product is an ordinary carry-less product followed by
// a reduction modulo x^128 + x^7 + x^2 + x + 1.
//
// Carry-less 32 x 32 -> 64 products come from integer multiplies of operands
// split into four masks of every fourth bit (x & 0x11111111, ...): a bit of
// the integer product collects at most 8 partial products, so its carries stay
// below the next bit of the same residue mod 4, and masking the sums keeps
// exactly the carry-less bits (the "holes" technique of constant-time GHASH
// implementations, e.g. BearSSL's ghash_ctmul).  Karatsuba turns the 128 x 128
// product into 9 such 32 x 32 products: 144 multiplies (v_mad_u64_u32 on the
// GPU), about 500 instructions, against 128 dependent shift-and-add steps
// (about 2000) of the bit-serial product.  No data-dependent branch or index.
//
// Host/device portable: the includer defines JFSX_GF_HD (the GPU build:
// __device__ __forceinline__); tests/harness/gf_host.cpp checks it against
// the bit-serial product of SP 800-38D Algorithm 1 on the host.
#pragma once
#include <stdint.h>

#ifndef JFSX_GF_HD
#define JFSX_GF_HD static inline
#endif
// scheduling-region breaks between the carry-less sub-products (GPU build):
// the ROCm 7.2 iterative-ILP scheduler, which the GCM kernels use, crashes on
// the whole product as one region
#ifndef JFSX_GF_BREAK
#define JFSX_GF_BREAK() ((void)0)
#endif

namespace jfsx_gf {

// bit reversal of a word (v_bfrev_b32 on the GPU)
JFSX_GF_HD uint32_t rev32(uint32_t v) {
#if defined(__has_builtin) && __has_builtin(__builtin_bitreverse32)
    return __builtin_bitreverse32(v);
#else
    v = ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
    v = ((v >> 2) & 0x33333333u) | ((v & 0x33333333u) << 2);
    v = ((v >> 4) & 0x0F0F0F0Fu) | ((v & 0x0F0F0F0Fu) << 4);
    return __builtin_bswap32(v);
#endif
}

// carry-less 32 x 32 -> 64
JFSX_GF_HD uint64_t clmul32(uint32_t x, uint32_t y) {
    const uint32_t x0 = x & 0x11111111u, x1 = x & 0x22222222u, x2 = x & 0x44444444u, x3 = x & 0x88888888u;
    const uint32_t y0 = y & 0x11111111u, y1 = y & 0x22222222u, y2 = y & 0x44444444u, y3 = y & 0x88888888u;
    const uint64_t z0 = ((uint64_t)x0 * y0) ^ ((uint64_t)x1 * y3) ^ ((uint64_t)x2 * y2) ^ ((uint64_t)x3 * y1);
    const uint64_t z1 = ((uint64_t)x0 * y1) ^ ((uint64_t)x1 * y0) ^ ((uint64_t)x2 * y3) ^ ((uint64_t)x3 * y2);
    JFSX_GF_BREAK();
    const uint64_t z2 = ((uint64_t)x0 * y2) ^ ((uint64_t)x1 * y1) ^ ((uint64_t)x2 * y0) ^ ((uint64_t)x3 * y3);
    const uint64_t z3 = ((uint64_t)x0 * y3) ^ ((uint64_t)x1 * y2) ^ ((uint64_t)x2 * y1) ^ ((uint64_t)x3 * y0);
    return (z0 & 0x1111111111111111ull) | (z1 & 0x2222222222222222ull) | (z2 & 0x4444444444444444ull) |
           (z3 & 0x8888888888888888ull);
}

// carry-less 64 x 64 -> 128 (lo, hi) by Karatsuba over 32-bit halves
JFSX_GF_HD void clmul64(uint64_t a, uint64_t b, uint64_t &lo, uint64_t &hi) {
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32);
    const uint64_t p0 = clmul32(a0, b0);
    JFSX_GF_BREAK();
    const uint64_t p2 = clmul32(a1, b1);
    JFSX_GF_BREAK();
    const uint64_t p1 = clmul32(a0 ^ a1, b0 ^ b1) ^ p0 ^ p2;
    JFSX_GF_BREAK();
    lo = p0 ^ (p1 << 32);
    hi = p2 ^ (p1 >> 32);
}

// z = x y in GCM's bit order; x, y, z as four words w[0..3] (reflected)
JFSX_GF_HD void mul(const uint32_t x[4], const uint32_t y[4], uint32_t z[4]) {
    // plain order, 64-bit halves: A = a1 x^64 + a0
    const uint64_t a0 = (uint64_t)rev32(x[0]) | (uint64_t)rev32(x[1]) << 32;
    const uint64_t a1 = (uint64_t)rev32(x[2]) | (uint64_t)rev32(x[3]) << 32;
    const uint64_t b0 = (uint64_t)rev32(y[0]) | (uint64_t)rev32(y[1]) << 32;
    const uint64_t b1 = (uint64_t)rev32(y[2]) | (uint64_t)rev32(y[3]) << 32;
    uint64_t l0, h0, l1, h1, lm, hm;
    clmul64(a0, b0, l0, h0);
    clmul64(a1, b1, l1, h1);
    clmul64(a0 ^ a1, b0 ^ b1, lm, hm);
    JFSX_GF_BREAK();
    lm ^= l0 ^ l1;
    hm ^= h0 ^ h1;
    // 256-bit product r3 r2 r1 r0 (64-bit words, r0 lowest)
    const uint64_t r0 = l0, r1 = h0 ^ lm, r2 = l1 ^ hm, r3 = h1;
    // reduce: (r3 r2) x^128 = (r3 r2)(x^7 + x^2 + x + 1); the bits shifted
    // past x^127 by << 7 / << 2 / << 1 (at most 7) fold once more
    const uint64_t f2 = r2 ^ (r2 << 1) ^ (r2 << 2) ^ (r2 << 7);
    const uint64_t f3 = r3 ^ (r3 << 1) ^ (r3 << 2) ^ (r3 << 7) ^ (r2 >> 63) ^ (r2 >> 62) ^ (r2 >> 57);
    const uint64_t o = (r3 >> 63) ^ (r3 >> 62) ^ (r3 >> 57);  // coefficients 128.. of (r3 r2)(x^7 + x^2 + x)
    const uint64_t c0 = r0 ^ f2 ^ o ^ (o << 1) ^ (o << 2) ^ (o << 7), c1 = r1 ^ f3;
    z[0] = rev32((uint32_t)c0);
    z[1] = rev32((uint32_t)(c0 >> 32));
    z[2] = rev32((uint32_t)c1);
    z[3] = rev32((uint32_t)(c1 >> 32));
}

}  // namespace jfsx_gf

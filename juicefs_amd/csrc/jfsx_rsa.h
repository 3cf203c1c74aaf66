// jfsx_rsa.h -- RSA-OAEP (SHA-256) private-key decryption arithmetic for the
// batched key unwrap.
//
// Replaces, per object, rsaEncryptor.Decrypt = rsa.DecryptOAEP(sha256.New(),
// rand, privKey, wrapped, []byte("keys")) (pkg/object/encrypt.go:124-134,
// :207-210), which the reference runs on the host for every block it opens.
// The arithmetic is RSA with the CRT (RFC 8017 5.1.2 / Go's precomputed
// Dp, Dq, Qinv): m1 = c^dp mod p, m2 = c^dq mod q, h = qinv (m1 - m2) mod p,
// m = m2 + h q; then EME-OAEP decoding (RFC 8017 7.1.2) with SHA-256 as hash
// and MGF1 hash.  Primes are 1024-bit (RSA-2048, the size the reference docs
// use), in 32 little-endian 32-bit limbs; products use Montgomery CIOS.
//
// Host/device portable: the includer defines JFSX_HD.  Every function is
// pinned on the CPU by tests/test_rsa.py against libcrypto's RSA-OAEP.
//
// Constant time with respect to the private key and the decrypted message,
// as Go's rsa.DecryptOAEP is (crypto/internal/bigmod, subtle.ConstantTime*):
// the exponentiation (mod_exp28) runs a fixed 3-bit window over the full
// 1024-bit exponent length, always multiplies (digit 0 multiplies by the
// Montgomery one), and reads its window table by a masked scan of all 8 rows; the
// modular corrections, the CRT recombination and the OAEP checks select with
// masks instead of branching.  Branches remain only on public values: the
// ciphertext length and c >= n (Go rejects both before the private
// operation), and the final valid / invalid outcome.
#pragma once
#include <stdint.h>

// test hook: the host harness records every Montgomery product and every
// window-table read to check that the sequence does not depend on the exponent
#ifndef JFSX_RSA_TRACE
#define JFSX_RSA_TRACE(tag, v) ((void)0)
#endif
// a register barrier: the compiler cannot see through it, so a mask built from
// a secret digit cannot become a branch or an address (the GPU includer passes
// its VGPR form)
#ifndef JFSX_RSA_OPAQUE
#define JFSX_RSA_OPAQUE(x) asm volatile("" : "+r"(x))
#endif

namespace jfsx_rsa {

constexpr int kLimbs = 32;        // 1024-bit prime
constexpr int kL28 = 37;          // the same in 28-bit limbs (1036 bits), the GPU exponentiation's form
constexpr int kModBytes = 256;    // RSA-2048 modulus
constexpr int kHash = 32;         // SHA-256

// ---------------------------------------------------------------------------
// multi-precision helpers (little-endian limbs)
// ---------------------------------------------------------------------------
// -m^-1 mod 2^32 (m odd), Newton iteration
JFSX_HD uint32_t mont_inv32(uint32_t m0) {
    uint32_t x = m0;  // correct to 3 bits
    for (int i = 0; i < 5; i++) x *= 2u - m0 * x;
    return 0u - x;
}

// a >= b ?
JFSX_HD bool geq(const uint32_t *a, const uint32_t *b, int n) {
    for (int i = n - 1; i >= 0; i--)
        if (a[i] != b[i]) return a[i] > b[i];
    return true;
}

// a -= b, returns borrow
JFSX_HD uint32_t sub_in(uint32_t *a, const uint32_t *b, int n) {
    uint64_t br = 0;
    for (int i = 0; i < n; i++) {
        const uint64_t d = (uint64_t)a[i] - b[i] - br;
        a[i] = (uint32_t)d;
        br = (d >> 32) & 1u;
    }
    return (uint32_t)br;
}

// a += b, returns carry
JFSX_HD uint32_t add_in(uint32_t *a, const uint32_t *b, int n) {
    uint64_t c = 0;
    for (int i = 0; i < n; i++) {
        c += (uint64_t)a[i] + b[i];
        a[i] = (uint32_t)c;
        c >>= 32;
    }
    return (uint32_t)c;
}

// all-ones if x != 0, else 0 (no branch)
JFSX_HD uint32_t ct_nz(uint32_t x) { return 0u - ((x | (0u - x)) >> 31); }

// a >= b as an all-ones / zero mask, over all n limbs (no early exit)
JFSX_HD uint32_t ct_geq(const uint32_t *a, const uint32_t *b, int n) {
    uint64_t br = 0;
    for (int i = 0; i < n; i++) br = (((uint64_t)a[i] - b[i] - br) >> 32) & 1u;
    return (uint32_t)br - 1u;  // no borrow: a >= b
}

// a = mask ? a - b : a, over n limbs; returns the borrow of a - b
JFSX_HD uint32_t ct_sub_if(uint32_t *a, const uint32_t *b, int n, uint32_t mask) {
    uint64_t br = 0;
    for (int i = 0; i < n; i++) {
        const uint64_t d = (uint64_t)a[i] - b[i] - br;
        br = (d >> 32) & 1u;
        a[i] = (a[i] & ~mask) | ((uint32_t)d & mask);
    }
    return (uint32_t)br;
}

// a += mask & b over n limbs
JFSX_HD void ct_add_if(uint32_t *a, const uint32_t *b, int n, uint32_t mask) {
    uint64_t c = 0;
    for (int i = 0; i < n; i++) {
        c += (uint64_t)a[i] + (b[i] & mask);
        a[i] = (uint32_t)c;
        c >>= 32;
    }
}

// out = a b R^-1 mod m (R = 2^1024), a, b < m; CIOS with one final subtract
JFSX_HD void mont_mul(const uint32_t *a, const uint32_t *b, const uint32_t *m, uint32_t minv, uint32_t *out) {
    JFSX_RSA_TRACE('M', 0);
    uint32_t t[kLimbs + 2];
#pragma unroll
    for (int j = 0; j < kLimbs + 2; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < kLimbs; i++) {
        const uint32_t ai = a[i];
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < kLimbs; j++) {
            c = (uint64_t)ai * b[j] + (c + t[j]);
            t[j] = (uint32_t)c;
            c >>= 32;
        }
        c += t[kLimbs];
        t[kLimbs] = (uint32_t)c;
        t[kLimbs + 1] = (uint32_t)(c >> 32);
        const uint32_t mi = t[0] * minv;
        c = ((uint64_t)mi * m[0] + t[0]) >> 32;
#pragma unroll
        for (int j = 1; j < kLimbs; j++) {
            c = (uint64_t)mi * m[j] + (c + t[j]);
            t[j - 1] = (uint32_t)c;
            c >>= 32;
        }
        c += t[kLimbs];
        t[kLimbs - 1] = (uint32_t)c;
        t[kLimbs] = t[kLimbs + 1] + (uint32_t)(c >> 32);
    }
    // t < 2m: subtract m once if t >= m
    uint32_t d[kLimbs];
    uint64_t br = 0;
#pragma unroll
    for (int j = 0; j < kLimbs; j++) {
        const uint64_t x = (uint64_t)t[j] - m[j] - br;
        d[j] = (uint32_t)x;
        br = (x >> 32) & 1u;
    }
    const bool keep = t[kLimbs] == 0 && br;  // t < m
#pragma unroll
    for (int j = 0; j < kLimbs; j++) out[j] = keep ? t[j] : d[j];
}

// 2^bits mod m by doubling (host side, once per key); R^2 mod m by default
JFSX_HD void mont_r2(const uint32_t *m, uint32_t *r2, int bits = 2 * 32 * kLimbs) {
    uint32_t x[kLimbs + 1];
    for (int j = 0; j <= kLimbs; j++) x[j] = 0;
    x[0] = 1;
    for (int k = 0; k < bits; k++) {  // x = 2^k mod m
        uint32_t c = 0;
        for (int j = 0; j <= kLimbs; j++) {
            const uint32_t nc = x[j] >> 31;
            x[j] = (x[j] << 1) | c;
            c = nc;
        }
        if (x[kLimbs] || geq(x, m, kLimbs)) {
            const uint32_t b = sub_in(x, m, kLimbs);
            x[kLimbs] -= b;
        }
    }
    for (int j = 0; j < kLimbs; j++) r2[j] = x[j];
}

// big-endian bytes <-> limbs
JFSX_HD void from_be(const uint8_t *b, int nbytes, uint32_t *x, int nlimbs) {
    for (int j = 0; j < nlimbs; j++) x[j] = 0;
    for (int i = 0; i < nbytes; i++) {
        const int bit = 8 * (nbytes - 1 - i);
        x[bit >> 5] |= (uint32_t)b[i] << (bit & 31);
    }
}
JFSX_HD void to_be(const uint32_t *x, int nlimbs, uint8_t *b, int nbytes) {
    for (int i = 0; i < nbytes; i++) {
        const int bit = 8 * (nbytes - 1 - i);
        b[i] = (bit >> 5) < nlimbs ? (uint8_t)(x[bit >> 5] >> (bit & 31)) : 0;
    }
}

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4) and MGF1
// ---------------------------------------------------------------------------
JFSX_HD uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

JFSX_HD void sha256_block(uint32_t h[8], const uint8_t *p) {
    const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5, 0xd807aa98,
        0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786,
        0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8,
        0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13,
        0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819,
        0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a,
        0x5b9cca4f, 0x682e6ff3, 0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
        const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
        const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// SHA-256 of a ‖ b (b may be empty), len(a) + len(b) < 2^29
JFSX_HD void sha256_2(const uint8_t *a, int la, const uint8_t *b, int lb, uint8_t out[32]) {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t blk[64];
    const int total = la + lb;
    int pos = 0, fill = 0;
    // stream the message bytes, then 0x80, zeros, BE64 bit length
    const int padded = ((total + 9 + 63) / 64) * 64;
    for (int i = 0; i < padded; i++) {
        uint8_t v;
        if (i < la) v = a[i];
        else if (i < total) v = b[i - la];
        else if (i == total) v = 0x80;
        else if (i >= padded - 8) v = (uint8_t)(((uint64_t)total * 8) >> (8 * (padded - 1 - i)));
        else v = 0;
        blk[fill++] = v;
        if (fill == 64) {
            sha256_block(h, blk);
            fill = 0;
        }
        pos++;
    }
    (void)pos;
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

// dst[0..len) ^= MGF1-SHA256(seed, len)
JFSX_HD void mgf1_xor(const uint8_t *seed, int slen, uint8_t *dst, int len) {
    uint8_t ctr[4], hsh[32];
    for (int c = 0, done = 0; done < len; c++) {
        ctr[0] = (uint8_t)(c >> 24); ctr[1] = (uint8_t)(c >> 16); ctr[2] = (uint8_t)(c >> 8); ctr[3] = (uint8_t)c;
        sha256_2(seed, slen, ctr, 4, hsh);
        for (int i = 0; i < 32 && done < len; i++, done++) dst[done] ^= hsh[i];
    }
}

// EME-OAEP decode (RFC 8017 7.1.2 step 3) of em[0..k), lhash = SHA-256(label).
// Returns the message length and moves the message to em[0..len), or -1
// ("crypto/rsa: decryption error").  As Go's decryptOAEP: the leading zero
// byte, the label hash and the 0x01 separator are checked without branching
// on the data (the separator by a masked scan of the whole of DB), and one
// combined valid / invalid outcome is branched on at the end.
JFSX_HD int oaep_decode(uint8_t *em, int k, const uint8_t lhash[32]) {
    uint8_t *seed = em + 1, *db = em + 1 + kHash;
    const int dblen = k - kHash - 1;
    mgf1_xor(db, dblen, seed, kHash);
    mgf1_xor(seed, kHash, db, dblen);
    uint32_t bad = ct_nz(em[0]);
    for (int i = 0; i < kHash; i++) bad |= ct_nz((uint32_t)(db[i] ^ lhash[i]));
    uint32_t looking = ~0u, index = 0, invalid = 0;
    for (int i = kHash; i < dblen; i++) {
        const uint32_t is0 = ~ct_nz(db[i]), is1 = ~ct_nz((uint32_t)db[i] ^ 1u);
        index = (index & ~(looking & is1)) | ((uint32_t)i & looking & is1);
        invalid |= looking & ~is0 & ~is1;
        looking &= ~is1;
    }
    if (bad | invalid | looking) return -1;
    const int mlen = dblen - (int)index - 1;
    for (int j = 0; j < mlen; j++) em[j] = db[index + 1 + j];
    return mlen;
}

// ---------------------------------------------------------------------------
// key material in device memory (written by the host once per key)
// ---------------------------------------------------------------------------
struct Key {
    uint32_t n[2 * kLimbs];             // modulus p q (ciphertexts must be < n)
    uint32_t p[kLimbs], q[kLimbs];      // primes
    uint32_t dp[kLimbs], dq[kLimbs];    // CRT exponents
    uint32_t qinv[kLimbs];              // q^-1 mod p
    uint32_t r2p[kLimbs], r2q[kLimbs];  // R^2 mod p, R^2 mod q
    uint32_t r2p28[kLimbs], r2q28[kLimbs];  // R'^2 mod p, q for the GPU's 28-bit limbs (R' = 2^(28 kL28))
    uint32_t pinv, qinv32;              // -p^-1, -q^-1 mod 2^32
    int32_t dp_bits, dq_bits;           // exponent bit lengths
    uint8_t lhash[32];                  // SHA-256(label)
};

JFSX_HD int bit_length(const uint32_t *x, int nlimbs) {
    for (int i = nlimbs - 1; i >= 0; i--)
        if (x[i]) return 32 * i + 32 - __builtin_clz(x[i]);
    return 0;
}

// Key from the CRT components (big-endian, 128 bytes each) and the OAEP
// label.  Returns false unless p, q are odd 1024-bit primes' shape.
JFSX_HD bool key_setup(Key &k, const uint8_t *p, const uint8_t *q, const uint8_t *dp, const uint8_t *dq,
                       const uint8_t *qinv, const uint8_t *label, int label_len) {
    const int nb = 4 * kLimbs;
    from_be(p, nb, k.p, kLimbs);
    from_be(q, nb, k.q, kLimbs);
    from_be(dp, nb, k.dp, kLimbs);
    from_be(dq, nb, k.dq, kLimbs);
    from_be(qinv, nb, k.qinv, kLimbs);
    if (!(k.p[0] & 1u) || !(k.q[0] & 1u) || bit_length(k.p, kLimbs) != 32 * kLimbs ||
        bit_length(k.q, kLimbs) != 32 * kLimbs)
        return false;
    k.pinv = mont_inv32(k.p[0]);
    k.qinv32 = mont_inv32(k.q[0]);
    mont_r2(k.p, k.r2p);
    mont_r2(k.q, k.r2q);
    mont_r2(k.p, k.r2p28, 2 * 28 * kL28);
    mont_r2(k.q, k.r2q28, 2 * 28 * kL28);
    k.dp_bits = bit_length(k.dp, kLimbs);
    k.dq_bits = bit_length(k.dq, kLimbs);
    if (k.dp_bits < 2 || k.dq_bits < 2) return false;
    for (int j = 0; j < 2 * kLimbs; j++) k.n[j] = 0;
    for (int i = 0; i < kLimbs; i++) {
        uint64_t c = 0;
        for (int j = 0; j < kLimbs; j++) {
            c = (uint64_t)k.p[i] * k.q[j] + (c + k.n[i + j]);
            k.n[i + j] = (uint32_t)c;
            c >>= 32;
        }
        k.n[i + kLimbs] = (uint32_t)c;
    }
    sha256_2(label, label_len, label, 0, k.lhash);
    return true;
}

// c mod m for a 2048-bit c = hi R + lo (hi, lo < R): (hi R mod m) + lo, reduced
JFSX_HD void reduce_2048(const uint32_t *c, const uint32_t *m, uint32_t minv, const uint32_t *r2, uint32_t *out) {
    uint32_t t[kLimbs + 1];
    mont_mul(c + kLimbs, r2, m, minv, t);  // hi R mod m (hi < R, r2 < m: CIOS bound holds)
    t[kLimbs] = add_in(t, c, kLimbs);      // + lo: < 3m since lo < R < 2m
    for (int rep = 0; rep < 2; rep++) {     // two masked corrections, always both
        const uint32_t ge = ct_nz(t[kLimbs]) | ct_geq(t, m, kLimbs);
        t[kLimbs] -= ct_sub_if(t, m, kLimbs, ge) & ge;
    }
    for (int j = 0; j < kLimbs; j++) out[j] = t[j];
}

// m = m2 + q (qinv (m1 - m2) mod p), the 2048-bit CRT recombination
JFSX_HD void crt(const Key &k, const uint32_t *m1, const uint32_t *m2, uint32_t *m) {
    uint32_t t[kLimbs + 1], h[kLimbs], u[kLimbs];
    for (int j = 0; j < kLimbs; j++) t[j] = m2[j];
    t[kLimbs] = 0;
    ct_sub_if(t, k.p, kLimbs, ct_geq(t, k.p, kLimbs));  // m2 < q < 2p
    for (int j = 0; j < kLimbs; j++) u[j] = m1[j];
    const uint32_t neg = 0u - sub_in(u, t, kLimbs);     // (m1 - m2) mod p
    ct_add_if(u, k.p, kLimbs, neg);
    mont_mul(u, k.qinv, k.p, k.pinv, h);               // u qinv R^-1
    mont_mul(h, k.r2p, k.p, k.pinv, h);                // u qinv
    for (int j = 0; j < 2 * kLimbs; j++) m[j] = j < kLimbs ? m2[j] : 0;
    for (int i = 0; i < kLimbs; i++) {  // m += h q, carries run to the top every time
        uint64_t c = 0;
        for (int j = 0; j < kLimbs; j++) {
            c = (uint64_t)h[i] * k.q[j] + (c + m[i + j]);
            m[i + j] = (uint32_t)c;
            c >>= 32;
        }
        for (int j = i + kLimbs; j < 2 * kLimbs; j++) {
            c += m[j];
            m[j] = (uint32_t)c;
            c >>= 32;
        }
    }
}

// ---------------------------------------------------------------------------
// The exponentiation the unwrap runs, in 28-bit limbs.  With 32-bit limbs every
// multiply-add of the CIOS carries into the next (a GPU thread spends ~9K
// instructions per product on the multiply-adds and the moves that build
// their 64-bit addends).  With 37 limbs of 28 bits a product is < 2^56, so
// each column's 64-bit accumulator takes every row's two products with no
// carry at all (37 rows x 2 x 2^56 < 2^63): a row is 74 independent
// multiply-adds, and carries are resolved once per product.  R' = 2^(28 kL28);
// R'^2 mod p, q come with the key (Key::r2p28, r2q28).
// ---------------------------------------------------------------------------
constexpr uint32_t kM28 = (1u << 28) - 1;

// 32-bit limbs (kLimbs) <-> 28-bit limbs (kL28)
JFSX_HD void to28(const uint32_t *x, uint32_t *y) {
#pragma unroll
    for (int j = 0; j < kL28; j++) {
        const int bit = 28 * j, l = bit >> 5, o = bit & 31;
        uint64_t v = x[l];
        if (l + 1 < kLimbs) v |= (uint64_t)x[l + 1] << 32;
        y[j] = (uint32_t)(v >> o) & kM28;
    }
}
JFSX_HD void from28(const uint32_t *y, uint32_t *x) {
#pragma unroll
    for (int j = 0; j < kLimbs; j++) {
        const int bit = 32 * j, l = bit / 28, o = bit % 28;  // o <= 24: two limbs cover the word
        uint64_t v = (uint64_t)y[l] >> o;
        if (l + 1 < kL28) v |= (uint64_t)y[l + 1] << (28 - o);
        x[j] = (uint32_t)v;
    }
}

// out = a b R'^-1 mod m: a, b < m in normalized 28-bit limbs, minv = -m^-1
// mod 2^28; out normalized and < m (one masked final subtract)
JFSX_HD void mont_mul28(const uint32_t *a, const uint32_t *b, const uint32_t *m, uint32_t minv, uint32_t *out) {
    JFSX_RSA_TRACE('M', 1);
    uint64_t acc[kL28];
#pragma unroll
    for (int j = 0; j < kL28; j++) acc[j] = 0;
#pragma unroll
    for (int i = 0; i < kL28; i++) {
        const uint32_t ai = a[i];
#pragma unroll
        for (int j = 0; j < kL28; j++) acc[j] += (uint64_t)ai * b[j];
        const uint32_t mi = ((uint32_t)acc[0] * minv) & kM28;
#pragma unroll
        for (int j = 0; j < kL28; j++) acc[j] += (uint64_t)mi * m[j];
        const uint64_t c = acc[0] >> 28;  // acc[0] is now a multiple of 2^28
#pragma unroll
        for (int j = 0; j < kL28 - 1; j++) acc[j] = acc[j + 1];
        acc[kL28 - 1] = 0;
        acc[0] += c;
    }
    // normalize (the value is < 2m < 2^1036), then subtract m unless t < m
    uint32_t t[kL28], d[kL28];
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < kL28; j++) {
        c += acc[j];
        t[j] = (uint32_t)c & kM28;
        c >>= 28;
    }
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < kL28; j++) {
        const uint32_t x = t[j] - m[j] - br;
        d[j] = x & kM28;
        br = x >> 31;
    }
    const uint32_t keep = 0u - br;  // t < m
#pragma unroll
    for (int j = 0; j < kL28; j++) out[j] = (t[j] & keep) | (d[j] & ~keep);
}

// The constant-time fixed-window schedule: kWDigits kWBits-bit digits of the
// exponent zero-extended to the prime's length, top first; per digit kWBits
// squarings and one multiply by tab[digit] (tab[0] = the Montgomery one),
// whatever the digit, the entry picked by a masked scan of all kWTab entries.
// One Montgomery multiply site in a loop over a step counter (the unrolled
// product is a few thousand instructions; one copy stays in the GPU's
// instruction cache), table writes at static indices only (so the table can
// live in registers), and the exponent only feeding masks through a register
// barrier.  A 3-bit window: the 8-entry table of 37-limb values fits the GPU
// thread's registers, a 16-entry one spills to scratch memory and the scan
// then reads it for every digit.
constexpr int kWBits = 3, kWTab = 1 << kWBits, kWDigits = (32 * kLimbs + kWBits - 1) / kWBits;

// digit d (0 = least significant) of e in kWBits-bit digits
JFSX_HD uint32_t w_digit(const uint32_t *e, int d) {
    const int b = kWBits * d, l = b >> 5, o = b & 31;
    uint64_t v = e[l];
    if (l + 1 < kLimbs) v |= (uint64_t)e[l + 1] << 32;
    return (uint32_t)(v >> o) & (kWTab - 1);
}

// x^e mod m (x < m; 32-bit limbs in and out), constant time in e
JFSX_HD void mod_exp28(const uint32_t *x32, const uint32_t *e, const uint32_t *m32, uint32_t minv32,
                       const uint32_t *r2_32, uint32_t *out32) {
    uint32_t m[kL28], x[kL28], r2[kL28];
    to28(m32, m);
    to28(x32, x);
    to28(r2_32, r2);
    const uint32_t minv = minv32 & kM28;
    uint32_t tab[kWTab][kL28];
    uint32_t acc[kL28], b[kL28];
    for (int w = 0; w < kWTab; w++)
        for (int j = 0; j < kL28; j++) tab[w][j] = 0;
    constexpr int kPer = kWBits + 1, kMain = kWTab + kPer * kWDigits;  // steps: table, digits, leave the domain
#pragma unroll 1
    for (int st = 0; st <= kMain; st++) {
        if (st == 0) {  // R' mod m = r2 * 1
#pragma unroll
            for (int j = 0; j < kL28; j++) acc[j] = r2[j], b[j] = j == 0;
        } else if (st == 1) {  // x R' mod m
#pragma unroll
            for (int j = 0; j < kL28; j++) acc[j] = x[j], b[j] = r2[j];
        } else if (st < kWTab) {  // tab[st] = tab[st - 1] * x R'
#pragma unroll
            for (int j = 0; j < kL28; j++) b[j] = tab[1][j];
        } else if (st < kMain) {
            const int r = st - kWTab;
            if (r % kPer < kWBits) {
#pragma unroll
                for (int j = 0; j < kL28; j++) b[j] = acc[j];
            } else {
                uint32_t idx = w_digit(e, kWDigits - 1 - r / kPer);
                JFSX_RSA_OPAQUE(idx);
#pragma unroll
                for (int j = 0; j < kL28; j++) b[j] = 0;
#pragma unroll
                for (uint32_t w = 0; w < (uint32_t)kWTab; w++) {
                    uint32_t msk = ~ct_nz(w ^ idx);
                    JFSX_RSA_OPAQUE(msk);
                    JFSX_RSA_TRACE('S', w);
#pragma unroll
                    for (int j = 0; j < kL28; j++) b[j] |= tab[w][j] & msk;
                }
            }
        } else {  // out of the Montgomery domain
#pragma unroll
            for (int j = 0; j < kL28; j++) b[j] = j == 0;
        }
        mont_mul28(acc, b, m, minv, acc);
        if (st < kWTab) {
#pragma unroll
            for (int w = 0; w < kWTab; w++)
#pragma unroll
                for (int j = 0; j < kL28; j++) tab[w][j] = st == w ? acc[j] : tab[w][j];
            if (st == kWTab - 1) {
#pragma unroll
                for (int j = 0; j < kL28; j++) acc[j] = tab[0][j];
            }
        }
    }
    from28(acc, out32);
}

// ---------------------------------------------------------------------------
// The same exponentiation on a PAIR of lanes (the GPU kernel's form).  One
// lane per exponentiation gives a batch of 16384 objects 32768 threads, 512
// waves: one wave on half of the chip's 1024 SIMDs, each issuing the whole
// ~4.4K-instruction product stream alone.  Two lanes per exponentiation split
// every product by columns -- lane 0 holds columns 0..18, lane 1 columns
// 19..37 (column 37 stays zero) -- so the batch is 1024 waves issuing about
// half the instructions each.  Per row of the product the lanes exchange four
// words: a_i from the lane holding it, the reduction multiplier m_i (lane 0
// computes it from column 0), and the 64-bit column 19 that moves into lane 0
// when the accumulator shifts down.  The final carry and borrow chains cross
// the lanes once each.  Same arithmetic, bounds and schedule as mod_exp28
// (one multiply site, masked table scan), so constant time in the exponent
// the same way.
//
// X is the exchange between the two lanes: X::hi (0 or 1), X::lo(v) / X::up(v)
// (v as held by lane 0 / lane 1, in both lanes), X::other(v) (the partner's
// v), X::tracing() (the lane that records the test trace).  The GPU kernel
// passes DPP moves; the CPU pin (tests/harness/rsa_host.cpp) runs the two
// lanes as two threads meeting at a barrier per exchange.
// ---------------------------------------------------------------------------
constexpr int kPC = (kL28 + 1) / 2;  // columns per lane (2 kPC = 38 >= kL28)

template <class X>
JFSX_HD uint64_t lo64(const X &x, uint64_t v) {
    return (uint64_t)x.lo((uint32_t)v) | (uint64_t)x.lo((uint32_t)(v >> 32)) << 32;
}
template <class X>
JFSX_HD uint64_t other64(const X &x, uint64_t v) {
    return (uint64_t)x.other((uint32_t)v) | (uint64_t)x.other((uint32_t)(v >> 32)) << 32;
}

// this lane's kPC limbs of a 28-bit-limb value f[0..kL28)
template <class X>
JFSX_HD void pair_pick(const X &x, const uint32_t *f, uint32_t *y) {
    const uint32_t up = 0u - x.hi;
#pragma unroll
    for (int j = 0; j < kPC; j++) y[j] = (f[j] & ~up) | ((kPC + j < kL28 ? f[kPC + j] : 0u) & up);
}

// out = a b R'^-1 mod m on the pair: a, b, m, out are this lane's kPC limbs
// (normalized); minv = -m^-1 mod 2^28
template <class X>
JFSX_HD void mont_mul28_pair(const X &x, const uint32_t *a, const uint32_t *b, const uint32_t *m, uint32_t minv,
                             uint32_t *out) {
    if (x.tracing()) JFSX_RSA_TRACE('M', 2);
    const uint64_t low = (uint64_t)0 - (uint64_t)(x.hi ^ 1u);  // all-ones in lane 0
    uint64_t acc[kPC];
#pragma unroll
    for (int j = 0; j < kPC; j++) acc[j] = 0;
    // one row: + a_i b, + m_i m (m_i from lane 0's column 0), then the
    // columns move down one: column 0 leaves (its carry joins column 1) and
    // lane 1's first column becomes lane 0's last
    auto row = [&](uint32_t ai) {
#pragma unroll
        for (int j = 0; j < kPC; j++) acc[j] += (uint64_t)ai * b[j];
        const uint32_t mi = x.lo(((uint32_t)acc[0] * minv) & kM28);
#pragma unroll
        for (int j = 0; j < kPC; j++) acc[j] += (uint64_t)mi * m[j];
        const uint64_t c = acc[0] >> 28, s = other64(x, acc[0]);
#pragma unroll
        for (int j = 0; j < kPC - 1; j++) acc[j] = acc[j + 1];
        acc[kPC - 1] = s & low;
        acc[0] += c & low;
    };
#pragma unroll
    for (int r = 0; r < kPC; r++) row(x.lo(a[r]));
#pragma unroll
    for (int r = 0; r < kL28 - kPC; r++) row(x.up(a[r]));
    // normalize: each lane on its own, then lane 0's carry through lane 1
    uint32_t t[kPC], d[kPC];
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < kPC; j++) {
        c += acc[j];
        t[j] = (uint32_t)c & kM28;
        c >>= 28;
    }
    c = lo64(x, c) & ~low;
#pragma unroll
    for (int j = 0; j < kPC; j++) {
        c += t[j];
        t[j] = (uint32_t)c & kM28;
        c >>= 28;
    }
    // t - m: lane 0's borrow first, then lane 1's chain from it
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < kPC; j++) br = (t[j] - m[j] - br) >> 31;
    br = x.lo(br) & (0u - x.hi);
#pragma unroll
    for (int j = 0; j < kPC; j++) {
        const uint32_t v = t[j] - m[j] - br;
        d[j] = v & kM28;
        br = v >> 31;
    }
    const uint32_t keep = 0u - x.up(br);  // t < m
#pragma unroll
    for (int j = 0; j < kPC; j++) out[j] = (t[j] & keep) | (d[j] & ~keep);
}

// x^e mod m (x < m; 32-bit limbs in, out32 in both lanes), constant time in e:
// mod_exp28's schedule on the pair
template <class X>
JFSX_HD void mod_exp28_pair(const X &x, const uint32_t *x32, const uint32_t *e, const uint32_t *m32,
                            uint32_t minv32, const uint32_t *r2_32, uint32_t *out32) {
    uint32_t m[kPC], xv[kPC], r2[kPC];
    {
        uint32_t f[kL28];
        to28(m32, f);
        pair_pick(x, f, m);
        to28(x32, f);
        pair_pick(x, f, xv);
        to28(r2_32, f);
        pair_pick(x, f, r2);
    }
    const uint32_t minv = minv32 & kM28, one0 = x.hi ^ 1u;  // the Montgomery 1's low limb sits in lane 0
    uint32_t tab[kWTab][kPC];
    uint32_t acc[kPC], b[kPC];
    for (int w = 0; w < kWTab; w++)
        for (int j = 0; j < kPC; j++) tab[w][j] = 0;
    constexpr int kPer = kWBits + 1, kMain = kWTab + kPer * kWDigits;
#pragma unroll 1
    for (int st = 0; st <= kMain; st++) {
        if (st == 0) {
#pragma unroll
            for (int j = 0; j < kPC; j++) acc[j] = r2[j], b[j] = j == 0 ? one0 : 0u;
        } else if (st == 1) {
#pragma unroll
            for (int j = 0; j < kPC; j++) acc[j] = xv[j], b[j] = r2[j];
        } else if (st < kWTab) {
#pragma unroll
            for (int j = 0; j < kPC; j++) b[j] = tab[1][j];
        } else if (st < kMain) {
            const int r = st - kWTab;
            if (r % kPer < kWBits) {
#pragma unroll
                for (int j = 0; j < kPC; j++) b[j] = acc[j];
            } else {
                uint32_t idx = w_digit(e, kWDigits - 1 - r / kPer);
                JFSX_RSA_OPAQUE(idx);
#pragma unroll
                for (int j = 0; j < kPC; j++) b[j] = 0;
#pragma unroll
                for (uint32_t w = 0; w < (uint32_t)kWTab; w++) {
                    uint32_t msk = ~ct_nz(w ^ idx);
                    JFSX_RSA_OPAQUE(msk);
                    if (x.tracing()) JFSX_RSA_TRACE('S', w);
#pragma unroll
                    for (int j = 0; j < kPC; j++) b[j] |= tab[w][j] & msk;
                }
            }
        } else {
#pragma unroll
            for (int j = 0; j < kPC; j++) b[j] = j == 0 ? one0 : 0u;
        }
        mont_mul28_pair(x, acc, b, m, minv, acc);
        if (st < kWTab) {
#pragma unroll
            for (int w = 0; w < kWTab; w++)
#pragma unroll
                for (int j = 0; j < kPC; j++) tab[w][j] = st == w ? acc[j] : tab[w][j];
            if (st == kWTab - 1) {
#pragma unroll
                for (int j = 0; j < kPC; j++) acc[j] = tab[0][j];
            }
        }
    }
    // both halves of the result in both lanes, back to 32-bit limbs
    uint32_t f[2 * kPC];
    const uint32_t up = 0u - x.hi;
#pragma unroll
    for (int j = 0; j < kPC; j++) {
        const uint32_t o = x.other(acc[j]);
        f[j] = (acc[j] & ~up) | (o & up);
        f[kPC + j] = (o & ~up) | (acc[j] & up);
    }
    from28(f, out32);
}

// One whole unwrap on one thread (the CPU pin; the GPU splits it into the
// two half exponentiations and a finish kernel): ct = k bytes, big-endian.
// Returns the message length (msg in em[0..len)) or -1.
JFSX_HD int decrypt(const Key &k, const uint8_t *ct, uint8_t em[kModBytes]) {
    uint32_t c[2 * kLimbs], m1[kLimbs], m2[kLimbs], m[2 * kLimbs], x[kLimbs];
    from_be(ct, kModBytes, c, 2 * kLimbs);
    if (geq(c, k.n, 2 * kLimbs)) return -1;
    reduce_2048(c, k.p, k.pinv, k.r2p, x);
    mod_exp28(x, k.dp, k.p, k.pinv, k.r2p28, m1);
    reduce_2048(c, k.q, k.qinv32, k.r2q, x);
    mod_exp28(x, k.dq, k.q, k.qinv32, k.r2q28, m2);
    crt(k, m1, m2, m);
    to_be(m, 2 * kLimbs, em, kModBytes);
    return oaep_decode(em, kModBytes, k.lhash);
}

}  // namespace jfsx_rsa

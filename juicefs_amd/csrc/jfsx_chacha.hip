// jfsx_chacha.hip -- ChaCha20-Poly1305 Seal/Open fused with CRC32C segment
// checksums (gfx950).
//
// Replaces aead.Seal / aead.Open of chacha20poly1305.New(key)
// (golang.org/x/crypto v0.19.0, called at pkg/object/encrypt.go:158-159, :192,
// :215) and checksum() of the plaintext (pkg/chunk/disk_cache.go:1218-1231).
// RFC 8439 AEAD with empty AAD: keystream block 0 gives the Poly1305 key
// (r, s); data uses block counters 1, 2, ...; the tag is
// Poly1305(C || pad16 || le64(0) || le64(len C)).
//
// Pure VALU work (no MFMA, no tables except the CRC slice-by-16 tables in LDS):
//   * cp_keysetup: one wave per block: (r, s), r^(2^k), r^253, (len block)*r.
//   * cp_main: one 256-thread workgroup per task.  A wave row is 64 lanes x
//     64 B = 4 KiB; each lane computes one ChaCha20 block per row and XORs its
//     64 contiguous bytes.  Poly1305 runs as a per-lane Horner chain over the
//     lane's 16-B blocks (r between consecutive blocks, r^253 across rows) in
//     26-bit limbs with v_mad_u64_u32; CRC32C per lane (shift 4032 B across
//     rows).  At stream end each lane's sum is lifted by r^e and the wave
//     reduces modulo 2^130-5 into one partial.
//   * cp_finalize: one wave per block: lift partials by r^pexp, add, add the
//     length block, add s -> tag; compare in Open; CRC verify.
#include "jfsx_dev.h"

namespace jfsx {

constexpr uint32_t kLdsCrcCp = 0;
constexpr uint32_t M26 = 0x3ffffffu;

// ---------------------------------------------------------------------------
// Poly1305 arithmetic mod p = 2^130 - 5, five 26-bit limbs
// ---------------------------------------------------------------------------
struct P5 {
    uint32_t l[5];
};

__device__ __forceinline__ P5 p_zero() { return P5{{0, 0, 0, 0, 0}}; }
__device__ __forceinline__ P5 p_one() { return P5{{1, 0, 0, 0, 0}}; }

// a * b mod p (partially reduced: limbs < 2^26 + small)
__device__ __forceinline__ P5 p_mul(const P5 &a, const P5 &b) {
    const uint32_t s1 = b.l[1] * 5, s2 = b.l[2] * 5, s3 = b.l[3] * 5, s4 = b.l[4] * 5;
    typedef uint64_t u64;
    u64 d0 = (u64)a.l[0] * b.l[0] + (u64)a.l[1] * s4 + (u64)a.l[2] * s3 + (u64)a.l[3] * s2 + (u64)a.l[4] * s1;
    u64 d1 = (u64)a.l[0] * b.l[1] + (u64)a.l[1] * b.l[0] + (u64)a.l[2] * s4 + (u64)a.l[3] * s3 + (u64)a.l[4] * s2;
    u64 d2 = (u64)a.l[0] * b.l[2] + (u64)a.l[1] * b.l[1] + (u64)a.l[2] * b.l[0] + (u64)a.l[3] * s4 + (u64)a.l[4] * s3;
    u64 d3 = (u64)a.l[0] * b.l[3] + (u64)a.l[1] * b.l[2] + (u64)a.l[2] * b.l[1] + (u64)a.l[3] * b.l[0] + (u64)a.l[4] * s4;
    u64 d4 = (u64)a.l[0] * b.l[4] + (u64)a.l[1] * b.l[3] + (u64)a.l[2] * b.l[2] + (u64)a.l[3] * b.l[1] + (u64)a.l[4] * b.l[0];
    P5 r;
    d1 += d0 >> 26; r.l[0] = (uint32_t)d0 & M26;
    d2 += d1 >> 26; r.l[1] = (uint32_t)d1 & M26;
    d3 += d2 >> 26; r.l[2] = (uint32_t)d2 & M26;
    d4 += d3 >> 26; r.l[3] = (uint32_t)d3 & M26;
    const u64 t = (u64)r.l[0] + (d4 >> 26) * 5;
    r.l[4] = (uint32_t)d4 & M26;
    r.l[0] = (uint32_t)t & M26;
    r.l[1] += (uint32_t)(t >> 26);
    return r;
}

// Horner step a * b + m mod p for the main loop: b is r or r^253 (limbs
// < 2^26), sb[i] = 5 * b.l[i] precomputed, m a message block (limbs < 2^26).
// The message limbs and each carry enter the next limb's product sum as its
// first addend, carries are 32-bit (every d_i < 2^57, so d_i >> 26 < 2^31),
// and the top carry folds back into limb 0 times 5 (d4 has no wrapped
// products: d4 < 2^54.4, 5 * (d4 >> 26) < 2^31).  Output limbs < 2^26 except
// l[1] < 2^26 + 2^6.
#define MADC(x, y, z) ((uint64_t)(x) * (y) + (z))

__device__ __forceinline__ P5 p_mul_add(const P5 &a, const P5 &b, const uint32_t (&sb)[5], const P5 &m) {
    typedef uint64_t u64;
    P5 r;
    u64 d = MADC(a.l[4], sb[1], MADC(a.l[3], sb[2], MADC(a.l[2], sb[3], MADC(a.l[1], sb[4],
            MADC(a.l[0], b.l[0], (u64)m.l[0])))));
    r.l[0] = (uint32_t)d & M26;
    uint32_t c = (uint32_t)(d >> 26);
    d = MADC(a.l[4], sb[2], MADC(a.l[3], sb[3], MADC(a.l[2], sb[4], MADC(a.l[1], b.l[0],
        MADC(a.l[0], b.l[1], (u64)(c + m.l[1]))))));
    r.l[1] = (uint32_t)d & M26;
    c = (uint32_t)(d >> 26);
    d = MADC(a.l[4], sb[3], MADC(a.l[3], sb[4], MADC(a.l[2], b.l[0], MADC(a.l[1], b.l[1],
        MADC(a.l[0], b.l[2], (u64)(c + m.l[2]))))));
    r.l[2] = (uint32_t)d & M26;
    c = (uint32_t)(d >> 26);
    d = MADC(a.l[4], sb[4], MADC(a.l[3], b.l[0], MADC(a.l[2], b.l[1], MADC(a.l[1], b.l[2],
        MADC(a.l[0], b.l[3], (u64)(c + m.l[3]))))));
    r.l[3] = (uint32_t)d & M26;
    c = (uint32_t)(d >> 26);
    d = MADC(a.l[4], b.l[0], MADC(a.l[3], b.l[1], MADC(a.l[2], b.l[2], MADC(a.l[1], b.l[3],
        MADC(a.l[0], b.l[4], (u64)(c + m.l[4]))))));
    r.l[4] = (uint32_t)d & M26;
    c = (uint32_t)(d >> 26);
    const uint32_t t = r.l[0] + c * 5u;
    r.l[0] = t & M26;
    r.l[1] += t >> 26;
    return r;
}

__device__ __forceinline__ P5 p_add(const P5 &a, const P5 &b) {
    P5 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.l[i] = a.l[i] + b.l[i];
    return r;
}

// canonical representative in [0, p)
__device__ __forceinline__ P5 p_freeze(P5 a) {
    uint32_t c;
#pragma unroll
    for (int rep = 0; rep < 2; rep++) {
        c = a.l[0] >> 26; a.l[0] &= M26; a.l[1] += c;
        c = a.l[1] >> 26; a.l[1] &= M26; a.l[2] += c;
        c = a.l[2] >> 26; a.l[2] &= M26; a.l[3] += c;
        c = a.l[3] >> 26; a.l[3] &= M26; a.l[4] += c;
        c = a.l[4] >> 26; a.l[4] &= M26; a.l[0] += c * 5;
    }
    // a < 2^130 now; subtract p if a >= p
    P5 g;
    c = a.l[0] + 5; g.l[0] = c & M26; c >>= 26;
    c += a.l[1]; g.l[1] = c & M26; c >>= 26;
    c += a.l[2]; g.l[2] = c & M26; c >>= 26;
    c += a.l[3]; g.l[3] = c & M26; c >>= 26;
    c += a.l[4]; g.l[4] = c & M26; c >>= 26;  // c = 1 iff a + 5 >= 2^130 iff a >= p
    return c ? g : a;
}

// 16 little-endian bytes (+ 2^128 when hibit) to limbs
__device__ __forceinline__ P5 p_from_words(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t hibit) {
    P5 r;
    r.l[0] = w0 & M26;
    r.l[1] = __builtin_amdgcn_alignbit(w1, w0, 26) & M26;
    r.l[2] = __builtin_amdgcn_alignbit(w2, w1, 20) & M26;
    r.l[3] = __builtin_amdgcn_alignbit(w3, w2, 14) & M26;
    r.l[4] = (w3 >> 8) | (hibit << 24);
    return r;
}

__device__ __forceinline__ P5 p_load(const uint32_t *s) { return P5{{s[0], s[1], s[2], s[3], s[4]}}; }

// r^e from the r^(2^k) table
__device__ __forceinline__ P5 p_pow(const uint32_t (*r2k)[5], uint64_t e) {
    P5 z = p_one();
    for (int k = 0; e; k++, e >>= 1)
        if (e & 1) z = p_mul(z, p_load(r2k[k]));
    return z;
}

// wave-wide sum mod p of canonical values
__device__ __forceinline__ P5 p_wave_sum(P5 a) {
    for (int off = 32; off > 0; off >>= 1) {
        P5 b;
#pragma unroll
        for (int i = 0; i < 5; i++) b.l[i] = __shfl_xor(a.l[i], off, 64);
        a = p_freeze(p_add(a, b));
    }
    return a;
}

// ---------------------------------------------------------------------------
// ChaCha20 block (RFC 8439 2.3)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }

#define XR16(d, a) rotl((d) ^ (a), 16)

#define CP_QR(a, b, c, d)          \
    a += b; d = XR16(d, a);        \
    c += d; b = rotl(b ^ c, 12);   \
    a += b; d = rotl(d ^ a, 8);    \
    c += d; b = rotl(b ^ c, 7);

// Counter-uniform first column round: of the first double round's column
// quarter rounds, three never touch the counter word (x12) and the fourth
// starts with a += b on key words.  A wave computes those once per task
// (wave-uniform, SGPRs) and each block starts from them: 37 of the block's
// 960 + 16 ALU ops are gone.
struct CpUni {
    uint32_t a0;      // x0 + x4
    uint32_t w[16];   // state after the three counter-free column QRs (x1..3, x5..7, x9..11, x13..15)
    uint32_t in[16];  // input words (for the final add; in[12] unused)
};

__device__ __forceinline__ CpUni cp_uniform(const uint32_t *key, const uint32_t *nonce) {
    CpUni u;
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], 0u, nonce[0], nonce[1], nonce[2]};
#pragma unroll
    for (int i = 0; i < 16; i++) u.in[i] = x[i];
    CP_QR(x[1], x[5], x[9], x[13]);
    CP_QR(x[2], x[6], x[10], x[14]);
    CP_QR(x[3], x[7], x[11], x[15]);
    u.a0 = x[0] + x[4];
#pragma unroll
    for (int i = 0; i < 16; i++) u.w[i] = x[i];
    // wave-uniform: keep them in SGPRs
    u.a0 = __builtin_amdgcn_readfirstlane(u.a0);
#pragma unroll
    for (int i = 0; i < 16; i++) {
        u.w[i] = __builtin_amdgcn_readfirstlane(u.w[i]);
        u.in[i] = __builtin_amdgcn_readfirstlane(u.in[i]);
    }
    return u;
}

__device__ __forceinline__ void chacha_block_u(const CpUni &u, uint32_t ctr, uint32_t out[16]) {
    // column QR(x0, x4, x8, x12) from a = x0 + x4
    uint32_t x0 = u.a0, x4 = u.in[4], x8 = u.in[8], x12 = XR16(ctr, x0);
    x8 += x12; x4 = rotl(x4 ^ x8, 12);
    x0 += x4; x12 = rotl(x12 ^ x0, 8);
    x8 += x12; x4 = rotl(x4 ^ x8, 7);
    uint32_t x1 = u.w[1], x2 = u.w[2], x3 = u.w[3], x5 = u.w[5], x6 = u.w[6], x7 = u.w[7], x9 = u.w[9],
             x10 = u.w[10], x11 = u.w[11], x13 = u.w[13], x14 = u.w[14], x15 = u.w[15];
    CP_QR(x0, x5, x10, x15);
    CP_QR(x1, x6, x11, x12);
    CP_QR(x2, x7, x8, x13);
    CP_QR(x3, x4, x9, x14);
#pragma unroll
    for (int i = 1; i < 10; i++) {
        CP_QR(x0, x4, x8, x12);
        CP_QR(x1, x5, x9, x13);
        CP_QR(x2, x6, x10, x14);
        CP_QR(x3, x7, x11, x15);
        CP_QR(x0, x5, x10, x15);
        CP_QR(x1, x6, x11, x12);
        CP_QR(x2, x7, x8, x13);
        CP_QR(x3, x4, x9, x14);
    }
    out[0] = x0 + u.in[0]; out[1] = x1 + u.in[1]; out[2] = x2 + u.in[2]; out[3] = x3 + u.in[3];
    out[4] = x4 + u.in[4]; out[5] = x5 + u.in[5]; out[6] = x6 + u.in[6]; out[7] = x7 + u.in[7];
    out[8] = x8 + u.in[8]; out[9] = x9 + u.in[9]; out[10] = x10 + u.in[10]; out[11] = x11 + u.in[11];
    out[12] = x12 + ctr; out[13] = x13 + u.in[13]; out[14] = x14 + u.in[14]; out[15] = x15 + u.in[15];
}

__device__ __forceinline__ void chacha_block(const uint32_t *key, const uint32_t *nonce, uint32_t ctr,
                                             uint32_t out[16]) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = key[0], x5 = key[1], x6 = key[2], x7 = key[3], x8 = key[4], x9 = key[5], x10 = key[6],
             x11 = key[7];
    uint32_t x12 = ctr, x13 = nonce[0], x14 = nonce[1], x15 = nonce[2];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        CP_QR(x0, x4, x8, x12);
        CP_QR(x1, x5, x9, x13);
        CP_QR(x2, x6, x10, x14);
        CP_QR(x3, x7, x11, x15);
        CP_QR(x0, x5, x10, x15);
        CP_QR(x1, x6, x11, x12);
        CP_QR(x2, x7, x8, x13);
        CP_QR(x3, x4, x9, x14);
    }
    out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u; out[3] = x3 + 0x6b206574u;
    out[4] = x4 + key[0]; out[5] = x5 + key[1]; out[6] = x6 + key[2]; out[7] = x7 + key[3];
    out[8] = x8 + key[4]; out[9] = x9 + key[5]; out[10] = x10 + key[6]; out[11] = x11 + key[7];
    out[12] = x12 + ctr; out[13] = x13 + nonce[0]; out[14] = x14 + nonce[1]; out[15] = x15 + nonce[2];
}

// ---------------------------------------------------------------------------
// main transform
// ---------------------------------------------------------------------------
struct CpStream {
    P5 A;            // Poly1305 lane accumulator
    uint64_t jlast;  // last 16-B block folded into A
    bool has;
    uint32_t C, lend;  // CRC lane accumulator and end of its last piece (segment relative)
    uint64_t seg0;
};

template <int CRCMODE>
__device__ __forceinline__ void cp_segment_end(const BlkDev &blk, const DevTables &tab, uint32_t lane,
                                               uint64_t seg0, uint64_t seg1, uint32_t C, uint32_t lend) {
    const uint32_t Lseg = (uint32_t)(seg1 - seg0);
    uint32_t v, K;
    if (Lseg == (uint32_t)kSeg) {
        v = crc_mulmod(tab.crcx[128 + lane], C);
        K = tab.crcx[96];
    } else {
        v = crc_mulmod(crc_xpow8(Lseg - lend, tab.crcx + 64), C);
        K = crc_mulmod(crc_xpow8(Lseg, tab.crcx + 64), 0xffffffffu);
    }
    const uint32_t raw = wave_xor(v);
    if (lane == 0) {
        const uint32_t crc = ~(K ^ raw);
        const uint64_t si = seg0 / kSeg;
        if ((CRCMODE & 3) == 1)
            *reinterpret_cast<uint32_t *>(blk.crc + 4 * si) = __builtin_bswap32(crc);
        else
            blk.crc_calc[si] = crc;
    }
}

// guarded row (block tail): pieces past the end are skipped, a partial piece is
// zero padded for Poly1305 and CRC'd byte-wise
template <bool OPEN, int CRCMODE>
__device__ __noinline__ CpStream cp_row_generic(const char *lds, const CpSched *sch, const BlkDev blk,
                                                const DevTables tab, uint32_t lane, CpStream st, uint64_t row,
                                                uint64_t end) {
    const uint64_t base = row + 64 * lane;
    uint32_t key[8], nonce[3];
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = sch->key[i];
#pragma unroll
    for (int i = 0; i < 3; i++) nonce[i] = sch->nonce[i];
    const P5 r1 = p_load(sch->r), r253 = p_load(sch->r253);
    uint32_t ks[16];
    if (base < end) chacha_block(key, nonce, (uint32_t)(base / 64 + 1), ks);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint64_t o = base + 16 * q;
        if (o >= end) break;
        const bool full = o + 16 <= end;
        const uint4 d = load_piece(blk.src, o, end);
        uint4 x = make_uint4(d.x ^ ks[4 * q], d.y ^ ks[4 * q + 1], d.z ^ ks[4 * q + 2], d.w ^ ks[4 * q + 3]);
        uint4 c = OPEN ? d : x, p = OPEN ? x : d;
        if (!full) {
            const int nv = (int)(end - o);
            uint32_t m[4];
            for (int k = 0; k < 4; k++) {
                int bytes = nv - 4 * k;
                m[k] = bytes >= 4 ? 0xffffffffu : (bytes <= 0 ? 0u : ((1u << (8 * bytes)) - 1u));
            }
            c.x &= m[0]; c.y &= m[1]; c.z &= m[2]; c.w &= m[3];
            p.x &= m[0]; p.y &= m[1]; p.z &= m[2]; p.w &= m[3];
        }
        store_piece(blk.dst, o, end, OPEN ? p : c);
        st.A = p_add(p_mul(st.A, q == 0 ? r253 : r1), p_from_words(c.x, c.y, c.z, c.w, 1));
        const uint4 cq = crc_src<CRCMODE>(c, p);
        st.jlast = o >> 4;
        st.has = true;
        if (CRCMODE) {
            if (full) {
                st.C = q == 0 ? crc_piece<kLdsCrcCp, 20>(lds, st.C, cq.x, cq.y, cq.z, cq.w)
                              : crc_piece<kLdsCrcCp, -1>(lds, st.C, cq.x, cq.y, cq.z, cq.w);
                st.lend = (uint32_t)(o + 16 - st.seg0);
            } else {
                const uint32_t pw[4] = {cq.x, cq.y, cq.z, cq.w};
                st.C = q == 0 ? crc_partial<kLdsCrcCp, 20>(lds, st.C, pw, (int)(end - o))
                              : crc_partial<kLdsCrcCp, -1>(lds, st.C, pw, (int)(end - o));
                st.lend = (uint32_t)(end - st.seg0);
            }
        }
    }
    if (CRCMODE) {
        const uint64_t seg1 = st.seg0 + kSeg < end ? st.seg0 + kSeg : end;
        if (row + 4096 >= seg1) {
            cp_segment_end<CRCMODE>(blk, tab, lane, st.seg0, seg1, st.C, st.lend);
            st.C = 0;
            st.lend = 0;
            st.seg0 = seg1;
        }
    }
    return st;
}

// One task (a block's <= 1 MiB range) on the workgroup's four waves, whole
// 32 KiB segments per wave; the CRC tables are already in LDS.
template <bool OPEN, int CRCMODE>
__device__ __forceinline__ void cp_task(const char *lds, const Task task, const BlkDev *__restrict__ blks,
                                        const CpSched *__restrict__ sched, uint32_t *__restrict__ partial,
                                        uint32_t *__restrict__ pexp, const DevTables &tab, uint32_t tid) {
    const BlkDev blk = blks[task.blk];
    const CpSched *sch = sched + task.blk;
    uint32_t key[8], nonce[3];
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = sch->key[i];
#pragma unroll
    for (int i = 0; i < 3; i++) nonce[i] = sch->nonce[i];
    const P5 r1 = p_load(sch->r), r253 = p_load(sch->r253);
    const CpUni uni = cp_uniform(key, nonce);
    uint32_t s1[5], s253[5];
#pragma unroll
    for (int i = 0; i < 5; i++) {
        s1[i] = 5u * r1.l[i];
        s253[i] = 5u * r253.l[i];
    }

    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t c0 = task.c0, c1 = task.c1;
    const uint32_t nseg = (uint32_t)((c1 - c0 + kSeg - 1) / kSeg);
    const uint32_t sa = wave * nseg / kCpWaves, sb = (wave + 1) * nseg / kCpWaves;
    const uint64_t sub0 = c0 + (uint64_t)sa * kSeg;
    const uint64_t sub1 = sb > sa ? (c0 + (uint64_t)sb * kSeg < c1 ? c0 + (uint64_t)sb * kSeg : c1) : sub0;
    const uint8_t *src = blk.src;
    uint8_t *dst = blk.dst;

    CpStream st;
    st.A = p_zero();
    st.jlast = 0;
    st.has = false;
    st.C = 0;
    st.lend = 0;
    st.seg0 = sub0;
    const uint64_t rf = (sub1 - sub0) / 4096;  // full rows
    const uint64_t lo = 64 * lane;
    for (uint64_t r = 0; r < rf; r++) {
        const uint64_t o = sub0 + 4096 * r + lo;
        uint4 d[4];
#pragma unroll
        for (int q = 0; q < 4; q++) d[q] = ald16(src + o + 16 * q);
        uint32_t ks[16];
        chacha_block_u(uni, (uint32_t)(o / 64 + 1), ks);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint4 x = make_uint4(d[q].x ^ ks[4 * q], d[q].y ^ ks[4 * q + 1], d[q].z ^ ks[4 * q + 2],
                                       d[q].w ^ ks[4 * q + 3]);
            const uint4 c = OPEN ? d[q] : x, p = OPEN ? x : d[q];
            ast16(dst + o + 16 * q, OPEN ? p : c);
            const uint4 cq = crc_src<CRCMODE>(c, p);
            st.A = q == 0 ? p_mul_add(st.A, r253, s253, p_from_words(c.x, c.y, c.z, c.w, 1))
                          : p_mul_add(st.A, r1, s1, p_from_words(c.x, c.y, c.z, c.w, 1));
            if (CRCMODE) {
                st.C = q == 0 ? crc_piece<kLdsCrcCp, 20>(lds, st.C, cq.x, cq.y, cq.z, cq.w)
                              : crc_piece<kLdsCrcCp, -1>(lds, st.C, cq.x, cq.y, cq.z, cq.w);
            }
        }
        if (CRCMODE && (r & 7) == 7) {
            cp_segment_end<CRCMODE>(blk, tab, lane, st.seg0, st.seg0 + kSeg, st.C, 0);
            st.C = 0;
            st.seg0 += kSeg;
        }
    }
    if (rf) {
        st.has = true;
        st.jlast = (sub0 + 4096 * (rf - 1) + lo + 48) >> 4;
        const uint64_t used = sub0 + 4096 * rf - st.seg0;  // bytes of the open segment already processed
        st.lend = used ? (uint32_t)(used - 4096 + lo + 64) : 0;
    }
    for (uint64_t row = sub0 + 4096 * rf; row < sub1; row += 4096)
        st = cp_row_generic<OPEN, CRCMODE>(lds, sch, blk, tab, lane, st, row, sub1);
    if (CRCMODE && st.seg0 < sub1) {
        cp_segment_end<CRCMODE>(blk, tab, lane, st.seg0, sub1, st.C, st.lend);
        st.seg0 = sub1;
    }

    // ---- stream epilogue ----
    const uint64_t wend = (sub1 + 15) >> 4;
    P5 z = p_zero();
    if (st.has && sub1 > sub0) z = p_freeze(p_mul(st.A, p_pow(sch->r2k, wend + 1 - st.jlast)));
    z = p_wave_sum(z);
    if (lane == 0) {
        const uint32_t slot = task.slot0 + wave;
#pragma unroll
        for (int i = 0; i < 5; i++) partial[8 * slot + i] = z.l[i];
        const uint64_t nblk = (blk.len + 15) >> 4;
        pexp[slot] = (uint32_t)(nblk - wend);
    }
}

// cp_main: persistent workgroups (kCpGroupsPerCu per CU, the occupancy the
// kernel's registers allow) taking tasks, largest first, from a queue; the
// CRC tables are staged once per workgroup.  See gcm_main_k for why a grid of
// one workgroup per task leaves CUs idle on mixed block sizes.
template <bool OPEN, int CRCMODE>
__global__ __launch_bounds__(kCpWaves * 64) void cp_main_k(const Task *__restrict__ tasks, uint32_t ntasks,
                                                          uint32_t *__restrict__ queue,
                                                          const BlkDev *__restrict__ blks,
                                                          const CpSched *__restrict__ sched,
                                                          uint32_t *__restrict__ partial, uint32_t *__restrict__ pexp,
                                                          DevTables tab) {
    __shared__ __attribute__((aligned(16))) char lds[CRCMODE ? 24576 : 16];
    __shared__ uint32_t s_task;
    const uint32_t tid = threadIdx.x;
    if (CRCMODE) {
        const uint4 *gc = reinterpret_cast<const uint4 *>(tab.crc);
        uint4 *lc = reinterpret_cast<uint4 *>(lds);
        for (uint32_t i = tid; i < 1536; i += kCpWaves * 64) lc[i] = gc[i];
    }
    if (tid == 0) s_task = atomicAdd(queue, 1u);
    for (;;) {
        __syncthreads();
        const uint32_t ti = __builtin_amdgcn_readfirstlane(s_task);
        if (ti >= ntasks) break;  // the same for every wave: the queue is exhausted
        __syncthreads();          // every wave holds ti: s_task may take the next index
        if (tid == 0) s_task = atomicAdd(queue, 1u);
        cp_task<OPEN, CRCMODE>(lds, tasks[ti], blks, sched, partial, pexp, tab, tid);
    }
}

// ---------------------------------------------------------------------------
// keysetup: one wave per block
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void cp_keysetup_k(const KeyIn *__restrict__ keys, const BlkDev *__restrict__ blks,
                                                   CpSched *__restrict__ sched) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    CpSched *sc = sched + b;
    const KeyIn k = keys[b];
    uint32_t blk0[16];
    chacha_block(k.key, k.nonce, 0, blk0);
    // clamp r (RFC 8439 2.5.1)
    const P5 r = p_from_words(blk0[0] & 0x0fffffffu, blk0[1] & 0x0ffffffcu, blk0[2] & 0x0ffffffcu,
                              blk0[3] & 0x0ffffffcu, 0);
    if (lane < 8) sc->key[lane] = k.key[lane];
    if (lane < 3) sc->nonce[lane] = k.nonce[lane];
    if (lane < 4) sc->s[lane] = blk0[4 + lane];
    P5 g = r;
    P5 r253 = p_one();
    for (int i = 0; i < 32; i++) {
        if ((int)lane == i)
            for (int q = 0; q < 5; q++) sc->r2k[i][q] = g.l[q];
        if ((253 >> i) & 1) r253 = p_mul(r253, g);
        g = p_mul(g, g);
    }
    if (lane == 0) {
        const uint64_t len = blks[b].len;
        const P5 L = p_from_words(0, 0, (uint32_t)len, (uint32_t)(len >> 32), 1);
        const P5 init = p_freeze(p_mul(L, r));
        for (int q = 0; q < 5; q++) {
            sc->r[q] = r.l[q];
            sc->r253[q] = r253.l[q];
            sc->init[q] = init.l[q];
        }
    }
}

// ---------------------------------------------------------------------------
// finalize: one wave per block
// ---------------------------------------------------------------------------
template <bool OPEN, int CRCMODE>
__global__ __launch_bounds__(64) void cp_finalize_k(const BlkDev *__restrict__ blks, const CpSched *__restrict__ sched,
                                                   const uint32_t *__restrict__ partial,
                                                   const uint32_t *__restrict__ pexp, BlkOut *__restrict__ out) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const BlkDev blk = blks[b];
    const CpSched *sc = sched + b;
    P5 acc = p_zero();
    for (uint32_t base = 0; base < blk.nslots; base += 64) {
        const uint32_t s = base + lane;
        P5 z = p_zero();
        if (s < blk.nslots) {
            const uint32_t slot = blk.slot0 + s;
            z = p_load(partial + 8 * slot);
            if (z.l[0] | z.l[1] | z.l[2] | z.l[3] | z.l[4]) z = p_freeze(p_mul(z, p_pow(sc->r2k, pexp[slot])));
        }
        acc = p_freeze(p_add(acc, p_wave_sum(z)));
    }
    acc = p_freeze(p_add(acc, p_load(sc->init)));
    // h + s mod 2^128
    const uint32_t h0 = acc.l[0] | (acc.l[1] << 26), h1 = (acc.l[1] >> 6) | (acc.l[2] << 20),
                   h2 = (acc.l[2] >> 12) | (acc.l[3] << 14), h3 = (acc.l[3] >> 18) | (acc.l[4] << 8);
    uint64_t t = (uint64_t)h0 + sc->s[0];
    BlkOut o;
    o.tag[0] = (uint32_t)t;
    t = (t >> 32) + h1 + sc->s[1];
    o.tag[1] = (uint32_t)t;
    t = (t >> 32) + h2 + sc->s[2];
    o.tag[2] = (uint32_t)t;
    t = (t >> 32) + h3 + sc->s[3];
    o.tag[3] = (uint32_t)t;
    o.status = JFSX_OK;
    o.bad_seg = -1;
    o.got = o.expect = 0;
    if (OPEN) {
        const uint32_t *tg = reinterpret_cast<const uint32_t *>(blk.tag_in);
        uint32_t d = 0;
        for (int q = 0; q < 4; q++) d |= o.tag[q] ^ tg[q];
        if (d) o.status = JFSX_ETAG;
    }
    if ((CRCMODE & 3) == 2) {
        crc_verify_block(blk, o, lane);
        if (o.bad_seg >= 0 && o.status == JFSX_OK) o.status = JFSX_ECRC;
    }
    if (lane == 0) out[b] = o;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_cp_keysetup(hipStream_t s, int n, const KeyIn *keys, const BlkDev *blks, CpSched *sched) {
    if (n > 0) hipLaunchKernelGGL(cp_keysetup_k, dim3(n), dim3(64), 0, s, keys, blks, sched);
}

void launch_cp_main(hipStream_t s, int ntasks, int ncu, uint32_t *queue, bool open, int crc_mode, const Task *tasks,
                    const BlkDev *blks, const CpSched *sched, uint32_t *partial, uint32_t *pexp, DevTables t) {
    if (ntasks <= 0) return;
    const int groups = ncu * kCpGroupsPerCu;
    dim3 g(ntasks < groups ? ntasks : groups), bl(kCpWaves * 64);
    // queue: zeroed by the caller (uploaded with the batch descriptors)
#define L(O, C) hipLaunchKernelGGL((cp_main_k<O, C>), g, bl, 0, s, tasks, (uint32_t)ntasks, queue, blks, sched, \
                                   partial, pexp, t)
    switch ((open ? 8 : 0) | crc_mode) {
        case 8: L(true, 0); break;
        case 9: L(true, 1); break;
        case 10: L(true, 2); break;
        case 13: L(true, 5); break;
        case 14: L(true, 6); break;
        case 0: L(false, 0); break;
        case 1: L(false, 1); break;
        case 2: L(false, 2); break;
        case 5: L(false, 5); break;
        case 6: L(false, 6); break;
    }
#undef L
}

void launch_cp_finalize(hipStream_t s, int n, bool open, int crc_mode, const BlkDev *blks, const CpSched *sched,
                        const uint32_t *partial, const uint32_t *pexp, BlkOut *out) {
    if (n <= 0) return;
#define L(O, C) hipLaunchKernelGGL((cp_finalize_k<O, C>), dim3(n), dim3(64), 0, s, blks, sched, partial, pexp, out)
    if (open) {
        if ((crc_mode & 3) == 2) L(true, 2); else L(true, 0);
    } else {
        if ((crc_mode & 3) == 2) L(false, 2); else L(false, 0);
    }
#undef L
}

}  // namespace jfsx

// jfsx_gcm.hip -- AES-256-GCM Seal/Open fused with CRC32C segment checksums (gfx950).
//
// Replaces, per block, aead.Seal / aead.Open of cipher.NewGCM(aes.NewCipher(key))
// (pkg/object/encrypt.go:150-156, :192, :215) and checksum() over the plaintext
// (pkg/chunk/disk_cache.go:1218-1231).  Output is bit-exact to SP 800-38D with a
// 96-bit nonce, 128-bit tag and empty AAD: J0 = nonce || 1, data counters start
// at inc32(J0) = 2, tag = E_K(J0) ^ GHASH_H(C || pad || 0^64 || BE64(8*len)).
//
// Work decomposition:
//   * gcm_keysetup: one wave per block.  AES-256 key expansion, H = E_K(0),
//     E_K(J0), H^(2^k), H^0..H^67, the GHASH byte-table basis x^i*H^64, and the
//     round-1 constants of the counter blocks.
//   * gcm_main: one 1024-thread workgroup per task (block, <=4 MiB range).
//     LDS holds a 32-way replicated T0|T2 AES table (64 KiB, conflict-free),
//     the 16 x 256 GHASH table for "multiply by H^64" (64 KiB) and the
//     slice-by-16 CRC32C tables (20 KiB).  Each wave owns whole 32 KiB
//     segments; a wave row is 64 lanes x 16 B = 1 KiB.  Per row a lane:
//     AES-CTR of its counter, XOR, store, GHASH Horner step acc = acc*H^64 ^ C,
//     CRC32C step over the plaintext.  At segment end the lane CRCs are
//     shifted to the segment end and XOR-reduced; at wave end the GHASH lane
//     accumulators are lifted by H^(e_lane) and reduced to one partial.
//   * gcm_finalize: one wave per block.  Lifts each wave partial by
//     H^(blocks after that wave), XORs, adds E_K(J0)^len-block -> tag; in Open
//     compares the tag; in VERIFY compares CRCs (first failing segment).
#include <cstdio>
#include <cstdlib>

// plaintext in and ciphertext out as non-temporal block streams (coalesced
// 1 KiB rows, read or written once): +0.7 % same box (profiles/r4/ab_gcm_rows.txt;
// the ChaCha kernel's 64-byte lane runs lose 33 % with the hint and keep 0)
#ifndef JFSX_AEAD_NT
#define JFSX_AEAD_NT 3
#endif
#include "jfsx_dev.h"

#define JFSX_HD __device__ __forceinline__
#define BS3(a, b, c, tt) __builtin_amdgcn_bitop3_b32((a), (b), (c), (tt))
#define PERM(hi, lo, sel) __builtin_amdgcn_perm((hi), (lo), (sel))
#define OPAQUE(x)                                 \
    do {                                          \
        (x) = __builtin_amdgcn_readfirstlane(x);  \
        asm volatile("" : "+s"(x));               \
    } while (0)
#include "jfsx_aes_bs.h"

namespace jfsx {

// ---------------------------------------------------------------------------
// LDS map of gcm_main (bytes): [0, 20K) CRC tables, [20K, 84K) GHASH table,
// [84K, 148K) AES T0|T2, [148K, +2K) GHASH basis staging.  Every table's base
// is reached through the 16-bit ds_read offset: the CRC and GHASH bases
// directly, the AES base as 0x10000 (bit 16 of the lane's v_perm operand loff)
// plus the offset 20K.  So no lookup spends a VALU op on its base.
// ---------------------------------------------------------------------------
// JFSX_GF_CT_LIFT (default 1): the main kernel's per-lane GHASH lifts by
// g_mul_ct instead of the bit-serial g_mul (A/B builds)
#ifndef JFSX_GF_CT_LIFT
#define JFSX_GF_CT_LIFT 1
#endif

constexpr uint32_t kLdsCrc = 0;
constexpr uint32_t kLdsGh = 20480;              // GHASH T[b][j]: kLdsGh + (b << 8) | (j << 4)
constexpr uint32_t kLdsAesOff = 20480;          // ds_read offset of the AES table
constexpr uint32_t kLdsAes = 65536 + kLdsAesOff;  // AES [idx][T0 x32 | T2 x32]: 0x10000 | (idx << 8) | (r << 2), + offset
constexpr uint32_t kLdsBasis = kLdsAes + 65536;
// row-split tasks: per segment of the task, the XOR of the waves' raw CRC
// shares (128 segments of 32 KiB per 4 MiB task) and a flag per segment
constexpr uint32_t kLdsSegRaw = kLdsBasis + 2048;
constexpr uint32_t kLdsSegFlag = kLdsSegRaw + 512;
constexpr uint32_t kLdsBytes = kLdsSegFlag + 512;

__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// round key i as the T-table rounds consume it (pre-rotated for rounds 2..13, see AES_COL)
__device__ __forceinline__ uint32_t rk_load(const uint32_t *rk, int i) {
    uint32_t k = rk[i];
    if (JFSX_RKR && i >= 8 && i < 56) {
        k = (k >> 8) | (k << 24);
        OPAQUE(k);  // keep it in an SGPR (a VALU rotate would cost 48 VGPRs)
    }
    return k;
}

// byte k of w moved to bits 8..15, the lane's replica offset (bits 0..7) and the
// table base (bit 16) taken from loff: the LDS byte address of T0[byte] for this
// lane's replica in one v_perm_b32
#define AES_SEL(k) (0x0c020000u | ((4u + (k)) << 8))
#define TA(w, k) lds_u32(lds, __builtin_amdgcn_perm((w), loff, AES_SEL(k)) + kLdsAesOff)
#define TB(w, k) lds_u32(lds, __builtin_amdgcn_perm((w), loff, AES_SEL(k)) + (kLdsAesOff + 128u))

// One full AES round on LE column words.  T1 = rotl8 T0 and T3 = rotl8 T2, and
// rotl8(a) ^ rotl8(b) = rotl8(a ^ b), so a column costs 4 v_perm (addresses),
// 4 ds_read_b32, one xor, one alignbit and one 3-input xor (v_bitop3 0x96).
#if JFSX_RKR
// rounds 2..13 hold their round keys pre-rotated (rk_load: rotr8), so the key
// joins the rotated pair's 3-input XOR and a column is 4 v_perm, 4 ds_read_b32,
// two v_bitop3 and one alignbit
#define AES_COL(o, i0, i1, i2, i3, rkv) \
    o = xor3(TA(i0, 0), TB(i2, 2), rotl8(xor3(TA(i1, 1), TB(i3, 3), (rkv))));
#else
#define AES_COL(o, i0, i1, i2, i3, rkv) \
    o = xor3(TA(i0, 0), TB(i2, 2), rotl8(TA(i1, 1) ^ TB(i3, 3))) ^ (rkv);
#endif
#define AES_ROUND(o0, o1, o2, o3, i0, i1, i2, i3, r) \
    AES_COL(o0, i0, i1, i2, i3, rk[4 * (r) + 0])     \
    AES_COL(o1, i1, i2, i3, i0, rk[4 * (r) + 1])     \
    AES_COL(o2, i2, i3, i0, i1, rk[4 * (r) + 2])     \
    AES_COL(o3, i3, i0, i1, i2, rk[4 * (r) + 3])

// last round: S-box bytes are byte 0 of T2, bytes 1/2 of T0, byte 3 of T2
#define AES_LAST(o, a, b, c, d, rkv)                                                             \
    o = __builtin_amdgcn_bitop3_b32(                                                             \
            __builtin_amdgcn_bitop3_b32(TB(a, 0), TA(b, 1), 0xffu, 0xe4) /* select: c ? a : b */,       \
            __builtin_amdgcn_bitop3_b32(TA(c, 2), TB(d, 3), 0x00ff0000u, 0xe4),                 \
            0x0000ffffu, 0xe4) ^ (rkv);

// Keystream blocks for NS independent counters (the chains interleave for ILP).
template <int NS>
__device__ __forceinline__ void aes_ctr_blocks(const char *lds, uint32_t loff, const uint32_t *rk, const uint32_t *k1,
                                               const uint32_t (&ctr)[NS], uint32_t (&ks)[NS][4]) {
    uint32_t a[NS][4], b[NS][4];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const uint32_t x3 = __builtin_bswap32(ctr[s]) ^ rk[3];
        // round 1: the columns' constant terms are precomputed (k1); only x3 varies
        a[s][0] = k1[0] ^ rotl8(TB(x3, 3));
        a[s][1] = k1[1] ^ TB(x3, 2);
        a[s][2] = k1[2] ^ rotl8(TA(x3, 1));
        a[s][3] = k1[3] ^ TA(x3, 0);
    }
#pragma unroll
    for (int r = 2; r <= 13; r += 2) {
#pragma unroll
        for (int s = 0; s < NS; s++) { AES_ROUND(b[s][0], b[s][1], b[s][2], b[s][3], a[s][0], a[s][1], a[s][2], a[s][3], r); }
#pragma unroll
        for (int s = 0; s < NS; s++) { AES_ROUND(a[s][0], a[s][1], a[s][2], a[s][3], b[s][0], b[s][1], b[s][2], b[s][3], r + 1); }
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
        AES_LAST(ks[s][0], a[s][0], a[s][1], a[s][2], a[s][3], rk[56]);
        AES_LAST(ks[s][1], a[s][1], a[s][2], a[s][3], a[s][0], rk[57]);
        AES_LAST(ks[s][2], a[s][2], a[s][3], a[s][0], a[s][1], rk[58]);
        AES_LAST(ks[s][3], a[s][3], a[s][0], a[s][1], a[s][2], rk[59]);
    }
}

// Counter-uniform rounds.  Within one 1 KiB row the 64 counters are C + lane,
// so the counter's upper 24 bits U are wave-uniform except for the lanes past a
// carry.  After round 1 only column 0 (the one fed by the counter's low byte)
// varies with the low byte; columns 1..3 depend on U alone, and so do 12 of
// round 2's 16 lookups.  aes_r2_uniform gives, for one U, round 2's per-column
// sum of those 12 lookups and the round key; a wave computes a window of 64 U
// values once (lane l <-> U0 + l) and each row reads its lanes' entries with
// v_readlane.  A row then needs 5 table lookups for rounds 1-2 instead of 20.
__device__ __forceinline__ void aes_r2_uniform(const char *lds, uint32_t loff, const uint32_t *rk, const uint32_t *k1,
                                               uint32_t U, uint32_t (&u)[4]) {
    const uint32_t x3 = __builtin_bswap32(U << 8) ^ rk[3];
    const uint32_t a1 = k1[1] ^ TB(x3, 2);
    const uint32_t a2 = k1[2] ^ rotl8(TA(x3, 1));
    const uint32_t a3 = k1[3] ^ TA(x3, 0);
#if JFSX_RKR
    u[0] = xor3(TB(a2, 2), rotl8(xor3(TA(a1, 1), TB(a3, 3), rk[8])), 0u);
    u[1] = xor3(TA(a1, 0), TB(a3, 2), rotl8(TA(a2, 1) ^ rk[9]));
    u[2] = xor3(TA(a2, 0), rotl8(xor3(TA(a3, 1), TB(a1, 3), rk[10])), 0u);
    u[3] = xor3(TA(a3, 0), TB(a1, 2), rotl8(TB(a2, 3) ^ rk[11]));
#else
    u[0] = xor3(TB(a2, 2), rotl8(TA(a1, 1) ^ TB(a3, 3)), rk[8]);
    u[1] = xor3(TA(a1, 0), TB(a3, 2), rotl8(TA(a2, 1))) ^ rk[9];
    u[2] = xor3(TA(a2, 0), rotl8(TA(a3, 1) ^ TB(a1, 3)), rk[10]);
    u[3] = xor3(TA(a3, 0), TB(a1, 2), rotl8(TB(a2, 3))) ^ rk[11];
#endif
}

// aes_ctr_blocks with rounds 1-2 taken from the lane's counter-uniform terms u;
// ks comes out without the last round key (rk[56..59]).
template <int NS>
__device__ __forceinline__ void aes_ctr_blocks_u(const char *lds, uint32_t loff, const uint32_t *rk,
                                                 const uint32_t *k1, const uint32_t (&ctr)[NS],
                                                 const uint32_t (&u)[NS][4], const uint32_t (&du)[NS][4],
                                                 const uint32_t (&cym)[NS], uint32_t (&ks)[NS][4]) {
    uint32_t a[NS][4], b[NS][4];
    // u, du wave-uniform (SGPR operands); carry lanes (cym = ~0) add du = u(U) ^ u(U + 1)
#define UC(t, w) (__builtin_amdgcn_bitop3_b32((t), cym[s], du[s][w], 0x78) ^ u[s][w]) /* t ^ (cym & du) ^ u */
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const uint32_t x3 = __builtin_bswap32(ctr[s]) ^ rk[3];
        const uint32_t a0 = k1[0] ^ rotl8(TB(x3, 3));
        b[s][0] = UC(TA(a0, 0), 0);
        b[s][1] = UC(rotl8(TB(a0, 3)), 1);
        b[s][2] = UC(TB(a0, 2), 2);
        b[s][3] = UC(rotl8(TA(a0, 1)), 3);
    }
#undef UC
#pragma unroll
    for (int s = 0; s < NS; s++) { AES_ROUND(a[s][0], a[s][1], a[s][2], a[s][3], b[s][0], b[s][1], b[s][2], b[s][3], 3); }
#pragma unroll
    for (int r = 4; r <= 13; r += 2) {
#pragma unroll
        for (int s = 0; s < NS; s++) { AES_ROUND(b[s][0], b[s][1], b[s][2], b[s][3], a[s][0], a[s][1], a[s][2], a[s][3], r); }
#pragma unroll
        for (int s = 0; s < NS; s++) { AES_ROUND(a[s][0], a[s][1], a[s][2], a[s][3], b[s][0], b[s][1], b[s][2], b[s][3], r + 1); }
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
        // the last round key is left out: the caller folds it into the data XOR
        AES_LAST(ks[s][0], a[s][0], a[s][1], a[s][2], a[s][3], 0u);
        AES_LAST(ks[s][1], a[s][1], a[s][2], a[s][3], a[s][0], 0u);
        AES_LAST(ks[s][2], a[s][2], a[s][3], a[s][0], a[s][1], 0u);
        AES_LAST(ks[s][3], a[s][3], a[s][0], a[s][1], a[s][2], 0u);
    }
}

// GHASH "multiply by H^64" with the byte-sliced table T[b][j] = (byte b at
// position j) * H^64.  Bank-conflict-free: lane l keeps its accumulator rotated
// by k = (l & 15) >> 2 dwords (R[i] = acc[(i + k) & 3]) and visits the 16 byte
// positions in the lane-dependent order j(t) = 4((t/4 + k) & 3) + ((t + l) & 3),
// so the 16 lanes of every ds_read_b128 group read 16 distinct 16-byte slots
// (slot = j).  One v_perm per lookup builds (b << 8) | (j << 4).
struct GhLane {
    uint32_t sel[4];  // v_perm selectors: byte0 <- off byte t&3, byte1 <- R[t/4] byte (t + l) & 3
    uint32_t off[4];  // j(t) << 4 for t = 4*dd + 0..3, one byte each
    bool r1, r2;      // rotation bits of k
    uint32_t p1, p2;  // the same bits as v_perm selectors (whole dword from src0 or src1)
};

__device__ __forceinline__ GhLane gh_lane(uint32_t lane) {
    GhLane g;
    const uint32_t q = lane & 15, k = q >> 2;
#pragma unroll
    for (int bb = 0; bb < 4; bb++) g.sel[bb] = 0x0c0c0000u | ((4u + ((bb + q) & 3)) << 8) | (uint32_t)bb;
#pragma unroll
    for (int dd = 0; dd < 4; dd++) {
        uint32_t o = 0;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const uint32_t j = 4 * ((dd + k) & 3) + ((bb + q) & 3);
            o |= (j << 4) << (8 * bb);
        }
        g.off[dd] = o;
    }
    g.r1 = (k & 1) != 0;
    g.r2 = (k & 2) != 0;
    g.p1 = g.r1 ? 0x07060504u : 0x03020100u;
    g.p2 = g.r2 ? 0x07060504u : 0x03020100u;
    return g;
}

// R = rho(a): R[i] = a[(i + k) & 3]
__device__ __forceinline__ void gh_rho(const uint32_t a[4], const GhLane &g, uint32_t R[4]) {
    uint32_t u[4];
#pragma unroll
    // v_perm with a per-lane whole-dword selector: no VCC to rebuild per select
    for (int i = 0; i < 4; i++) u[i] = JFSX_GHPERM ? PERM(a[(i + 2) & 3], a[i], g.p2) : (g.r2 ? a[(i + 2) & 3] : a[i]);
#pragma unroll
    for (int i = 0; i < 4; i++) R[i] = JFSX_GHPERM ? PERM(u[(i + 1) & 3], u[i], g.p1) : (g.r1 ? u[(i + 1) & 3] : u[i]);
}
// a = rho^-1(R): a[i] = R[(i - k) & 3]
__device__ __forceinline__ void gh_rho_inv(const uint32_t R[4], const GhLane &g, uint32_t a[4]) {
    uint32_t u[4];
#pragma unroll
    for (int i = 0; i < 4; i++) u[i] = g.r1 ? R[(i + 3) & 3] : R[i];
#pragma unroll
    for (int i = 0; i < 4; i++) a[i] = g.r2 ? u[(i + 2) & 3] : u[i];
}

// One Horner step in the rotated frame: R <- rho(unrho(R) * H^64 ^ c)
__device__ __forceinline__ void ghash_step(const char *lds, uint32_t R[4], const GhLane &g, uint4 c) {
#if JFSX_GH8 == 4
    // four quarters of 4 lookups each: at most 16 VGPRs of table entries in flight
    uint32_t S[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int h = 0; h < 4; h++) {
        uint4 t[4];
#pragma unroll
        for (int q = 0; q < 4; q++) t[q] = lds_u4(lds, kLdsGh + __builtin_amdgcn_perm(R[h], g.off[h], g.sel[q]));
#define GX(f, i) S[i] = xor3(xor3(t[0].f, t[1].f, t[2].f), t[3].f, S[i])
        GX(x, 0); GX(y, 1); GX(z, 2); GX(w, 3);
#undef GX
        __builtin_amdgcn_sched_barrier(0);
    }
#elif JFSX_GH8
    // two halves of 8 lookups each: at most 32 VGPRs of table entries in flight
    uint32_t S[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
    for (int h = 0; h < 2; h++) {
        uint4 t[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const int dd = 2 * h + (q >> 2), bb = q & 3;
            t[q] = lds_u4(lds, kLdsGh + __builtin_amdgcn_perm(R[dd], g.off[dd], g.sel[bb]));
        }
#define GX(f, i) S[i] = xor3(xor3(t[0].f, t[1].f, t[2].f), xor3(t[3].f, t[4].f, t[5].f), xor3(t[6].f, t[7].f, S[i]))
        GX(x, 0); GX(y, 1); GX(z, 2); GX(w, 3);
#undef GX
        __builtin_amdgcn_sched_barrier(0);
    }
#else
    uint4 t[16];
#pragma unroll
    for (int dd = 0; dd < 4; dd++)
#pragma unroll
        for (int bb = 0; bb < 4; bb++)
            t[4 * dd + bb] = lds_u4(lds, kLdsGh + __builtin_amdgcn_perm(R[dd], g.off[dd], g.sel[bb]));
    // 16-way XOR as a 3-input tree (v_bitop3), then the new block
#define GX(f, cf) xor3(xor3(xor3(t[0].f, t[1].f, t[2].f), xor3(t[3].f, t[4].f, t[5].f), xor3(t[6].f, t[7].f, t[8].f)), \
                       xor3(t[9].f, t[10].f, t[11].f), xor3(xor3(t[12].f, t[13].f, t[14].f), t[15].f, cf))
    const uint32_t S[4] = {GX(x, c.x), GX(y, c.y), GX(z, c.z), GX(w, c.w)};
#undef GX
#endif
    gh_rho(S, g, R);
}

// Per-stream state of one wave: a contiguous, segment-aligned sub-chunk.
struct Stream {
    uint64_t sub0, sub1;  // byte range of the block
    uint32_t acc[4];      // GHASH lane accumulator, memory order, rotated by rho (see GhLane)
    uint64_t jlast;       // last 16-B block index folded into acc
    bool has;
    uint32_t A, lend;     // CRC lane accumulator, end of its last piece (segment relative)
    uint64_t seg0;        // start of the current segment
};

// CRC32C of segment [seg0, seg1) (seg1: its true end in the block) from this
// stream's lane accumulators A.  A lane's last piece in the segment ends at
// lend (segment relative), or, when lend == 0, at the end of its slot in the
// row that ends at tailRef (shift xl to the row end, then seg1 - tailRef more
// bytes).  When the stream covers only part of the segment (row-split tasks)
// the wave's raw share is XORed into the task's LDS slot and the CRC is
// finished once all waves are done (gcm_main_k's end); otherwise it is stored.
// the segment's raw share into the task's LDS slot (lane 0 only)
__device__ __forceinline__ void crc_share(char *lds, uint32_t slot, uint32_t raw) {
    atomicXor(reinterpret_cast<uint32_t *>(lds + kLdsSegRaw) + slot, raw);
    reinterpret_cast<uint32_t *>(lds + kLdsSegFlag)[slot] = 1u;
}

// Fast-loop form: a whole 32 KiB segment ended with the stream's row in its
// last row (every lane's last piece there): shift by xl, reduce, store -- or,
// when the stream began inside the segment, hand in the share.
template <int CRCMODE>
__device__ __forceinline__ void crc_segment_done(const BlkDev &blk, const DevTables &tab, uint32_t lane, uint32_t xl,
                                                 uint64_t seg0, uint32_t A, bool partial, char *lds, uint64_t c0) {
    const uint32_t raw = wave_xor(crc_mulmod(xl, A));
    if (lane == 0) {
        if (partial) {
            crc_share(lds, (uint32_t)((seg0 - c0) / kSeg), raw);
            return;
        }
        const uint32_t crc = ~(tab.crcx[96] ^ raw);
        const uint64_t si = seg0 / kSeg;
        if ((CRCMODE & 3) == 1)
            *reinterpret_cast<uint32_t *>(blk.crc + 4 * si) = __builtin_bswap32(crc);
        else
            blk.crc_calc[si] = crc;
    }
}

template <int CRCMODE>
__device__ __noinline__ void crc_segment_end(const BlkDev &blk, const DevTables &tab, uint32_t lane, uint32_t xl,
                                             uint64_t seg0, uint64_t seg1, uint32_t A, uint32_t lend,
                                             uint64_t tailRef, bool partial, char *lds, uint32_t slot) {
    const uint32_t Lseg = (uint32_t)(seg1 - seg0);
    uint32_t v;
    if (lend == 0) {
        const uint32_t sh = tailRef == seg1 ? xl : crc_mulmod(crc_xpow8_fast((uint32_t)(seg1 - tailRef), tab.crcx), xl);
        v = crc_mulmod(sh, A);
    } else {
        v = crc_mulmod(crc_xpow8_fast(Lseg - lend, tab.crcx), A);
    }
    const uint32_t raw = wave_xor(v);
    if (lane == 0) {
        if (partial) {
            crc_share(lds, slot, raw);
            return;
        }
        const uint32_t K = Lseg == (uint32_t)kSeg ? tab.crcx[96] : crc_mulmod(crc_xpow8_fast(Lseg, tab.crcx), 0xffffffffu);
        const uint32_t crc = ~(K ^ raw);
        const uint64_t si = seg0 / kSeg;
        if ((CRCMODE & 3) == 1)
            *reinterpret_cast<uint32_t *>(blk.crc + 4 * si) = __builtin_bswap32(crc);
        else
            blk.crc_calc[si] = crc;
    }
}

// Generic (guarded) processing of one row of one stream: handles the ragged
// tail of a block (partial 16-B piece, lanes past the end, partial segment).
template <bool OPEN, int CRCMODE>
__device__ __noinline__ Stream row_generic(char *lds, uint32_t loff, const GhLane gl, const GcmSched *sch,
                                           const BlkDev blk, const DevTables tab, uint32_t lane, uint32_t xl, Stream st,
                                           uint64_t row, uint64_t c0, uint64_t c1) {
    uint32_t rk[60];
#pragma unroll
    for (int i = 0; i < 60; i++) rk[i] = rk_load(sch->rk, i);
    const uint32_t k1[4] = {sch->k1[0], sch->k1[1], sch->k1[2], sch->k1[3]};
    const uint64_t o = row + 16 * lane;
    const uint64_t end = st.sub1;
    const bool valid = o < end, full = o + 16 <= end;
    uint4 d = load_piece(blk.src, o, end);
    const uint32_t ctr[1] = {(uint32_t)((o >> 4) + 2)};
    uint32_t ks[1][4];
    aes_ctr_blocks<1>(lds, loff, rk, k1, ctr, ks);
    uint4 x = make_uint4(d.x ^ ks[0][0], d.y ^ ks[0][1], d.z ^ ks[0][2], d.w ^ ks[0][3]);
    uint4 c = OPEN ? d : x, p = OPEN ? x : d;
    if (!full) {
        const int nv = valid ? (int)(end - o) : 0;
        uint32_t m[4];
        for (int k = 0; k < 4; k++) {
            int bytes = nv - 4 * k;
            m[k] = bytes >= 4 ? 0xffffffffu : (bytes <= 0 ? 0u : ((1u << (8 * bytes)) - 1u));
        }
        c.x &= m[0]; c.y &= m[1]; c.z &= m[2]; c.w &= m[3];
        p.x &= m[0]; p.y &= m[1]; p.z &= m[2]; p.w &= m[3];
    }
    if (valid) store_piece(blk.dst, o, end, OPEN ? p : c);
    uint32_t t[4] = {st.acc[0], st.acc[1], st.acc[2], st.acc[3]};
    ghash_step(lds, t, gl, c);
    if (valid) {
        st.acc[0] = t[0]; st.acc[1] = t[1]; st.acc[2] = t[2]; st.acc[3] = t[3];
        st.jlast = o >> 4;
        st.has = true;
    }
    const uint4 cq = crc_src<CRCMODE>(c, p);
    if (CRCMODE) {
        if (full) {
            st.A = crc_piece<kLdsCrc>(lds, st.A, cq.x, cq.y, cq.z, cq.w);
            st.lend = (uint32_t)(o + 16 - st.seg0);
        } else if (valid) {
            const uint32_t pw[4] = {cq.x, cq.y, cq.z, cq.w};
            st.A = crc_partial<kLdsCrc>(lds, st.A, pw, (int)(end - o));
            st.lend = (uint32_t)(end - st.seg0);
        }
        const uint64_t seg1 = st.seg0 + kSeg < c1 ? st.seg0 + kSeg : c1;  // the segment's true end
        if (row + 1024 >= seg1) {
            crc_segment_end<CRCMODE>(blk, tab, lane, xl, st.seg0, seg1, st.A, st.lend, row, st.seg0 < st.sub0, lds,
                                     (uint32_t)((st.seg0 - c0) / kSeg));
            st.A = 0;
            st.lend = 0;
            st.seg0 = seg1;
        }
    }
    return st;
}

// gcm_main: one workgroup per task; each wave runs NS streams in lock-step.
// BS = 0: T-table AES in LDS, 16 waves (4/SIMD, <= 128 VGPRs).
// BS = 1: whole 32 KiB segments use the bitsliced AES on the VALU
//         (jfsx_aes_bs.h; 128 VGPRs of state), 8 waves (2/SIMD, <= 256 VGPRs).
// BS = 2: hybrid, 8 waves of the BS = 1 shape: the last nbs waves run the
//         bitsliced AES on whole segments at the front of the task, the other
//         8 - nbs waves split the rest by rows with the T-table AES at a
//         raised priority, so the LDS pipe the T-table waves feed and the VALU
//         the bitsliced waves fill run at once (hyb below).
template <int BS>
struct GcmShape {
    static constexpr uint32_t waves = BS ? 8u : (uint32_t)kWaves;
    static constexpr uint32_t threads = waves * 64u;
};
// hybrid split (BS = 2), a kernel argument: bits 0..3 nbs (bitsliced waves),
// bits 8..15 rho = 16 x (bitsliced wave rate / T-table wave rate), bits 16..17
// the T-table waves' s_setprio level
__device__ __forceinline__ uint32_t hyb_nbs(uint32_t h) { return h & 15u; }
__device__ __forceinline__ uint32_t hyb_rho(uint32_t h) { return (h >> 8) & 255u; }

// JFSX_KS_PHASES probe build: the workgroup running block 0's first task
// stamps the 100 MHz clock at the main kernel's phase boundaries (g_main_ts:
// kernel start, tables staged, GHASH table built, rows done, epilogue done,
// task done); jfsx_debug_main_phases reads them back
#ifdef JFSX_KS_PHASES
__device__ unsigned long long g_main_ts[8];
#define MAIN_STAMP(cond, i)                                                                  \
    do {                                                                                     \
        __syncthreads();                                                                     \
        if ((cond) && threadIdx.x == 0) g_main_ts[i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define MAIN_STAMP(cond, i) ((void)0)
#endif

#ifdef JFSX_ABLATE_TRACE
// diagnostic build only (make variant V=TRACE): per workgroup start / end
// times (s_memrealtime, 100 MHz), HW_ID | XCC_ID << 32 and the task's bytes
__device__ uint64_t g_wgtrace[4 * 65536];
#endif

// One task (a block's <= 4 MiB byte range) on the whole workgroup.  The AES
// and CRC tables are already in LDS; the GHASH table of the task's key is
// built here.  Every thread of the workgroup calls this.
template <bool OPEN, int CRCMODE, int NS, int BS>
__device__ __forceinline__ void gcm_task(char *lds, const Task task, const BlkDev *__restrict__ blks,
                                         const GcmSched *__restrict__ sched, uint32_t *__restrict__ partial,
                                         uint32_t *__restrict__ pexp, const DevTables &tab, uint32_t tid,
                                         uint32_t wave, uint32_t lane, uint32_t loff, const GhLane &gl, uint32_t xl,
                                         uint32_t hyb) {
#ifdef JFSX_ABLATE_TRACE
    const uint64_t trace_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const BlkDev blk = blks[task.blk];
    const GcmSched *sch = sched + task.blk;
    if (tid < 128)
        reinterpret_cast<uint4 *>(lds + kLdsBasis)[tid] = reinterpret_cast<const uint4 *>(sch->basis)[tid];
    if (tid < 256) reinterpret_cast<uint32_t *>(lds + kLdsSegRaw)[tid] = 0u;  // raw shares and flags
    __syncthreads();
    {
        uint4 *lg = reinterpret_cast<uint4 *>(lds + kLdsGh);
        const uint4 *lb = reinterpret_cast<const uint4 *>(lds + kLdsBasis);
#ifdef JFSX_ABLATE_GHBUILD
        if (false)  // timing experiment only: wrong tags
#endif
        // entry (b, j) at byte (b << 8) | (j << 4) is the XOR of basis[8j + k]
        // over the set bits 7 - k of b: a thread shares the six low bits' sum
        // across the four entries that differ only in bits 7..6
        for (uint32_t u = tid; u < 1024; u += GcmShape<BS>::threads) {
            const uint32_t j = u & 15, blow = u >> 4;
            uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int k = 2; k < 8; k++) {
                if ((blow >> (7 - k)) & 1) {
                    const uint4 v = lb[8 * j + k];
                    z.x ^= v.x; z.y ^= v.y; z.z ^= v.z; z.w ^= v.w;
                }
            }
            const uint4 h0 = lb[8 * j], h1 = lb[8 * j + 1];
            lg[(blow << 4) | j] = z;
            lg[((blow | 64) << 4) | j] = make_uint4(z.x ^ h1.x, z.y ^ h1.y, z.z ^ h1.z, z.w ^ h1.w);
            lg[((blow | 128) << 4) | j] = make_uint4(z.x ^ h0.x, z.y ^ h0.y, z.z ^ h0.z, z.w ^ h0.w);
            lg[((blow | 192) << 4) | j] =
                make_uint4(z.x ^ h0.x ^ h1.x, z.y ^ h0.y ^ h1.y, z.z ^ h0.z ^ h1.z, z.w ^ h0.w ^ h1.w);
        }
    }
    __syncthreads();

    const bool first_task = task.blk == 0 && task.c0 == 0;
    MAIN_STAMP(first_task, 2);
    const uint64_t c0 = task.c0, c1 = task.c1;
    const uint32_t nseg = (uint32_t)((c1 - c0 + kSeg - 1) / kSeg);
    constexpr uint32_t V = GcmShape<BS>::waves * NS;  // virtual waves (streams) per task

    // Row split (T-table kernel, one stream per wave): the task's rows are cut
    // into 16 contiguous runs of equal length, so a task of any size keeps
    // every wave busy (a 64 KiB block has 2 segments: with whole segments per
    // wave 14 of 16 waves would idle).  A segment shared by two waves gets its
    // CRC from both waves' raw shares (crc_segment_end, task end below).  The
    // bitsliced kernel keys whole 32 KiB segments and keeps the segment split.
    constexpr bool kRowSplit = !BS && NS == 1;
    // segments shared by two waves' row ranges (their CRC from raw shares)
    constexpr bool kShares = kRowSplit || (BS == 2 && NS == 1);
    // hybrid: waves [nt, 8) are bitsliced and take q whole segments each from
    // the front of the task; waves [0, nt) row-split the rest
    const uint32_t nbs = BS == 2 ? hyb_nbs(hyb) : 0u, nt = GcmShape<BS>::waves - nbs;
    const bool isbs = BS == 1 || (BS == 2 && wave >= nt);
    uint32_t q = 0;
    if (BS == 2 && nbs) {
        const uint32_t rho = hyb_rho(hyb), whole = (uint32_t)((c1 - c0) / kSeg);
        q = nseg * rho / (nbs * rho + nt * 16u);
        if (nbs * q > whole) q = whole / nbs;
    }
    const uint64_t tt0 = c0 + (uint64_t)nbs * q * kSeg;  // the T-table waves' region [tt0, c1)
    // in pairs of rows: every stream starts on an even row, as the two-row
    // loop's segment-end test assumes (only its second row can end a segment)
    const uint32_t npairs = (uint32_t)((c1 - c0 + 2047) / 2048);
    Stream st[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const uint32_t v = wave * NS + s;
        if (BS == 2 && isbs) {
            st[s].sub0 = c0 + (uint64_t)(wave - nt) * q * kSeg;
            st[s].sub1 = st[s].sub0 + (uint64_t)q * kSeg;
        } else if (BS == 2) {
            // groups of JFSX_HYB_UR rows (a divisor of 32): every stream starts
            // on a multiple of UR rows, so only the last row of a UR block can
            // end a segment
            constexpr uint32_t G = JFSX_HYB_UR;
            const uint32_t ng = (uint32_t)((c1 - tt0 + 1024 * G - 1) / (1024 * G));
            const uint32_t ra = G * (wave * ng / nt), rb = G * ((wave + 1) * ng / nt);
            st[s].sub0 = tt0 + (uint64_t)ra * 1024;
            st[s].sub1 = rb > ra ? (tt0 + (uint64_t)rb * 1024 < c1 ? tt0 + (uint64_t)rb * 1024 : c1) : st[s].sub0;
        } else if (kRowSplit) {
            const uint32_t ra = 2 * (v * npairs / V), rb = 2 * ((v + 1) * npairs / V);
            st[s].sub0 = c0 + (uint64_t)ra * 1024;
            st[s].sub1 = rb > ra ? (c0 + (uint64_t)rb * 1024 < c1 ? c0 + (uint64_t)rb * 1024 : c1) : st[s].sub0;
        } else {
            const uint32_t sa = v * nseg / V, sb = (v + 1) * nseg / V;
            st[s].sub0 = c0 + (uint64_t)sa * kSeg;
            st[s].sub1 = sb > sa ? (c0 + (uint64_t)sb * kSeg < c1 ? c0 + (uint64_t)sb * kSeg : c1) : st[s].sub0;
        }
        st[s].acc[0] = st[s].acc[1] = st[s].acc[2] = st[s].acc[3] = 0;
        st[s].jlast = 0;
        st[s].has = false;
        st[s].A = 0;
        st[s].lend = 0;
        st[s].seg0 = c0 + (st[s].sub0 - c0) / kSeg * kSeg;  // start of the segment holding the stream's first row
    }
    // rows that are full for every non-empty stream: the fast path.  Empty
    // streams (tasks with fewer segments than streams) alias stream 0's loads
    // and skip every side effect (wave-uniform branch).
    bool act[NS];
    uint64_t rf = ~0ull, ld0[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        act[s] = st[s].sub1 > st[s].sub0;
        ld0[s] = act[s] ? st[s].sub0 : st[0].sub0;
        if (act[s]) {
            const uint64_t fr = (st[s].sub1 - st[s].sub0) / 1024;
            rf = fr < rf ? fr : rf;
        }
    }
    if (rf == ~0ull) rf = 0;
    const uint8_t *src = blk.src;
    uint8_t *dst = blk.dst;
    const uint64_t lo = 16 * lane;

    uint64_t r0 = 0;
    // BS: whole 32 KiB segments take their 32 rows of keystream from one
    // bitsliced AES pass (lane slot k = row k), then the rows stream through
    // XOR / store / GHASH / CRC with the keystream in registers.
    if (BS && isbs && NS == 1 && act[0] && rf >= 32) {
        const uint64_t nfs = rf / 32;
        const uint32_t nrk[3] = {sch->c012[0], sch->c012[1], sch->c012[2]};
        const uint32_t rk3 = sch->rk[3];
        constexpr int PF = 4;  // rows of loads in flight
        uint4 pf[PF];
#pragma unroll
        for (int q = 0; q < PF; q++) pf[q] = ald16(src + ld0[0] + 1024 * q + lo);
        for (uint64_t sg = 0; sg < nfs; sg++) {
            const uint64_t base = ld0[0] + (uint64_t)kSeg * sg;
            uint32_t ks[128];
            jfsx_bs::ctr32(ks, nrk, rk3, (uint32_t)((base >> 4) + lane + 2),
                           [&](int r, int w) { return sch->bsu[r][w]; }, sch->r1c);
            const bool more = sg + 1 < nfs;
#pragma unroll
            for (int k = 0; k < 32; k++) {
                const uint4 d = pf[k % PF];
                const uint64_t o = base + 1024 * k + lo;
                if (k + PF < 32 || more) pf[k % PF] = ald16(src + o + 1024 * PF);
                const uint4 x = make_uint4(d.x ^ ks[k], d.y ^ ks[32 + k], d.z ^ ks[64 + k], d.w ^ ks[96 + k]);
                const uint4 c = OPEN ? d : x, p = OPEN ? x : d;
                ast16(dst + o, OPEN ? p : c);
                const uint4 cq = crc_src<CRCMODE>(c, p);
#ifndef JFSX_ABLATE_GHASH
                ghash_step(lds, st[0].acc, gl, c);
#endif
                if (CRCMODE) st[0].A = crc_piece<kLdsCrc>(lds, st[0].A, cq.x, cq.y, cq.z, cq.w);
            }
            if (CRCMODE) {
                crc_segment_done<CRCMODE>(blk, tab, lane, xl, st[0].seg0, st[0].A, false, lds, c0);
                st[0].A = 0;
                st[0].seg0 += kSeg;
            }
        }
        r0 = 32 * nfs;
    }
    // T-table AES (LDS) for the rows outside whole segments; the schedule is
    // read here, after the bitsliced loop, so it holds no SGPRs through it
    uint32_t rk[60];
#pragma unroll
    for (int i = 0; i < 60; i++) rk[i] = rk_load(sch->rk, i);
    uint32_t k1[4] = {sch->k1[0], sch->k1[1], sch->k1[2], sch->k1[3]};
    uint4 nxt[NS];
#pragma unroll
    for (int s = 0; s < NS; s++)
        nxt[s] = r0 < rf ? ald16(src + ld0[s] + 1024 * r0 + lo) : make_uint4(0, 0, 0, 0);
#if JFSX_U2
    // UR rows of one stream per iteration (2 in the 16-wave shape; the 8-wave
    // shape has twice the VGPRs and takes JFSX_HYB_UR): the UR AES chains
    // interleave, GHASH/CRC stay sequential (register peak of one row)
    constexpr int UR = BS == 2 ? JFSX_HYB_UR : JFSX_UR0;
    if (NS == 1 && act[0] && rf >= r0 + UR) {
        uint4 nn[UR];
#pragma unroll
        for (int u = 0; u < UR; u++) nn[u] = ald16(src + ld0[0] + 1024 * (r0 + u) + lo);
#if JFSX_UCTR
        uint32_t uw[4] = {0, 0, 0, 0};
        uint32_t uw0 = 0;
        bool uwok = false;
#endif
        // task row index of the stream's first row: a multiple of 2 (16-wave
        // shape, row pairs) or of UR (8-wave shape), so the compiler drops the
        // segment-end test of rows that cannot end a segment
        constexpr uint32_t RA = BS == 2 ? (32 % UR == 0 ? (uint32_t)UR : 1u) : 2u;
        const uint32_t rb0 = (uint32_t)((ld0[0] - c0) >> 10) / RA * RA;
        // software pipelining (8-wave shape, JFSX_HYB_SWP): the GHASH and CRC
        // lookups of UR block i - 1 share a basic block with the AES of block
        // i (independent LDS work to fill the rounds' latency); its segment
        // end, if any, is handled after block i's stores
        constexpr bool SWP = BS == 2 && JFSX_HYB_SWP;
        static_assert(!SWP || 32 % UR == 0, "software pipelining needs UR | 32");
        uint4 pc[UR], pq[UR];
        bool pend = false;
        uint32_t pr0 = 0;
        for (; r0 + UR - 1 < rf; r0 += UR) {
            uint4 dd[UR];
#pragma unroll
            for (int u = 0; u < UR; u++) dd[u] = nn[u];
            const uint64_t o0 = ld0[0] + 1024 * r0 + lo;
            if (r0 + 2 * UR - 1 < rf) {
#pragma unroll
                for (int u = 0; u < UR; u++) nn[u] = ald16(src + o0 + 1024 * (UR + u));
            }
            if (SWP && pend) {
#pragma unroll
                for (int u = 0; u < UR; u++) {
#ifndef JFSX_ABLATE_GHASH
                    ghash_step(lds, st[0].acc, gl, pc[u]);
#endif
                    if (CRCMODE) st[0].A = crc_piece<kLdsCrc>(lds, st[0].A, pq[u].x, pq[u].y, pq[u].z, pq[u].w);
                }
            }
            uint32_t ctrs[UR];
#pragma unroll
            for (int u = 0; u < UR; u++) ctrs[u] = (uint32_t)((o0 >> 4) + 2 + 64 * u);
            uint32_t ks2[UR][4];
#if JFSX_UCTR
            {
                // row counters C + 64 u (C = the first row's lane-0 counter, wave-uniform)
                uint32_t C = (uint32_t)(((ld0[0] + 1024 * r0) >> 4) + 2);
                OPAQUE(C);
                // the window must hold U(C) .. U(C + 64 UR - 1 + 1)
                if (!uwok || (C >> 8) < uw0 || ((C + 64u * UR + 63u) >> 8) - uw0 > 63u) {
                    uw0 = C >> 8;
                    aes_r2_uniform(lds, loff, rk, k1, uw0 + lane, uw);
                    uwok = true;
                }
                uint32_t u2[UR][4], d2[UR][4], cym[UR];
#pragma unroll
                for (int u = 0; u < UR; u++) {
                    const uint32_t Cr = C + 64u * u;
                    const uint32_t i0 = (Cr >> 8) - uw0;
                    // ~0 on the lanes whose counter carried into U + 1, else 0
                    cym[u] = (uint32_t)__builtin_amdgcn_sbfe((int)((Cr & 255u) + lane), 8, 1);
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        u2[u][k] = __builtin_amdgcn_readlane(uw[k], i0);
                        d2[u][k] = u2[u][k] ^ __builtin_amdgcn_readlane(uw[k], i0 + 1);
                    }
                }
                aes_ctr_blocks_u<UR>(lds, loff, rk, k1, ctrs, u2, d2, cym, ks2);
            }
#else
            aes_ctr_blocks<UR>(lds, loff, rk, k1, ctrs, ks2);
#endif
#pragma unroll
            for (int u = 0; u < UR; u++) {
                const uint64_t o = o0 + 1024 * u;
#if JFSX_UCTR
                // data ^ keystream ^ last round key in one v_bitop3
                const uint4 x = make_uint4(xor3(dd[u].x, ks2[u][0], rk[56]), xor3(dd[u].y, ks2[u][1], rk[57]),
                                           xor3(dd[u].z, ks2[u][2], rk[58]), xor3(dd[u].w, ks2[u][3], rk[59]));
#else
                const uint4 x = make_uint4(dd[u].x ^ ks2[u][0], dd[u].y ^ ks2[u][1], dd[u].z ^ ks2[u][2],
                                           dd[u].w ^ ks2[u][3]);
#endif
                const uint4 c = OPEN ? dd[u] : x, p = OPEN ? x : dd[u];
                ast16(dst + o, OPEN ? p : c);
                const uint4 cq = crc_src<CRCMODE>(c, p);
                if (SWP) {
                    pc[u] = c;
                    pq[u] = cq;
                    continue;
                }
#ifndef JFSX_ABLATE_GHASH
                ghash_step(lds, st[0].acc, gl, c);
#endif
                if (CRCMODE) st[0].A = crc_piece<kLdsCrc>(lds, st[0].A, cq.x, cq.y, cq.z, cq.w);
                if (CRCMODE && ((rb0 + (uint32_t)r0 + u) & 31) == 31) {
                    crc_segment_done<CRCMODE>(blk, tab, lane, xl, st[0].seg0, st[0].A, st[0].seg0 < st[0].sub0, lds,
                                              c0);
                    st[0].A = 0;
                    st[0].seg0 += kSeg;
                }
            }
            if (SWP) {
                // the previous block's segment end (its CRC went in above)
                if (CRCMODE && pend && ((rb0 + pr0 + UR - 1) & 31) == 31) {
                    crc_segment_done<CRCMODE>(blk, tab, lane, xl, st[0].seg0, st[0].A, st[0].seg0 < st[0].sub0, lds,
                                              c0);
                    st[0].A = 0;
                    st[0].seg0 += kSeg;
                }
                pend = true;
                pr0 = (uint32_t)r0;
            }
        }
        if (SWP && pend) {
#pragma unroll
            for (int u = 0; u < UR; u++) {
#ifndef JFSX_ABLATE_GHASH
                ghash_step(lds, st[0].acc, gl, pc[u]);
#endif
                if (CRCMODE) st[0].A = crc_piece<kLdsCrc>(lds, st[0].A, pq[u].x, pq[u].y, pq[u].z, pq[u].w);
            }
            if (CRCMODE && ((rb0 + pr0 + UR - 1) & 31) == 31) {
                crc_segment_done<CRCMODE>(blk, tab, lane, xl, st[0].seg0, st[0].A, st[0].seg0 < st[0].sub0, lds, c0);
                st[0].A = 0;
                st[0].seg0 += kSeg;
            }
        }
        if (r0 < rf) nxt[0] = ald16(src + ld0[0] + 1024 * r0 + lo);
    }
#endif
    for (uint64_t r = r0; r < rf; r++) {
        uint4 d[NS];
        uint32_t ctr[NS];
#pragma unroll
        for (int s = 0; s < NS; s++) {
            d[s] = nxt[s];
            const uint64_t o = ld0[s] + 1024 * r + lo;
            if (r + 1 < rf) nxt[s] = ald16(src + o + 1024);
            ctr[s] = (uint32_t)((o >> 4) + 2);
        }
        uint32_t ks[NS][4];
        aes_ctr_blocks<NS>(lds, loff, rk, k1, ctr, ks);
#pragma unroll
        for (int s = 0; s < NS; s++) {
            if (!act[s]) continue;
            const uint64_t o = st[s].sub0 + 1024 * r + lo;
            const uint4 x = make_uint4(d[s].x ^ ks[s][0], d[s].y ^ ks[s][1], d[s].z ^ ks[s][2], d[s].w ^ ks[s][3]);
            const uint4 c = OPEN ? d[s] : x, p = OPEN ? x : d[s];
            ast16(dst + o, OPEN ? p : c);
            const uint4 cq = crc_src<CRCMODE>(c, p);
            ghash_step(lds, st[s].acc, gl, c);
            if (CRCMODE) st[s].A = crc_piece<kLdsCrc>(lds, st[s].A, cq.x, cq.y, cq.z, cq.w);
        }
        if (CRCMODE && ((uint32_t)((ld0[0] - c0) >> 10) + (uint32_t)r & 31) == 31) {
            // (NS > 1 only with the segment split: every stream starts on a segment)
#pragma unroll
            for (int s = 0; s < NS; s++) {
                if (!act[s]) continue;
                crc_segment_done<CRCMODE>(blk, tab, lane, xl, st[s].seg0, st[s].A, st[s].seg0 < st[s].sub0, lds, c0);
                st[s].A = 0;
                st[s].seg0 += kSeg;
            }
        }
    }
#pragma unroll
    for (int s = 0; s < NS; s++) {
        if (rf && act[s]) {
            st[s].has = true;
            st[s].jlast = (st[s].sub0 + 1024 * (rf - 1) + lo) >> 4;
        }
        // lanes whose last piece lies in the last full row: their CRC shift to
        // a segment end starts at that row's end (lend == 0, crc_segment_end)
        const uint64_t tailRef = st[s].sub0 + 1024 * rf;
        // ragged remainder of this stream (block tail or unequal streams)
        for (uint64_t row = tailRef; row < st[s].sub1; row += 1024)
            st[s] = row_generic<OPEN, CRCMODE>(lds, loff, gl, sch, blk, tab, lane, xl, st[s], row, c0, c1);
        // a stream that ended inside a segment still owes that segment's CRC
        // (or, when another wave holds the rest of the segment, its share)
        if (CRCMODE && act[s] && st[s].seg0 < st[s].sub1) {
            const uint64_t seg1 = st[s].seg0 + kSeg < c1 ? st[s].seg0 + kSeg : c1;
            crc_segment_end<CRCMODE>(blk, tab, lane, xl, st[s].seg0, seg1, st[s].A, st[s].lend, tailRef,
                                     st[s].seg0 < st[s].sub0 || st[s].sub1 < seg1, lds,
                                     (uint32_t)((st[s].seg0 - c0) / kSeg));
            st[s].seg0 = st[s].sub1;
        }
    }

    MAIN_STAMP(first_task, 3);
    // ---- stream epilogues: lift lane accumulators to the stream end, reduce ----
    const uint64_t nblk = (blk.len + 15) >> 4;
#pragma unroll
    for (int s = 0; s < NS; s++) {
        const uint64_t wend = (st[s].sub1 + 15) >> 4;  // blocks before the stream end
        g128 z = {{0, 0, 0, 0}};
        if (st[s].has && st[s].sub1 > st[s].sub0) {
            const uint32_t e = (uint32_t)(wend + 1 - st[s].jlast);  // in [2, 65]
            uint32_t a[4];
            gh_rho_inv(st[s].acc, gl, a);
#ifdef JFSX_ABLATE_LIFT
            z = g_from_mem(a);  // timing experiment only: wrong tags
#else
            z = JFSX_GF_CT_LIFT ? g_mul_ct_call(g_from_mem(a), g_from_mem(sch->hpow[e]))
                                : g_mul(g_from_mem(a), g_from_mem(sch->hpow[e]));
#endif
        }
        uint32_t zm[4];
        g_to_mem(z, zm);
        for (int k = 0; k < 4; k++) zm[k] = wave_xor(zm[k]);
        if (lane == 0) {
            const uint32_t slot = task.slot0 + wave * NS + s;
            partial[4 * slot + 0] = zm[0];
            partial[4 * slot + 1] = zm[1];
            partial[4 * slot + 2] = zm[2];
            partial[4 * slot + 3] = zm[3];
            pexp[slot] = (uint32_t)(nblk - wend);
            // the 8-wave bitsliced shape leaves the upper half of the task's
            // kSlotsPerTask slots unused: zero them for gcm_finalize
            for (uint32_t u = task.slot0 + GcmShape<BS>::waves * NS + wave * NS + s; u < task.slot0 + kSlotsPerTask;
                 u += GcmShape<BS>::waves * NS) {
                partial[4 * u + 0] = partial[4 * u + 1] = partial[4 * u + 2] = partial[4 * u + 3] = 0;
                pexp[u] = 0;
            }
        }
    }

#ifdef JFSX_ABLATE_TRACE
    __syncthreads();
    if (tid == 0 && task.trace < 65536) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_wgtrace[4 * task.trace + 0] = trace_t0;
        g_wgtrace[4 * task.trace + 1] = __builtin_amdgcn_s_memrealtime();
        g_wgtrace[4 * task.trace + 2] = hw | ((uint64_t)xcc << 32);
        g_wgtrace[4 * task.trace + 3] = task.c1 - task.c0;
    }
#endif
    MAIN_STAMP(first_task, 4);
    // ---- segments shared by two or more waves: sum the raw shares, finish ----
    if (CRCMODE && kShares) {
        __syncthreads();
        if (wave == 0) {
            const uint32_t *raw = reinterpret_cast<const uint32_t *>(lds + kLdsSegRaw);
            const uint32_t *flag = reinterpret_cast<const uint32_t *>(lds + kLdsSegFlag);
            for (uint32_t k = lane; k < nseg; k += 64) {
                if (!flag[k]) continue;
                const uint64_t s0 = c0 + (uint64_t)k * kSeg;
                const uint32_t Lseg = (uint32_t)((s0 + kSeg < c1 ? s0 + kSeg : c1) - s0);
                const uint32_t K = Lseg == (uint32_t)kSeg ? tab.crcx[96]
                                                          : crc_mulmod(crc_xpow8_fast(Lseg, tab.crcx), 0xffffffffu);
                const uint32_t crc = ~(K ^ raw[k]);
                const uint64_t si = s0 / kSeg;
                if ((CRCMODE & 3) == 1)
                    *reinterpret_cast<uint32_t *>(blk.crc + 4 * si) = __builtin_bswap32(crc);
                else
                    blk.crc_calc[si] = crc;
            }
        }
    }
    MAIN_STAMP(first_task, 5);
}

// gcm_main: persistent workgroups, one per CU (the LDS tables allow one),
// taking tasks from a queue until it is empty.  The AES and CRC tables are
// staged once per workgroup.  Tasks come largest first (the host sorts them),
// so the queue's tail is made of small tasks.  A grid of one workgroup per
// task would leave CUs idle between tasks of mixed sizes: workgroups are
// dispatched in order, round-robin over the XCDs, and the next one waits for
// a CU of its own XCD (measured with the TRACE variant on configs[4]'s
// 64 KiB-4 MiB blocks: CUs 79 % busy, 115 us mean gap between tasks).
template <bool OPEN, int CRCMODE, int NS, int BS>
__global__ __launch_bounds__(GcmShape<BS>::threads) void gcm_main_k(const Task *__restrict__ tasks, uint32_t ntasks,
                                                       uint32_t *__restrict__ queue,
                                                       const BlkDev *__restrict__ blks,
                                                       const GcmSched *__restrict__ sched,
                                                       uint32_t *__restrict__ partial, uint32_t *__restrict__ pexp,
                                                       DevTables tab, uint32_t hyb) {
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    __shared__ uint32_t s_task;
    const uint32_t tid = threadIdx.x;
#ifdef JFSX_KS_PHASES
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
#endif
    {
        const uint4 *ga = reinterpret_cast<const uint4 *>(tab.aes);
        uint4 *la = reinterpret_cast<uint4 *>(lds + kLdsAes);
        for (uint32_t i = tid; i < 4096; i += GcmShape<BS>::threads) la[i] = ga[i];
        if (CRCMODE) {
            const uint4 *gc = reinterpret_cast<const uint4 *>(tab.crc);
            uint4 *lc = reinterpret_cast<uint4 *>(lds + kLdsCrc);
            for (uint32_t i = tid; i < 1280; i += GcmShape<BS>::threads) lc[i] = gc[i];
        }
    }
#ifdef JFSX_KS_PHASES
    __syncthreads();
    const unsigned long long t_staged = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && tasks[0].blk == 0 && blockIdx.x == 0) {  // the WG that is likely to pop task 0
        g_main_ts[0] = t_start;
        g_main_ts[1] = t_staged;
    }
#endif
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;  // wave index in an SGPR
    const uint32_t loff = ((lane & 31) << 2) | 0x00010000u;  // AES replica offset | table base
    const GhLane gl = gh_lane(lane);
    const uint32_t xl = CRCMODE ? tab.crcx[lane] : 0u;
    if (BS == 2 && wave < GcmShape<BS>::waves - hyb_nbs(hyb)) {
        // the T-table waves win VALU arbitration against the bitsliced ones
        switch ((hyb >> 16) & 3u) {
            case 1: __builtin_amdgcn_s_setprio(1); break;
            case 2: __builtin_amdgcn_s_setprio(2); break;
            case 3: __builtin_amdgcn_s_setprio(3); break;
            default: break;
        }
    }
    if (tid == 0) s_task = atomicAdd(queue, 1u);
    for (;;) {
        // also orders this task's table writes after the previous task's readers
        __syncthreads();
        const uint32_t ti = __builtin_amdgcn_readfirstlane(s_task);
        if (ti >= ntasks) break;  // the same for every wave: the queue is exhausted
        __syncthreads();          // every wave holds ti: s_task may take the next index
        if (tid == 0) s_task = atomicAdd(queue, 1u);  // the next task's index arrives during this one
        gcm_task<OPEN, CRCMODE, NS, BS>(lds, tasks[ti], blks, sched, partial, pexp, tab, tid, wave, lane, loff, gl,
                                        xl, hyb);
    }
}

// ---------------------------------------------------------------------------
// keysetup: one wave per block; AES via the (global) T-table image
// ---------------------------------------------------------------------------
// keysetup's lookups go to a compact copy of T0 | T2 staged in LDS (entry x
// at 2x, 2x + 1): every lane looks up the same index (a broadcast), and a
// dependent chain of LDS reads costs a fraction of the same chain through L2
__device__ __forceinline__ uint32_t gT0(const uint32_t *aes, uint32_t x) { return aes[2 * x]; }
__device__ __forceinline__ uint32_t gT2(const uint32_t *aes, uint32_t x) { return aes[2 * x + 1]; }
__device__ __forceinline__ uint32_t gS(const uint32_t *aes, uint32_t x) { return (aes[2 * x] >> 8) & 0xffu; }

__device__ uint32_t gcol(const uint32_t *aes, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return gT0(aes, a & 0xff) ^ rotl8(gT0(aes, (b >> 8) & 0xff)) ^ gT2(aes, (c >> 16) & 0xff) ^
           rotl8(gT2(aes, d >> 24));
}

// rk: the schedule in LDS (broadcast reads); the state stays in registers
__device__ void aes_enc_global(const uint32_t *aes, const uint32_t *rk, const uint32_t in[4], uint32_t out[4]) {
    uint32_t s[4], t[4];
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = in[c] ^ rk[c];
    for (int r = 1; r < 14; r++) {
#pragma unroll
        for (int c = 0; c < 4; c++) t[c] = gcol(aes, s[c], s[(c + 1) & 3], s[(c + 2) & 3], s[(c + 3) & 3]) ^ rk[4 * r + c];
#pragma unroll
        for (int c = 0; c < 4; c++) s[c] = t[c];
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t a = s[c], b = s[(c + 1) & 3], cc = s[(c + 2) & 3], d = s[(c + 3) & 3];
        out[c] = (gS(aes, a & 0xff) | (gS(aes, (b >> 8) & 0xff) << 8) | (gS(aes, (cc >> 16) & 0xff) << 16) |
                  (gS(aes, d >> 24) << 24)) ^ rk[56 + c];
    }
}

// z = x * y in GF(2^128) for a wave-uniform y and a per-lane x, four bits of
// x per step (Horner from the high coefficients: z = z x^4 + y N_t), the 16
// multiples y (n3 + n2 x + n1 x^2 + n0 x^3) in LDS.  About 600 instructions
// against g_mul's 2000; every lane of the wave must call it (barriers).
// JFSX_GF_CT (default 1): keysetup's and finalize's GF products by
// integer multiplies (g_mul_ct, jfsx_gf.h) instead of LDS nibble tables
#ifndef JFSX_GF_CT
#define JFSX_GF_CT 1
#endif
#ifndef JFSX_KS_NIB
#define JFSX_KS_NIB 1  // 0: keysetup with the bit-serial g_mul (A/B)
#endif
__device__ __forceinline__ g128 g_mul_uy(const g128 &x, const g128 &y, uint4 *M, uint32_t lane) {
    const g128 y1 = g_mulx(y), y2 = g_mulx(y1), y3 = g_mulx(y2);
    __syncthreads();  // the previous call's readers are done with M
    if (lane < 16) {
        uint32_t m[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            m[k] = ((lane & 8) ? y.w[k] : 0u) ^ ((lane & 4) ? y1.w[k] : 0u) ^ ((lane & 2) ? y2.w[k] : 0u) ^
                   ((lane & 1) ? y3.w[k] : 0u);
        M[lane] = make_uint4(m[0], m[1], m[2], m[3]);
    }
    __syncthreads();
    g128 z = {{0, 0, 0, 0}};
#pragma unroll 4
    for (int t = 31; t >= 0; t--) {
        // z x^4: the four coefficients shifted out (low bits of w[3]) fold
        // back as in four g_mulx steps
        const uint32_t sh = z.w[3] & 15u;
        z.w[3] = __builtin_amdgcn_alignbit(z.w[2], z.w[3], 4);
        z.w[2] = __builtin_amdgcn_alignbit(z.w[1], z.w[2], 4);
        z.w[1] = __builtin_amdgcn_alignbit(z.w[0], z.w[1], 4);
        z.w[0] = (z.w[0] >> 4) ^ ((sh & 1u) ? 0xE1000000u >> 3 : 0u) ^ ((sh & 2u) ? 0xE1000000u >> 2 : 0u) ^
                 ((sh & 4u) ? 0xE1000000u >> 1 : 0u) ^ ((sh & 8u) ? 0xE1000000u : 0u);
        const uint32_t n = (x.w[t >> 3] >> (28 - 4 * (t & 7))) & 15u;
        const uint4 mv = M[n];
        z.w[0] ^= mv.x, z.w[1] ^= mv.y, z.w[2] ^= mv.z, z.w[3] ^= mv.w;
    }
    return z;
}

// g_mul_uy for a one-wave kernel (keysetup): the 32 table rows x selects are
// loaded before the Horner chain starts (they depend on x alone), so the
// chain is VALU work only instead of one dependent LDS round trip per step.
// Holds the rows in 128 VGPRs -- fine in keysetup's 64-thread workgroup, not
// in the 1024-thread finalize, which keeps g_mul_uy.
__device__ __forceinline__ g128 g_mul_uy_pre(const g128 &x, const g128 &y, uint4 *M, uint32_t lane) {
    const g128 y1 = g_mulx(y), y2 = g_mulx(y1), y3 = g_mulx(y2);
    __syncthreads();  // the previous call's readers are done with M
    if (lane < 16) {
        uint32_t m[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            m[k] = ((lane & 8) ? y.w[k] : 0u) ^ ((lane & 4) ? y1.w[k] : 0u) ^ ((lane & 2) ? y2.w[k] : 0u) ^
                   ((lane & 1) ? y3.w[k] : 0u);
        M[lane] = make_uint4(m[0], m[1], m[2], m[3]);
    }
    __syncthreads();
    uint4 mv[32];
#pragma unroll
    for (int t = 0; t < 32; t++) mv[t] = M[(x.w[t >> 3] >> (28 - 4 * (t & 7))) & 15u];
    g128 z = {{0, 0, 0, 0}};
#pragma unroll
    for (int t = 31; t >= 0; t--) {
        const uint32_t sh = z.w[3] & 15u;
        z.w[3] = __builtin_amdgcn_alignbit(z.w[2], z.w[3], 4);
        z.w[2] = __builtin_amdgcn_alignbit(z.w[1], z.w[2], 4);
        z.w[1] = __builtin_amdgcn_alignbit(z.w[0], z.w[1], 4);
        z.w[0] = (z.w[0] >> 4) ^ ((sh & 1u) ? 0xE1000000u >> 3 : 0u) ^ ((sh & 2u) ? 0xE1000000u >> 2 : 0u) ^
                 ((sh & 4u) ? 0xE1000000u >> 1 : 0u) ^ ((sh & 8u) ? 0xE1000000u : 0u);
        z.w[0] ^= mv[t].x, z.w[1] ^= mv[t].y, z.w[2] ^= mv[t].z, z.w[3] ^= mv[t].w;
    }
    return z;
}

// JFSX_KS_PHASES (a probe build, scripts/build_variant.sh): workgroup 0 of
// each keysetup launch stamps the constant 100 MHz clock at its phase
// boundaries into g_ks_ts; jfsx_debug_ks_phases reads them back
#ifdef JFSX_KS_PHASES
__device__ unsigned long long g_ks_ts[16];
#define KS_STAMP(i)                                                          \
    do {                                                                     \
        __syncthreads();                                                     \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_ks_ts[i] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define KS_STAMP(i) ((void)0)
#endif

// x^S * v in one step for a static S in 1..64 (S g_mulx steps at once): in
// this bit order a product by x^S rotates the 128-bit register W0..W3 right
// by S, and the S coefficients that wrapped to the top (T) reduce by
// x^128 = 1 + x + x^2 + x^7: add T >> 1, T >> 2 and T >> 7 (nothing of T
// leaves the register for S <= 64, so one fold suffices)
template <int S>
__device__ __forceinline__ g128 g_mulxs(g128 v) {
    constexpr int q = S / 32, r = S % 32;
    uint32_t a[4], b[4], t[4];
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = v.w[(k - q + 4) & 3];
#pragma unroll
    for (int k = 0; k < 4; k++) b[k] = r ? __builtin_amdgcn_alignbit(a[(k + 3) & 3], a[k], r) : a[k];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int top = S - 32 * k;  // bits of T in word k
        t[k] = top >= 32 ? b[k] : top > 0 ? b[k] & ~(0xffffffffu >> top) : 0u;
    }
    g128 z;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t p = k ? t[k - 1] : 0u;
        z.w[k] = b[k] ^ __builtin_amdgcn_alignbit(p, t[k], 1) ^ __builtin_amdgcn_alignbit(p, t[k], 2) ^
                 __builtin_amdgcn_alignbit(p, t[k], 7);
    }
    return z;
}

// x^i * v for a per-lane i < 128: the products by x^(2^k) of i's set bits,
// each taken by select (no divergence)
__device__ __forceinline__ g128 g_mul_xpow(g128 v, uint32_t i) {
    g128 u;
#define JFSX_XPOW_STEP(K)                                       \
    u = g_mulxs<(1 << K)>(v);                                   \
    if ((i >> K) & 1u) v = u;
    JFSX_XPOW_STEP(0)
    JFSX_XPOW_STEP(1)
    JFSX_XPOW_STEP(2)
    JFSX_XPOW_STEP(3)
    JFSX_XPOW_STEP(4)
    JFSX_XPOW_STEP(5)
    JFSX_XPOW_STEP(6)
#undef JFSX_XPOW_STEP
    return v;
}

// One wave per block.  A per-object group of a few small blocks waits for
// this kernel before its main kernel, so its latency counts: the key schedule
// is expanded in lane 0's registers, H = E_K(0) and E_K(J0) are encrypted by
// two halves of the wave at once, only the H^(2^k) the block's exponents can
// reach are squared (k < bit length of its 16-byte block count, + margin;
// gcm_finalize_k reads h2k[k] only for bits its exponents have), the basis
// x^i H^64 is one x^i product per lane (g_mul_xpow) instead of a 128-step
// chain, and the bitsliced S-box masks are made only for a kernel that uses
// them (need_bs: the bitsliced or hybrid main kernel).
__global__ __launch_bounds__(64) void gcm_keysetup_k(const KeyIn *__restrict__ keys, const BlkDev *__restrict__ blks,
                                                    GcmSched *__restrict__ sched, const uint32_t *__restrict__ gtab,
                                                    int need_bs) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    KS_STAMP(0);
    GcmSched *sc = sched + b;
    const KeyIn k = keys[b];
    __shared__ uint32_t aes[512];  // T0 | T2, compact (gT0 / gT2 / gS)
    for (uint32_t x = lane; x < 256; x += 64) {
        aes[2 * x] = gtab[x * 64];
        aes[2 * x + 1] = gtab[x * 64 + 32];
    }
    __syncthreads();
    KS_STAMP(1);
    // AES-256 key expansion (FIPS-197 5.2), little-endian dwords: lane 0
    // expands in registers (static indices), then the schedule goes to LDS,
    // where every lane reads the words it needs by index
    __shared__ uint32_t sw[60];
    if (lane == 0) {
        uint32_t e[60];
#pragma unroll
        for (int i = 0; i < 8; i++) e[i] = k.key[i];
        uint32_t rcon = 1;
#pragma unroll
        for (int i = 8; i < 60; i++) {
            uint32_t t = e[i - 1];
            if ((i & 7) == 0) {
                t = (t >> 8) | (t << 24);  // RotWord
                t = gS(aes, t & 0xff) | (gS(aes, (t >> 8) & 0xff) << 8) | (gS(aes, (t >> 16) & 0xff) << 16) |
                    (gS(aes, t >> 24) << 24);
                t ^= rcon;
                rcon <<= 1;
            } else if ((i & 7) == 4) {
                t = gS(aes, t & 0xff) | (gS(aes, (t >> 8) & 0xff) << 8) | (gS(aes, (t >> 16) & 0xff) << 16) |
                    (gS(aes, t >> 24) << 24);
            }
            e[i] = e[i - 8] ^ t;
        }
#pragma unroll
        for (int i = 0; i < 60; i++) sw[i] = e[i];
    }
    __syncthreads();
    KS_STAMP(2);
    const uint32_t *w = sw;
    if (lane < 60) sc->rk[lane] = sw[lane];
    if (need_bs) {
        // bitsliced-AES masks: lane 4(r-1) + w computes dword w of u_r
        const uint32_t my = lane < 56 ? jfsx_bs::round_mask_word(sw, 1 + (int)(lane >> 2), (int)(lane & 3)) : 0u;
        if (lane < 56) sc->bsu[1 + (lane >> 2)][lane & 3] = my;
        // round-1 constants: S-boxes of the 12 nonce bytes (lanes 0..11), then
        // MixColumns of each column's uniform part (lanes 0..3)
        const uint32_t x0w[3] = {k.nonce[0] ^ w[0], k.nonce[1] ^ w[1], k.nonce[2] ^ w[2]};
        const uint32_t sb = lane < 12 ? jfsx_bs::sbox_byte((x0w[lane >> 2] >> (8 * (lane & 3))) & 0xffu) : 0u;
        uint32_t sbn[12];
        for (int i = 0; i < 12; i++) sbn[i] = (uint32_t)__shfl(sb, i, 64);
        const uint32_t u1[4] = {(uint32_t)__shfl(my, 0, 64), (uint32_t)__shfl(my, 1, 64), (uint32_t)__shfl(my, 2, 64),
                                (uint32_t)__shfl(my, 3, 64)};
        if (lane < 4) sc->r1c[lane] = jfsx_bs::round1_const(sbn, u1, (int)lane);
    }
    // round-0 state of the counter blocks (nonce || ctr) and round-1 constants
    const uint32_t x0 = k.nonce[0] ^ w[0], x1 = k.nonce[1] ^ w[1], x2 = k.nonce[2] ^ w[2];
    if (lane == 0) {
        sc->c012[0] = x0; sc->c012[1] = x1; sc->c012[2] = x2;
        sc->k1[0] = w[4] ^ gT0(aes, x0 & 0xff) ^ rotl8(gT0(aes, (x1 >> 8) & 0xff)) ^ gT2(aes, (x2 >> 16) & 0xff);
        sc->k1[1] = w[5] ^ gT0(aes, x1 & 0xff) ^ rotl8(gT0(aes, (x2 >> 8) & 0xff)) ^ rotl8(gT2(aes, x0 >> 24));
        sc->k1[2] = w[6] ^ gT0(aes, x2 & 0xff) ^ gT2(aes, (x0 >> 16) & 0xff) ^ rotl8(gT2(aes, x1 >> 24));
        sc->k1[3] = w[7] ^ rotl8(gT0(aes, (x0 >> 8) & 0xff)) ^ gT2(aes, (x1 >> 16) & 0xff) ^ rotl8(gT2(aes, x2 >> 24));
    }
    KS_STAMP(3);
    // H = E_K(0) on lanes 0..31 and E_K(J0) on lanes 32..63, at once
    uint32_t in[4], o[4], Hm[4], EJ0[4];
    {
        const bool j = lane >= 32;
        in[0] = j ? k.nonce[0] : 0u;
        in[1] = j ? k.nonce[1] : 0u;
        in[2] = j ? k.nonce[2] : 0u;
        in[3] = j ? 0x01000000u : 0u;  // J0 = nonce || BE32(1)
        aes_enc_global(aes, w, in, o);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            Hm[q] = (uint32_t)__shfl(o[q], 0, 64);
            EJ0[q] = (uint32_t)__shfl(o[q], 32, 64);
        }
    }
    const g128 H = g_from_mem(Hm);
    KS_STAMP(4);
    // H^(2^k) for the k this block's exponents can reach (at least k < 8,
    // which the lane powers below use)
    uint32_t nsq;
    {
        const uint64_t nb16 = (blks[b].len + 15) / 16 + 2;
        const uint32_t bits = 64u - (uint32_t)__builtin_clzll(nb16);
        nsq = bits + 1 < 8 ? 8u : bits + 1 > 32 ? 32u : bits + 1;
    }
    __shared__ g128 hs[8];  // H^(2^k), k < 8: uniform values read by index (LDS, not scratch)
    g128 g = H;
    for (uint32_t i = 0; i < nsq; i++) {
        if (i < 8 && lane == 0) hs[i] = g;
        if (lane == i) {
            uint32_t m[4];
            g_to_mem(g, m);
            for (int q = 0; q < 4; q++) sc->h2k[i][q] = m[q];
        }
        g = g_sqr(g);
    }
    __syncthreads();
    KS_STAMP(5);
#if JFSX_KS_NIB
    // H^e for e = lane (bits 0..5: six products by the uniform H^(2^q), each
    // kept where the lane's bit is set), then H^(64 + e) = H^e H^64, e < 4
    __shared__ uint4 gM[16];
    {
        g128 z = {{0x80000000u, 0, 0, 0}};  // x^0 = 1
        for (int q = 0; q < 6; q++) {
            const g128 m = JFSX_GF_CT ? g_mul_ct_call(z, hs[q]) : g_mul_uy_pre(z, hs[q], gM, lane);
            if ((lane >> q) & 1) z = m;
        }
        const g128 z64 = JFSX_GF_CT ? g_mul_ct_call(z, hs[6]) : g_mul_uy_pre(z, hs[6], gM, lane);
        uint32_t m[4];
        g_to_mem(z, m);
        for (int q = 0; q < 4; q++) sc->hpow[lane][q] = m[q];
        if (lane < 4) {
            g_to_mem(z64, m);
            for (int q = 0; q < 4; q++) sc->hpow[64 + lane][q] = m[q];
        }
    }
#else
    // H^e for e = lane and lane + 64 (< 68)
    for (int rep = 0; rep < 2; rep++) {
        const uint32_t e = lane + 64 * rep;
        if (e >= 68) break;
        g128 z = {{0x80000000u, 0, 0, 0}};  // x^0 = 1
        for (int q = 0; q < 7; q++)
            if ((e >> q) & 1) z = g_mul(z, hs[q]);
        uint32_t m[4];
        g_to_mem(z, m);
        for (int q = 0; q < 4; q++) sc->hpow[e][q] = m[q];
    }
#endif
    KS_STAMP(6);
    // basis x^i H^64: i = lane, and i = lane + 64 as x^64 times that
    {
        const g128 v = g_mul_xpow(hs[6], lane), v64 = g_mulxs<64>(v);
        uint32_t m[4];
        g_to_mem(v, m);
        for (int q = 0; q < 4; q++) sc->basis[lane][q] = m[q];
        g_to_mem(v64, m);
        for (int q = 0; q < 4; q++) sc->basis[64 + lane][q] = m[q];
    }
    KS_STAMP(7);
    // init = E_K(J0) ^ (len block) * H, len block = 0^64 || BE64(8*len)
    {
        const uint64_t bits = blks[b].len * 8;
        g128 L = {{0, 0, (uint32_t)(bits >> 32), (uint32_t)bits}};
#if JFSX_KS_NIB
        const g128 LH = JFSX_GF_CT ? g_mul_ct_call(L, H) : g_mul_uy_pre(L, H, gM, lane);  // lane 0 stores
#else
        const g128 LH = lane == 0 ? g_mul(L, H) : L;
#endif
        if (lane == 0) {
            uint32_t m[4];
            g_to_mem(LH, m);
            for (int q = 0; q < 4; q++) sc->init[q] = m[q] ^ EJ0[q];
        }
    }
    KS_STAMP(8);
}

#ifdef JFSX_KS_PHASES
extern "C" int jfsx_debug_main_phases(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_main_ts), sizeof(g_main_ts)) == hipSuccess ? 0 : -1;
}
extern "C" int jfsx_debug_ks_phases(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ks_ts), sizeof(g_ks_ts)) == hipSuccess ? 0 : -1;
}
#endif

// ---------------------------------------------------------------------------
// finalize: one workgroup per block, one thread per partial slot
// ---------------------------------------------------------------------------
// Each slot's partial is lifted by H^e (e = pexp) as products by the powers
// H^(2^k) the block's exponents use: per k, 16 threads build the 4-bit table
// of that (block-uniform) power in LDS and every thread whose e has bit k set
// takes the table product (g_mul_uy) -- 32 lookups instead of a bit-serial
// 128-step product per set bit.  A small batch (the per-object path) has
// blocks of many short tasks and so many slots: the workgroup grows to one
// thread per slot (up to 1024) instead of one wave looping over them.
// TH: the launch's thread cap.  TH = 64 (blocks of at most 64 slots: a group
// of small per-object blocks) takes g_mul_uy_pre, whose table rows sit in
// registers a 1024-thread workgroup does not have.
template <bool OPEN, int CRCMODE, int TH>
__global__ __launch_bounds__(TH) void gcm_finalize_k(const BlkDev *__restrict__ blks, const GcmSched *__restrict__ sched,
                                                      const uint32_t *__restrict__ partial,
                                                      const uint32_t *__restrict__ pexp, BlkOut *__restrict__ out) {
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nthr = blockDim.x;
    const uint32_t nw = nthr >> 6;
    __shared__ uint4 M[16];
    __shared__ uint32_t sor[16];
    __shared__ uint32_t sred[16][4];
    __shared__ uint32_t h2k[32][4];  // the block's H^(2^k), staged once (not a global load per product)
    const BlkDev blk = blks[b];
    const GcmSched *sc = sched + b;
    for (uint32_t i = tid; i < 128; i += nthr) h2k[i >> 2][i & 3] = sc->h2k[i >> 2][i & 3];  // 64-thread launches too
    __syncthreads();
    uint32_t acc[4] = {0, 0, 0, 0};
    for (uint32_t base = 0; base < blk.nslots; base += nthr) {
        const uint32_t s = base + tid;
        uint32_t m[4] = {0, 0, 0, 0}, e = 0;
        if (s < blk.nslots) {
            const uint32_t slot = blk.slot0 + s;
            for (int q = 0; q < 4; q++) m[q] = partial[4 * slot + q];
            if (m[0] | m[1] | m[2] | m[3]) e = pexp[slot];
        }
        // the powers any slot of the block needs (block-uniform loop below)
        uint32_t eo = e;
        for (int off = 32; off > 0; off >>= 1) eo |= __shfl_xor(eo, off, 64);
        if (lane == 0) sor[wave] = eo;
        __syncthreads();
        eo = 0;
        for (uint32_t w = 0; w < nw; w++) eo |= sor[w];
        g128 z = g_from_mem(m);
        for (int k = 0; k < 32 && (eo >> k); k++) {
            if (!((eo >> k) & 1u)) continue;
            const g128 zk = JFSX_GF_CT ? g_mul_ct_call(z, g_from_mem(h2k[k]))
                            : TH == 64 ? g_mul_uy_pre(z, g_from_mem(h2k[k]), M, tid)
                                       : g_mul_uy(z, g_from_mem(h2k[k]), M, tid);
            if ((e >> k) & 1u) z = zk;
        }
        g_to_mem(z, m);
        for (int q = 0; q < 4; q++) acc[q] ^= m[q];
        __syncthreads();  // sor is rewritten by the next round
    }
    for (int q = 0; q < 4; q++) acc[q] = wave_xor(acc[q]);
    if (lane == 0)
        for (int q = 0; q < 4; q++) sred[wave][q] = acc[q];
    __syncthreads();
    if (wave) return;
    for (int q = 0; q < 4; q++) {
        uint32_t t = sc->init[q];
        for (uint32_t w = 0; w < nw; w++) t ^= sred[w][q];
        acc[q] = t;
    }
    BlkOut o;
    o.status = JFSX_OK;
    o.bad_seg = -1;
    o.got = o.expect = 0;
    for (int q = 0; q < 4; q++) o.tag[q] = acc[q];
    if (OPEN) {
        const uint32_t *t = reinterpret_cast<const uint32_t *>(blk.tag_in);
        uint32_t d = 0;
        for (int q = 0; q < 4; q++) d |= acc[q] ^ t[q];
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
// need_bs: the bitsliced main kernel runs (JFSX_CTX_BITSLICE, or the hybrid
// shape selected by JFSX_GCM_HYBRID), so the schedule carries its S-box masks
void launch_gcm_keysetup(hipStream_t s, int n, const KeyIn *keys, const BlkDev *blks, GcmSched *sched, DevTables t,
                         bool bitslice) {
    static const bool hybrid = getenv("JFSX_GCM_HYBRID") != nullptr;
    if (n > 0)
        hipLaunchKernelGGL(gcm_keysetup_k, dim3(n), dim3(64), 0, s, keys, blks, sched, t.aes,
                           (int)(bitslice || hybrid));
}

void launch_gcm_main(hipStream_t s, int ntasks, int ncu, uint32_t *queue, bool open, int crc_mode, bool bitslice,
                     const Task *tasks, const BlkDev *blks, const GcmSched *sched, uint32_t *partial, uint32_t *pexp,
                     DevTables t) {
    if (ntasks <= 0) return;
    const unsigned grid = (unsigned)(ntasks < ncu ? ntasks : ncu);  // persistent: one workgroup per CU
    // queue: zeroed by the caller (uploaded with the batch descriptors)
    // JFSX_GCM_HYBRID="nbs,rho,prio" selects the hybrid shape (BS = 2) for the
    // T-table context (an A/B switch; see GcmShape)
    static const uint32_t hyb = [] {
        const char *e = getenv("JFSX_GCM_HYBRID");
        unsigned nbs = 0, rho = 16, prio = 2;
        if (!e || sscanf(e, "%u,%u,%u", &nbs, &rho, &prio) < 1) return 0xffffffffu;
        return (nbs & 7u) | ((rho & 255u) << 8) | ((prio & 3u) << 16);
    }();
#define L(O, C)                                                                                              \
    do {                                                                                                     \
        if (bitslice)                                                                                        \
            hipLaunchKernelGGL((gcm_main_k<O, C, 1, 1>), dim3(grid), dim3(GcmShape<1>::threads), 0, s, tasks,    \
                               (uint32_t)ntasks, queue, blks, sched, partial, pexp, t, 0u);                  \
        else if (hyb != 0xffffffffu)                                                                         \
            hipLaunchKernelGGL((gcm_main_k<O, C, 1, 2>), dim3(grid), dim3(GcmShape<2>::threads), 0, s, tasks,    \
                               (uint32_t)ntasks, queue, blks, sched, partial, pexp, t, hyb);                 \
        else                                                                                                 \
            hipLaunchKernelGGL((gcm_main_k<O, C, kStreams, 0>), dim3(grid), dim3(GcmShape<0>::threads), 0, s,    \
                               tasks, (uint32_t)ntasks, queue, blks, sched, partial, pexp, t, 0u);           \
    } while (0)
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

void launch_gcm_finalize(hipStream_t s, int n, bool open, int crc_mode, const BlkDev *blks, const GcmSched *sched,
                         const uint32_t *partial, const uint32_t *pexp, BlkOut *out, uint32_t max_slots) {
    if (n <= 0) return;
    // one thread per slot of the block with the most slots, 64..1024
    const uint32_t th = max_slots <= 64 ? 64u : max_slots >= 1024 ? 1024u : (max_slots + 63) / 64 * 64;
#define L(O, C)                                                                                          \
    do {                                                                                                 \
        if (th == 64)                                                                                    \
            hipLaunchKernelGGL((gcm_finalize_k<O, C, 64>), dim3(n), dim3(64), 0, s, blks, sched, partial, pexp, out); \
        else                                                                                             \
            hipLaunchKernelGGL((gcm_finalize_k<O, C, 1024>), dim3(n), dim3(th), 0, s, blks, sched, partial, pexp, out); \
    } while (0)
    if (open) {
        if ((crc_mode & 3) == 2) L(true, 2); else L(true, 0);
    } else {
        if ((crc_mode & 3) == 2) L(false, 2); else L(false, 0);
    }
#undef L
}

}  // namespace jfsx

#ifdef JFSX_ABLATE_TRACE
extern "C" __attribute__((visibility("default"))) int jfsx_debug_wgtrace(uint64_t *out, int n) {
    if (n > 65536) n = 65536;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jfsx::g_wgtrace), 32 * (size_t)n) == hipSuccess ? 0 : -5;
}
#endif

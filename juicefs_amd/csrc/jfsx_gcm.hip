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
#include "jfsx_dev.h"

namespace jfsx {

// ---------------------------------------------------------------------------
// LDS map of gcm_main (bytes): [0, 64K) AES T0|T2, [64K, 128K) GHASH table,
// [128K, 148K) CRC tables, [148K, +2K) GHASH basis staging.
// ---------------------------------------------------------------------------
constexpr uint32_t kLdsAes = 0;
constexpr uint32_t kLdsGh = 65536;
constexpr uint32_t kLdsCrc = 131072;
constexpr uint32_t kLdsBasis = 131072 + 20480;
constexpr uint32_t kLdsBytes = kLdsBasis + 2048;

__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }

// byte k of w moved to bits 8..15, lane offset kept in bits 0..7: the byte
// address of T0[byte] for this lane's replica (v_perm_b32, one VALU op)
#define AES_SEL(k) (0x0c0c0000u | ((4u + (k)) << 8))
#define TA(w, k) lds_u32(lds, __builtin_amdgcn_perm((w), loff, AES_SEL(k)))
#define TB(w, k) lds_u32(lds, __builtin_amdgcn_perm((w), loff, AES_SEL(k)) + 128u)

// One full AES round on LE column words (T1 = rotl8 T0, T3 = rotl8 T2).
#define AES_ROUND(o0, o1, o2, o3, i0, i1, i2, i3, r)                                        \
    o0 = TA(i0, 0) ^ rotl8(TA(i1, 1)) ^ TB(i2, 2) ^ rotl8(TB(i3, 3)) ^ rk[4 * (r) + 0];      \
    o1 = TA(i1, 0) ^ rotl8(TA(i2, 1)) ^ TB(i3, 2) ^ rotl8(TB(i0, 3)) ^ rk[4 * (r) + 1];      \
    o2 = TA(i2, 0) ^ rotl8(TA(i3, 1)) ^ TB(i0, 2) ^ rotl8(TB(i1, 3)) ^ rk[4 * (r) + 2];      \
    o3 = TA(i3, 0) ^ rotl8(TA(i0, 1)) ^ TB(i1, 2) ^ rotl8(TB(i2, 3)) ^ rk[4 * (r) + 3];

#define AES_LAST(o, a, b, c, d, rkv) \
    o = ((TB(a, 0) & 0xffu) | (TA(b, 1) & 0xff00u) | (TA(c, 2) & 0xff0000u) | (TB(d, 3) & 0xff000000u)) ^ (rkv);

// Keystream block for counter value ctr (the BE32 in bytes 12..15).
__device__ __forceinline__ void aes_ctr_block(const char *lds, uint32_t loff, const uint32_t *rk,
                                              const uint32_t *k1, uint32_t ctr, uint32_t ks[4]) {
    uint32_t x3 = __builtin_bswap32(ctr) ^ rk[3];
    // round 1: columns' constant terms precomputed (k1); only x3 varies
    uint32_t a0 = k1[0] ^ rotl8(TB(x3, 3));
    uint32_t a1 = k1[1] ^ TB(x3, 2);
    uint32_t a2 = k1[2] ^ rotl8(TA(x3, 1));
    uint32_t a3 = k1[3] ^ TA(x3, 0);
    uint32_t b0, b1, b2, b3;
    AES_ROUND(b0, b1, b2, b3, a0, a1, a2, a3, 2);
    AES_ROUND(a0, a1, a2, a3, b0, b1, b2, b3, 3);
    AES_ROUND(b0, b1, b2, b3, a0, a1, a2, a3, 4);
    AES_ROUND(a0, a1, a2, a3, b0, b1, b2, b3, 5);
    AES_ROUND(b0, b1, b2, b3, a0, a1, a2, a3, 6);
    AES_ROUND(a0, a1, a2, a3, b0, b1, b2, b3, 7);
    AES_ROUND(b0, b1, b2, b3, a0, a1, a2, a3, 8);
    AES_ROUND(a0, a1, a2, a3, b0, b1, b2, b3, 9);
    AES_ROUND(b0, b1, b2, b3, a0, a1, a2, a3, 10);
    AES_ROUND(a0, a1, a2, a3, b0, b1, b2, b3, 11);
    AES_ROUND(b0, b1, b2, b3, a0, a1, a2, a3, 12);
    AES_ROUND(a0, a1, a2, a3, b0, b1, b2, b3, 13);
    AES_LAST(ks[0], a0, a1, a2, a3, rk[56]);
    AES_LAST(ks[1], a1, a2, a3, a0, rk[57]);
    AES_LAST(ks[2], a2, a3, a0, a1, rk[58]);
    AES_LAST(ks[3], a3, a0, a1, a2, rk[59]);
}

// acc * H^64 with the byte-sliced table: XOR_j T[j][byte_j(acc)]
__device__ __forceinline__ void ghash_mul_tab(const char *lds, uint32_t acc[4]) {
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        uint32_t b = (acc[j >> 2] >> (8 * (j & 3))) & 0xffu;
        uint4 t = lds_u4(lds, (b << 4) + kLdsGh + 4096u * j);
        z0 ^= t.x; z1 ^= t.y; z2 ^= t.z; z3 ^= t.w;
    }
    acc[0] = z0; acc[1] = z1; acc[2] = z2; acc[3] = z3;
}

template <bool OPEN, int CRCMODE>
__global__ __launch_bounds__(kThreads) void gcm_main_k(const Task *__restrict__ tasks,
                                                       const BlkDev *__restrict__ blks,
                                                       const GcmSched *__restrict__ sched,
                                                       uint32_t *__restrict__ partial, uint32_t *__restrict__ pexp,
                                                       DevTables tab) {
    __shared__ __attribute__((aligned(16))) char lds[kLdsBytes];
    const Task task = tasks[blockIdx.x];
    const BlkDev blk = blks[task.blk];
    const GcmSched *sch = sched + task.blk;
    const uint32_t tid = threadIdx.x;

    // ---- stage tables ----
    {
        const uint4 *ga = reinterpret_cast<const uint4 *>(tab.aes);
        uint4 *la = reinterpret_cast<uint4 *>(lds + kLdsAes);
        for (uint32_t i = tid; i < 4096; i += kThreads) la[i] = ga[i];
        const uint4 *gc = reinterpret_cast<const uint4 *>(tab.crc);
        uint4 *lc = reinterpret_cast<uint4 *>(lds + kLdsCrc);
        for (uint32_t i = tid; i < 1280; i += kThreads) lc[i] = gc[i];
        if (tid < 128)
            reinterpret_cast<uint4 *>(lds + kLdsBasis)[tid] = reinterpret_cast<const uint4 *>(sch->basis)[tid];
    }
    __syncthreads();
    {
        uint4 *lg = reinterpret_cast<uint4 *>(lds + kLdsGh);
        const uint4 *lb = reinterpret_cast<const uint4 *>(lds + kLdsBasis);
        for (uint32_t e = tid; e < 4096; e += kThreads) {
            uint32_t j = e >> 8, b = e & 255;
            uint4 z = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if ((b >> (7 - k)) & 1) {
                    uint4 v = lb[8 * j + k];
                    z.x ^= v.x; z.y ^= v.y; z.z ^= v.z; z.w ^= v.w;
                }
            }
            lg[e] = z;
        }
    }
    __syncthreads();

    uint32_t rk[60];
#pragma unroll
    for (int i = 0; i < 60; i++) rk[i] = sch->rk[i];
    uint32_t k1[4] = {sch->k1[0], sch->k1[1], sch->k1[2], sch->k1[3]};

    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint32_t loff = (lane & 31) << 2;
    const uint64_t c0 = task.c0, c1 = task.c1;
    const uint32_t nseg = (uint32_t)((c1 - c0 + kSeg - 1) / kSeg);
    const uint32_t sa = wave * nseg / kWaves, sb = (wave + 1) * nseg / kWaves;
    const uint64_t sub0 = c0 + (uint64_t)sa * kSeg;
    const uint64_t sub1 = sb > sa ? (c0 + (uint64_t)sb * kSeg < c1 ? c0 + (uint64_t)sb * kSeg : c1) : sub0;
    const uint8_t *src = blk.src;
    uint8_t *dst = blk.dst;
    const uint32_t xl = CRCMODE ? tab.crcx[lane] : 0u;

    uint32_t acc[4] = {0, 0, 0, 0};
    uint64_t jlast = 0;
    bool has = false;
    uint32_t A = 0, lend = 0;
    uint64_t seg0 = sub0;

    const uint64_t nrows = (sub1 - sub0 + 1023) / 1024;
    uint4 nxt = make_uint4(0, 0, 0, 0);
    if (nrows) nxt = load_piece(src, sub0 + 16 * lane, sub1);
    for (uint64_t r = 0; r < nrows; r++) {
        const uint64_t row = sub0 + 1024 * r;
        const uint64_t o = row + 16 * lane;
        uint4 d = nxt;
        if (r + 1 < nrows) nxt = load_piece(src, o + 1024, sub1);
        const bool valid = o < sub1;
        const bool full = o + 16 <= sub1;
        const uint64_t j = o >> 4;
        uint32_t ks[4];
        aes_ctr_block(lds, loff, rk, k1, (uint32_t)(j + 2), ks);
        uint4 x = make_uint4(d.x ^ ks[0], d.y ^ ks[1], d.z ^ ks[2], d.w ^ ks[3]);
        uint4 c = OPEN ? d : x;   // ciphertext
        uint4 p = OPEN ? x : d;   // plaintext
        if (!full) {
            // zero the bytes past the end (GHASH pads C with zeros)
            const int nv = valid ? (int)(sub1 - o) : 0;
            uint32_t m[4];
            for (int k = 0; k < 4; k++) {
                int bytes = nv - 4 * k;
                m[k] = bytes >= 4 ? 0xffffffffu : (bytes <= 0 ? 0u : ((1u << (8 * bytes)) - 1u));
            }
            c.x &= m[0]; c.y &= m[1]; c.z &= m[2]; c.w &= m[3];
            p.x &= m[0]; p.y &= m[1]; p.z &= m[2]; p.w &= m[3];
        }
        if (valid) store_piece(dst, o, sub1, OPEN ? p : c);
        // GHASH Horner step
        {
            uint32_t t[4] = {acc[0], acc[1], acc[2], acc[3]};
            ghash_mul_tab(lds, t);
            if (valid) {
                acc[0] = t[0] ^ c.x; acc[1] = t[1] ^ c.y; acc[2] = t[2] ^ c.z; acc[3] = t[3] ^ c.w;
                jlast = j;
                has = true;
            }
        }
        if (CRCMODE) {
            if (full) {
                A = crc_piece<kLdsCrc>(lds, A, p.x, p.y, p.z, p.w);
                lend = (uint32_t)(o + 16 - seg0);
            } else if (valid) {
                const uint32_t pw[4] = {p.x, p.y, p.z, p.w};
                A = crc_partial<kLdsCrc>(lds, A, pw, (int)(sub1 - o));
                lend = (uint32_t)(sub1 - seg0);
            }
            const uint64_t seg1 = seg0 + kSeg < sub1 ? seg0 + kSeg : sub1;
            if (row + 1024 >= seg1) {  // segment end
                const uint32_t Lseg = (uint32_t)(seg1 - seg0);
                uint32_t v;
                uint32_t K;
                if (Lseg == (uint32_t)kSeg) {
                    v = crc_mulmod(xl, A);
                    K = tab.crcx[64 + 32];
                } else {
                    v = crc_mulmod(crc_xpow8(Lseg - lend, tab.crcx + 64), A);
                    K = crc_mulmod(crc_xpow8(Lseg, tab.crcx + 64), 0xffffffffu);
                }
                const uint32_t raw = wave_xor(v);
                if (lane == 0) {
                    const uint32_t crc = ~(K ^ raw);
                    const uint64_t si = seg0 / kSeg;
                    if (CRCMODE == 1) {
                        *reinterpret_cast<uint32_t *>(blk.crc + 4 * si) = __builtin_bswap32(crc);
                    } else {
                        blk.crc_calc[si] = crc;
                    }
                }
                A = 0;
                lend = 0;
                seg0 = seg1;
            }
        }
    }

    // ---- wave epilogue: lift lane accumulators to the wave end, reduce ----
    const uint64_t wend = (sub1 + 15) >> 4;  // blocks before the wave end
    g128 z = {{0, 0, 0, 0}};
    if (has) {
        const uint32_t e = (uint32_t)(wend + 1 - jlast);  // in [2, 65]
        g128 h = g_from_mem(sch->hpow[e]);
        z = g_mul(g_from_mem(acc), h);
    }
    uint32_t zm[4];
    g_to_mem(z, zm);
    for (int k = 0; k < 4; k++) zm[k] = wave_xor(zm[k]);
    if (lane == 0) {
        const uint32_t slot = task.slot0 + wave;
        partial[4 * slot + 0] = zm[0];
        partial[4 * slot + 1] = zm[1];
        partial[4 * slot + 2] = zm[2];
        partial[4 * slot + 3] = zm[3];
        const uint64_t nblk = (blk.len + 15) >> 4;
        pexp[slot] = (uint32_t)(nblk - wend);
    }
}

// ---------------------------------------------------------------------------
// keysetup: one wave per block; AES via the (global) T-table image
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t gT0(const uint32_t *aes, uint32_t x) { return aes[x * 64]; }
__device__ __forceinline__ uint32_t gT2(const uint32_t *aes, uint32_t x) { return aes[x * 64 + 32]; }
__device__ __forceinline__ uint32_t gS(const uint32_t *aes, uint32_t x) { return (aes[x * 64] >> 8) & 0xffu; }

__device__ uint32_t gcol(const uint32_t *aes, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return gT0(aes, a & 0xff) ^ rotl8(gT0(aes, (b >> 8) & 0xff)) ^ gT2(aes, (c >> 16) & 0xff) ^
           rotl8(gT2(aes, d >> 24));
}

__device__ void aes_enc_global(const uint32_t *aes, const uint32_t *rk, const uint32_t in[4], uint32_t out[4]) {
    uint32_t s[4], t[4];
    for (int c = 0; c < 4; c++) s[c] = in[c] ^ rk[c];
    for (int r = 1; r < 14; r++) {
        for (int c = 0; c < 4; c++) t[c] = gcol(aes, s[c], s[(c + 1) & 3], s[(c + 2) & 3], s[(c + 3) & 3]) ^ rk[4 * r + c];
        for (int c = 0; c < 4; c++) s[c] = t[c];
    }
    for (int c = 0; c < 4; c++) {
        uint32_t a = s[c], b = s[(c + 1) & 3], cc = s[(c + 2) & 3], d = s[(c + 3) & 3];
        out[c] = (gS(aes, a & 0xff) | (gS(aes, (b >> 8) & 0xff) << 8) | (gS(aes, (cc >> 16) & 0xff) << 16) |
                  (gS(aes, d >> 24) << 24)) ^ rk[56 + c];
    }
}

__global__ __launch_bounds__(64) void gcm_keysetup_k(const KeyIn *__restrict__ keys, const BlkDev *__restrict__ blks,
                                                    GcmSched *__restrict__ sched, const uint32_t *__restrict__ aes) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    GcmSched *sc = sched + b;
    const KeyIn k = keys[b];
    // AES-256 key expansion (FIPS-197 5.2), little-endian dwords
    uint32_t w[60];
    for (int i = 0; i < 8; i++) w[i] = k.key[i];
    uint32_t rcon = 1;
    for (int i = 8; i < 60; i++) {
        uint32_t t = w[i - 1];
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
        w[i] = w[i - 8] ^ t;
    }
    if (lane < 60) sc->rk[lane] = w[lane];
    // round-0 state of the counter blocks (nonce || ctr) and round-1 constants
    const uint32_t x0 = k.nonce[0] ^ w[0], x1 = k.nonce[1] ^ w[1], x2 = k.nonce[2] ^ w[2];
    if (lane == 0) {
        sc->c012[0] = x0; sc->c012[1] = x1; sc->c012[2] = x2;
        sc->k1[0] = w[4] ^ gT0(aes, x0 & 0xff) ^ rotl8(gT0(aes, (x1 >> 8) & 0xff)) ^ gT2(aes, (x2 >> 16) & 0xff);
        sc->k1[1] = w[5] ^ gT0(aes, x1 & 0xff) ^ rotl8(gT0(aes, (x2 >> 8) & 0xff)) ^ rotl8(gT2(aes, x0 >> 24));
        sc->k1[2] = w[6] ^ gT0(aes, x2 & 0xff) ^ gT2(aes, (x0 >> 16) & 0xff) ^ rotl8(gT2(aes, x1 >> 24));
        sc->k1[3] = w[7] ^ rotl8(gT0(aes, (x0 >> 8) & 0xff)) ^ gT2(aes, (x1 >> 16) & 0xff) ^ rotl8(gT2(aes, x2 >> 24));
    }
    // H = E_K(0), E_K(J0)
    uint32_t zero[4] = {0, 0, 0, 0}, Hm[4], J0[4], EJ0[4];
    aes_enc_global(aes, w, zero, Hm);
    J0[0] = k.nonce[0]; J0[1] = k.nonce[1]; J0[2] = k.nonce[2]; J0[3] = 0x01000000u;  // BE32(1)
    aes_enc_global(aes, w, J0, EJ0);
    const g128 H = g_from_mem(Hm);
    // H^(2^k)
    g128 hs[8];
    g128 g = H;
    for (int i = 0; i < 32; i++) {
        if (i < 8) hs[i] = g;
        if ((int)lane == i) {
            uint32_t m[4];
            g_to_mem(g, m);
            for (int q = 0; q < 4; q++) sc->h2k[i][q] = m[q];
        }
        g = g_sqr(g);
    }
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
    // basis x^i * H^64
    g128 v = hs[6];
    for (int i = 0; i < 128; i++) {
        if ((i & 63) == (int)lane) {
            uint32_t m[4];
            g_to_mem(v, m);
            for (int q = 0; q < 4; q++) sc->basis[i][q] = m[q];
        }
        v = g_mulx(v);
    }
    // init = E_K(J0) ^ (len block) * H, len block = 0^64 || BE64(8*len)
    if (lane == 0) {
        const uint64_t bits = blks[b].len * 8;
        g128 L = {{0, 0, (uint32_t)(bits >> 32), (uint32_t)bits}};
        g128 LH = g_mul(L, H);
        uint32_t m[4];
        g_to_mem(LH, m);
        for (int q = 0; q < 4; q++) sc->init[q] = m[q] ^ EJ0[q];
    }
}

// ---------------------------------------------------------------------------
// finalize: one wave per block
// ---------------------------------------------------------------------------
template <bool OPEN, int CRCMODE>
__global__ __launch_bounds__(64) void gcm_finalize_k(const BlkDev *__restrict__ blks, const GcmSched *__restrict__ sched,
                                                    const uint32_t *__restrict__ partial,
                                                    const uint32_t *__restrict__ pexp, BlkOut *__restrict__ out) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const BlkDev blk = blks[b];
    const GcmSched *sc = sched + b;
    uint32_t acc[4] = {0, 0, 0, 0};
    for (uint32_t base = 0; base < blk.nslots; base += 64) {
        const uint32_t s = base + lane;
        if (s < blk.nslots) {
            const uint32_t slot = blk.slot0 + s;
            uint32_t m[4] = {partial[4 * slot], partial[4 * slot + 1], partial[4 * slot + 2], partial[4 * slot + 3]};
            if (m[0] | m[1] | m[2] | m[3]) {
                g128 z = g_from_mem(m);
                uint32_t e = pexp[slot];
                for (int k = 0; e; k++, e >>= 1)
                    if (e & 1) z = g_mul(z, g_from_mem(sc->h2k[k]));
                g_to_mem(z, m);
                for (int q = 0; q < 4; q++) acc[q] ^= m[q];
            }
        }
    }
    for (int q = 0; q < 4; q++) acc[q] = wave_xor(acc[q]) ^ sc->init[q];
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
    if (CRCMODE == 2) {
        crc_verify_block(blk, o, lane);
        if (o.bad_seg >= 0 && o.status == JFSX_OK) o.status = JFSX_ECRC;
    }
    if (lane == 0) out[b] = o;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
void launch_gcm_keysetup(hipStream_t s, int n, const KeyIn *keys, const BlkDev *blks, GcmSched *sched, DevTables t) {
    if (n > 0) hipLaunchKernelGGL(gcm_keysetup_k, dim3(n), dim3(64), 0, s, keys, blks, sched, t.aes);
}

void launch_gcm_main(hipStream_t s, int ntasks, bool open, int crc_mode, const Task *tasks, const BlkDev *blks,
                     const GcmSched *sched, uint32_t *partial, uint32_t *pexp, DevTables t) {
    if (ntasks <= 0) return;
    dim3 g(ntasks), bl(kThreads);
#define L(O, C) hipLaunchKernelGGL((gcm_main_k<O, C>), g, bl, 0, s, tasks, blks, sched, partial, pexp, t)
    if (open) {
        if (crc_mode == 0) L(true, 0); else if (crc_mode == 1) L(true, 1); else L(true, 2);
    } else {
        if (crc_mode == 0) L(false, 0); else if (crc_mode == 1) L(false, 1); else L(false, 2);
    }
#undef L
}

void launch_gcm_finalize(hipStream_t s, int n, bool open, int crc_mode, const BlkDev *blks, const GcmSched *sched,
                         const uint32_t *partial, const uint32_t *pexp, BlkOut *out) {
    if (n <= 0) return;
#define L(O, C) hipLaunchKernelGGL((gcm_finalize_k<O, C>), dim3(n), dim3(64), 0, s, blks, sched, partial, pexp, out)
    if (open) {
        if (crc_mode == 2) L(true, 2); else L(true, 0);
    } else {
        if (crc_mode == 2) L(false, 2); else L(false, 0);
    }
#undef L
}

}  // namespace jfsx

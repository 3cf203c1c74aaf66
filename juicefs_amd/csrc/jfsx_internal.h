// jfsx_internal.h -- shared structures and device helpers of libjfsx (gfx950).
//
// Data layout in HBM (per batch, all device resident):
//   BlkDev[n]      pointers/lengths of each block, slot range for partial tags
//   KeyIn[n]       32-B key + 12-B nonce per block
//   GcmSched[n]    per-key schedule written by gcm_keysetup (4.9 KiB/key)
//   Task[t]        (block, byte range) handled by one workgroup
//   partial[s]     per-wave GHASH / Poly1305 partial sums, s = task*16 + wave
//   pexp[s]        power of H (or r) that lifts partial[s] to its final place
//   crc scratch    computed CRCs for VERIFY mode (compared in finalize)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/jfsx.h"

#define JFSX_GF_HD __device__ __forceinline__
#define JFSX_GF_BREAK() __builtin_amdgcn_sched_barrier(0)
#include "jfsx_gf.h"

namespace jfsx {

constexpr int kSeg = 32768;         // csBlock (disk_cache.go:1207)
#ifndef JFSX_WAVES
#define JFSX_WAVES 16
#endif
constexpr int kWaves = JFSX_WAVES;  // waves per transform workgroup
constexpr int kThreads = kWaves * 64;
#ifndef JFSX_STREAMS
#define JFSX_STREAMS 1
#endif
// GHASH table walk issued in groups of lookups with a scheduling fence between
// them (lower peak VGPRs): 4 = four quarters of 4, 1 = two halves of 8
// (default; +0.7% over quarters at 8 GiB, equal at 64 GiB, fewer spills),
// 0 = all 16 at once.
#ifndef JFSX_GH8
#define JFSX_GH8 1
#endif
// Two-row unrolled T-table loop (two AES chains interleaved); with the GHASH
// quarters it fits the 128-VGPR cap (+2% measured).
// rows per iteration of the default shape's T-table loop (2 fits 128 VGPRs)
#ifndef JFSX_UR0
#define JFSX_UR0 2
#endif
// rows per iteration of the 8-wave (BS = 2) shape's T-table loop
#ifndef JFSX_HYB_UR
#define JFSX_HYB_UR 4
#endif
// software-pipelined GHASH/CRC in the 8-wave shape's T-table loop
#ifndef JFSX_HYB_SWP
#define JFSX_HYB_SWP 0
#endif
#ifndef JFSX_U2
#define JFSX_U2 1
#endif
// Counter-uniform rounds 1-2 in the two-row loop (aes_r2_uniform, jfsx_gcm.hip).
#ifndef JFSX_UCTR
#define JFSX_UCTR 1
#endif
// GHASH accumulator rotation (gh_rho) by v_perm selectors instead of v_cndmask.
#ifndef JFSX_GHPERM
#define JFSX_GHPERM 1
#endif
// CRC table addresses by an SDWA byte-select shift (byte_x4, jfsx_dev.h).
#ifndef JFSX_CRCSDWA
#define JFSX_CRCSDWA 1
#endif
// T-table rounds 2..13 with pre-rotated round keys folded into a v_bitop3 (AES_COL).
#ifndef JFSX_RKR
#define JFSX_RKR 1
#endif
constexpr int kStreams = JFSX_STREAMS;        // independent segment streams per wave (ILP)
constexpr int kSlotsPerTask = kWaves * kStreams;  // GHASH/Poly partial slots per task
constexpr int kMaxTaskBytes = 4 << 20;
constexpr uint32_t kCrcPoly = 0x82F63B78u;  // reflected Castagnoli

struct KeyIn {
    uint32_t key[8];
    uint32_t nonce[3];
    uint32_t pad;
};

struct BlkDev {
    const uint8_t *src;
    uint8_t *dst;
    uint64_t len;
    uint8_t *crc;          // GEN: BE32 out; VERIFY: expected BE32 in
    uint32_t *crc_calc;    // VERIFY: computed CRCs (native u32), else null
    uint32_t slot0;        // first partial slot of this block
    uint32_t nslots;       // number of partial slots (16 per task)
    const uint8_t *tag_in; // OPEN: expected tag (device copy), else null
};

struct Task {
    uint32_t blk;
    uint32_t slot0;
    uint64_t c0, c1;  // byte range of the block; c0 % kSeg == 0
#ifdef JFSX_ABLATE_TRACE
    uint32_t trace, pad;  // diagnostic builds: index in the planned order
#endif
};

// LZ4 stage (jfsx_lz4.hip): one block per wave
struct ZDev {
    const uint8_t *src;
    uint8_t *dst;
    uint64_t len;  // input bytes
    uint64_t cap;  // dst capacity
};
struct ZOut {
    uint64_t out_len;
    int32_t status;
    int32_t fallback;  // zstd decompression: why the serial decoder took the object (0: it did not)
};

struct BlkOut {        // written by finalize, copied back to the host
    uint32_t tag[4];
    int32_t status;
    int32_t bad_seg;
    uint32_t got, expect;
};

// per-key AES-256-GCM schedule
struct GcmSched {
    uint32_t rk[60];         // round keys, little-endian dwords of the byte schedule
    uint32_t k1[4];          // round-1 constants of the counter block (columns' constant terms ^ rk[4..7])
    uint32_t c012[3];        // round-0 state words 0..2 (nonce ^ rk[0..2])
    uint32_t pad;
    uint32_t init[4];        // E_K(J0) ^ GHASH contribution of the length block (memory order)
    uint32_t basis[128][4];  // x^i * H^64, memory order
    uint32_t hpow[68][4];    // H^k, memory order (k = 0..67)
    uint32_t h2k[32][4];     // H^(2^k), memory order
    uint32_t bsu[16][4];     // bitsliced-AES S-box output masks of rounds 1..14 (jfsx_aes_bs.h)
    uint32_t r1c[4];         // CTR round-1 constants of the 32-slot layout (round1_const)
};

// per-key ChaCha20-Poly1305 schedule (Poly1305 values in 26-bit limbs)
struct CpSched {
    uint32_t key[8];
    uint32_t nonce[3];
    uint32_t pad0;
    uint32_t s[4];          // Poly1305 s (keystream block 0, bytes 16..31)
    uint32_t r[5];          // clamped r
    uint32_t r253[5];       // r^253: gap between a lane's row chunks (4 KiB rows)
    uint32_t init[5];       // (length block) * r
    uint32_t pad1;
    uint32_t r2k[32][5];    // r^(2^k)
};

constexpr uint64_t kCrcTaskBytes = 4 << 20;  // bytes per CRC-only task (crc_segments_k)
constexpr int kCpWaves = 4;                 // waves per ChaCha20-Poly1305 workgroup
constexpr int kCpTaskBytes = 1 << 20;       // bytes per ChaCha task (<= kCpWaves * segments)
constexpr int kCpGroupsPerCu = 4;           // cp_main_k occupancy: 4 waves/SIMD at <= 128 VGPRs

// ---------------------------------------------------------------------------
// GF(2^128) in GCM convention.  "BE words": w[0] holds bytes 0..3 big-endian;
// bit 31 of w[0] is the coefficient of x^0.  Memory order = the 16 bytes as
// stored, loaded as little-endian dwords (w[k] = bswap(d[k])).
// ---------------------------------------------------------------------------
struct g128 {
    uint32_t w[4];
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ g128 g_from_mem(const uint32_t d[4]) {
    g128 r;
    for (int k = 0; k < 4; k++) r.w[k] = bswap32(d[k]);
    return r;
}
__device__ __forceinline__ void g_to_mem(const g128 &a, uint32_t d[4]) {
    for (int k = 0; k < 4; k++) d[k] = bswap32(a.w[k]);
}

// multiply by x (right shift in this convention, reduce with 0xE1 << 120)
__device__ __forceinline__ g128 g_mulx(g128 v) {
    uint32_t lsb = v.w[3] & 1u;
    v.w[3] = __builtin_amdgcn_alignbit(v.w[2], v.w[3], 1);
    v.w[2] = __builtin_amdgcn_alignbit(v.w[1], v.w[2], 1);
    v.w[1] = __builtin_amdgcn_alignbit(v.w[0], v.w[1], 1);
    v.w[0] = (v.w[0] >> 1) ^ (0xE1000000u & (0u - lsb));
    return v;
}

// per-lane x times per-lane y from integer multiplies (jfsx_gf.h): about 500
// instructions against g_mul's 2000, no LDS, no barrier
__device__ __forceinline__ g128 g_mul_ct(const g128 &x, const g128 &y) {
    g128 z;
    jfsx_gf::mul(x.w, y.w, z.w);
    return z;
}

// the same as a call: the GCM kernels take it this way (inlined into them,
// the iterative-ILP scheduler of the ROCm 7.2 compiler crashes)
__device__ __noinline__ g128 g_mul_ct_call(g128 x, g128 y) { return g_mul_ct(x, y); }

// generic bit-serial product (SP 800-38D Algorithm 1)
__device__ __noinline__ g128 g_mul(g128 x, g128 y) {
    g128 z = {{0, 0, 0, 0}};
    g128 v = y;
#pragma unroll 1
    for (int k = 0; k < 4; k++) {
        uint32_t xw = x.w[k];
#pragma unroll 8
        for (int i = 0; i < 32; i++) {
            uint32_t m = 0u - (xw >> 31);
            xw <<= 1;
            z.w[0] ^= v.w[0] & m;
            z.w[1] ^= v.w[1] & m;
            z.w[2] ^= v.w[2] & m;
            z.w[3] ^= v.w[3] & m;
            v = g_mulx(v);
        }
    }
    return z;
}

// spread the low 16 bits of x to the even bit positions
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// squaring is linear over GF(2): coefficient i -> 2i, then reduce
__device__ __forceinline__ g128 g_sqr(g128 a) {
    uint32_t W[8];
    for (int k = 0; k < 4; k++) {
        W[2 * k] = spread16(a.w[k] >> 16) << 1;
        W[2 * k + 1] = spread16(a.w[k]) << 1;
    }
    // high half H = W[4..7] (x^128..x^255): add H*(1 + x + x^2 + x^7) at x^0
    uint32_t h0 = W[4], h1 = W[5], h2 = W[6], h3 = W[7];
    uint32_t o = (h3 << 31) ^ (h3 << 30) ^ (h3 << 25);  // bits pushed past x^127
    g128 r;
    r.w[0] = W[0] ^ h0 ^ (h0 >> 1) ^ (h0 >> 2) ^ (h0 >> 7);
    r.w[1] = W[1] ^ h1 ^ __builtin_amdgcn_alignbit(h0, h1, 1) ^ __builtin_amdgcn_alignbit(h0, h1, 2) ^
             __builtin_amdgcn_alignbit(h0, h1, 7);
    r.w[2] = W[2] ^ h2 ^ __builtin_amdgcn_alignbit(h1, h2, 1) ^ __builtin_amdgcn_alignbit(h1, h2, 2) ^
             __builtin_amdgcn_alignbit(h1, h2, 7);
    r.w[3] = W[3] ^ h3 ^ __builtin_amdgcn_alignbit(h2, h3, 1) ^ __builtin_amdgcn_alignbit(h2, h3, 2) ^
             __builtin_amdgcn_alignbit(h2, h3, 7);
    r.w[0] ^= o ^ (o >> 1) ^ (o >> 2) ^ (o >> 7);
    return r;
}

// ---------------------------------------------------------------------------
// CRC32C in GF(2)[x]/P, reflected: bit 31 is the coefficient of x^0.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t crc_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll 8
    for (int i = 0; i < 32; i++) {
        p ^= b & (0u - (a >> 31));
        a <<= 1;
        b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
    }
    return p;
}

// x^(8n) mod P using x8pow[k] = x^(8*2^k) mod P
__device__ __forceinline__ uint32_t crc_xpow8(uint64_t n, const uint32_t *x8pow) {
    uint32_t r = 0x80000000u;  // x^0
    for (int k = 0; n; k++, n >>= 1)
        if (n & 1) r = crc_mulmod(x8pow[k], r);
    return r;
}

// x^(8n) mod P for n < 32768 from the context's crcx table: whole 1 KiB rows
// (crcx[96 + k] = x^(8*1024k)), then 16-byte steps (crcx[63 - j] =
// x^(8*16j)), then the last 0..15 bytes by squares (crcx[64 + b]) -- at most
// five products instead of one per set bit of n
__device__ __forceinline__ uint32_t crc_xpow8_fast(uint32_t n, const uint32_t *crcx) {
    const uint32_t k = n >> 10, j = (n >> 4) & 63, r = n & 15;
    uint32_t v = k ? crcx[96 + k] : 0x80000000u;
    if (j) v = k ? crc_mulmod(v, crcx[63 - j]) : crcx[63 - j];
    for (int b = 0; b < 4; b++)
        if ((r >> b) & 1) v = crc_mulmod(v, crcx[64 + b]);
    return v;
}

// wave-wide XOR reduction
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v ^= __shfl_xor(v, off, 64);
    return v;
}

}  // namespace jfsx

// launchers (defined in the .hip files, called by jfsx_api.cpp)
struct JfsxTables;
namespace jfsx {
struct DevTables {
    const uint32_t *aes;    // 16384 dwords: T0|T2 replicated x32 per index
    const uint32_t *crc;    // 32 x 256 dwords: U0..U15 (slice-by-16), shift 1008 B, 4032 B, 1024 B, 4096 B
    const uint32_t *crcx;   // 64 lane shift constants, 32 x8pow, K_full
};
void launch_gcm_keysetup(hipStream_t s, int n, const KeyIn *keys, const BlkDev *blks, GcmSched *sched,
                         DevTables t, bool bitslice);
// persistent over min(ntasks, ncu) workgroups; queue: 4 device bytes the caller zeroed (enqueue_aead uploads it)
void launch_gcm_main(hipStream_t s, int ntasks, int ncu, uint32_t *queue, bool open, int crc_mode, bool bitslice,
                     const Task *tasks, const BlkDev *blks, const GcmSched *sched, uint32_t *partial, uint32_t *pexp,
                     DevTables t);
// max_slots: the most partial slots any block of the batch has (sizes the workgroup)
void launch_gcm_finalize(hipStream_t s, int n, bool open, int crc_mode, const BlkDev *blks, const GcmSched *sched,
                         const uint32_t *partial, const uint32_t *pexp, BlkOut *out, uint32_t max_slots);
void launch_cp_keysetup(hipStream_t s, int n, const KeyIn *keys, const BlkDev *blks, CpSched *sched);
void launch_cp_main(hipStream_t s, int ntasks, int ncu, uint32_t *queue, bool open, int crc_mode, const Task *tasks,
                    const BlkDev *blks, const CpSched *sched, uint32_t *partial, uint32_t *pexp, DevTables t);
void launch_cp_finalize(hipStream_t s, int n, bool open, int crc_mode, const BlkDev *blks, const CpSched *sched,
                        const uint32_t *partial, const uint32_t *pexp, BlkOut *out);
void launch_crc_segments(hipStream_t s, int ntasks, const Task *tasks, const BlkDev *blks, DevTables t);
void launch_crc_finalize(hipStream_t s, int n, int crc_mode, const BlkDev *blks, BlkOut *out);
void launch_gen_synthetic(hipStream_t s, uint8_t *dst, uint64_t len, uint64_t seed, uint64_t block);
void launch_pull(hipStream_t s, void *dst, const void *src, size_t bytes);
void launch_gen_synthetic_batch(hipStream_t s, uint8_t *dst, uint64_t stride, int n, const uint64_t *lens,
                                uint64_t seed, uint64_t block0);
// tabs: n x 16 KiB of device memory, the blocks' LZ4 hash tables
constexpr size_t kLz4TabBytes = 16384;
void launch_lz4_compress(hipStream_t s, int n, int ncu, const ZDev *blks, ZOut *outs, uint32_t *tabs);
void launch_lz4_decompress(hipStream_t s, int n, const ZDev *blks, ZOut *outs);
// Zstandard frames (jfsx_zstd.hip): scratch = n x kZstdScratch bytes (literal
// buffer + the literal window's read-ahead, then a log-12 Huffman table)
constexpr size_t kZstdHufOff = 128 * 1024 + 320;
constexpr size_t kZstdScratch = kZstdHufOff + 8192;
// Block-parallel decoding (jfsx_zstd2.h): zstd_par_waves(n, ncu) persistent
// waves, each with a kZstdArena-byte arena (tables, literals, sequences);
// waves = 0 selects the serial one-wave-per-object kernel (n x kZstdScratch).
constexpr size_t kZstdArena = (size_t)64 * 9216 + ((size_t)4 << 20) + ((size_t)1 << 18) + (size_t)12 * (768u << 10);
constexpr int kZstdWavesPerCu = 8;
int zstd_par_waves(int n, int ncu);
void launch_zstd_decompress(hipStream_t s, int n, const ZDev *blks, ZOut *outs, uint8_t *scratch, int waves);
// Zstandard level-1 compression (jfsx_zstdc.hip): `waves` persistent
// one-wave workgroups take objects w, w + waves, ... (a uniform strided loop);
// each owns kZstdcScratch bytes of scratch (hash table, sequences, literals)
constexpr size_t kZstdcScratch = 960 * 1024;
constexpr size_t kZcScratchStride = kZstdcScratch;
constexpr int kZcWavesPerCu = 16;
void launch_zstd_compress(hipStream_t s, int n, int waves, const ZDev *blks, ZOut *outs, uint8_t *scratch,
                          uint32_t *queue);
// batched RSA-OAEP unwrap (jfsx_rsa.hip): key = device jfsx_rsa::Key
void async_detach(jfsx_ctx *c);  // jfsx_agg.cpp
void launch_rsa_unwrap(hipStream_t s, const void *key, int n, const uint8_t *ct, uint32_t *mh, uint8_t *em,
                       int32_t *len);
}  // namespace jfsx

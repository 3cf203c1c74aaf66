// jfsx_crc.hip -- CRC32C per 32 KiB segment over ranges (gfx950), and the
// synthetic-input generator.
//
// crc32c_segments replaces the CRC loops of checksum() (pkg/chunk/disk_cache.go:
// 1218-1231) and of cacheFile.ReadAt (disk_cache.go:1315-1327) for cache hits,
// none-cipher volumes and the staging re-read (pkg/chunk/cached_store.go:961-971).
// One wave per 32 KiB segment, 64 lanes x 16 B per row, slice-by-16 tables in
// LDS; lane CRCs are shifted to the segment end (GF(2) multiply by x^(8d) mod P)
// and XOR-reduced across the wave.
#include "jfsx_dev.h"

namespace jfsx {

// Slice-by-16 reads 20 random table dwords per 16 B; with one copy of each
// table, 32 lanes of random bytes land on the 32 LDS banks with ~3.5-way
// conflicts and the kernel is LDS-bound near 4.2 TB/s.  Here every byte lookup
// is split into its two nibble lookups (the tables are linear: T[b] =
// T[b & 15] ^ T[b & 240]) and each 16-entry nibble table is replicated 32x,
// one replica per bank, so lane l always reads bank l mod 32: conflict-free at
// twice the lookups.  A v_perm builds each address in one VALU op:
//   perm(x & 0x0f0f0f0f, lb) = (lo nibble of byte k) << 8 | lb
//   perm((x >> 4) & 0x0f0f0f0f, lb) = (hi nibble of byte k) << 8 | lb
// with lb = 4 * (lane mod 32) | 0x10000 (byte 2 of lb is selected for the
// tables above 64 KiB, past the ds_read offset field) and the table in the
// ds_read immediate: table t (lo) / t + 0.5 (hi) at t * 4096 + hi * 128, nibble
// stride 256 B -- 20 x 4 KiB = 80 KiB, two 16-wave workgroups per CU.
// Tables t = 0..15 are U0..U15 (slice-by-16); t = 16..19 shift a lane CRC by
// one 1 KiB row, so A' = S1024(A) ^ U(piece) and the 32 data lookups of a row
// do not wait for A.  Each workgroup stages the tables once per task (0.5 to
// 4 MiB) and every wave loops over segments.
// JFSX_CRC_SPAN = 64 (default): in whole segments a lane owns 64 contiguous
// bytes of every 4 KiB span (lane l: bytes 64l..64l+63), four 16-B pieces
// chained through the slice-by-16 state (crc ^ first word, no lookups between
// them), and the lane CRC moves from span to span by one 4096-B shift:
// A' = S4096(A) ^ crc_raw(0, chunk) -- 34 nibble lookups per 16 B instead of
// the 40 of the 16-B-per-lane rows (A' = S1024(A) ^ U(piece)).  Tables
// t = 16..19 in LDS are then the 4096-B shift; the guarded path (ragged
// segment ends) keeps 1 KiB rows and takes its 1024-B shift from global memory.
// JFSX_CRC_BYTE = 1: slice-by-4 byte tables U12..U15 replicated once per bank
// (table entry stride 256 B, two tables interleaved per 64 KiB: address =
// byte << 8 | 4 * (lane mod 32) | region << 16, one v_perm each) -- 16
// conflict-free lookups and about 28 VALU per 16 B instead of 34 and ~60,
// at 144 KiB of LDS (one 16-wave workgroup per CU).  A lane's 64-B chunk is a
// chain of 16 slice-by-4 steps; two spans' chains run interleaved, and the
// 4096-B span shift keeps its nibble tables (region 2).
// default since round 4: byte tables (JFSX_CRC_BYTE = 1) with quad-transposed
// coalesced loads (JFSX_CRC_XPOSE = 1), 6.03-6.05 TB/s at 64 GiB against 5.33
// for the nibble kernel on the same box (profiles/r4/ab_crc.txt)
#ifndef JFSX_CRC_BYTE
#define JFSX_CRC_BYTE 1
#endif
#ifndef JFSX_CRC_SPAN
#define JFSX_CRC_SPAN 64
#endif
constexpr uint32_t kCrcWaves = 16;
#ifndef JFSX_CRC_PF
#define JFSX_CRC_PF 4
#endif
constexpr int kCrcPf = JFSX_CRC_PF;  // rows of 16 B per lane in flight
#if JFSX_CRC_BYTE
constexpr uint32_t kCrcLds = 0x24000;  // 147456 B: byte tables 128 KiB + shift nibble tables 16 KiB
#else
constexpr uint32_t kCrcLds = 20 * 4096;  // 81920 B
#endif

#define NIB(t, h, xm, k)                                                                                          \
    lds_u32(lds, __builtin_amdgcn_perm((xm), lb, ((t) >= 16 ? 0x0c020000u : 0x0c0c0000u) | ((4u + (k)) << 8)) + \
                     (((t)&15) * 4096u + (h)*128u))
#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)

// the 8 nibble lookups of word x through tables t..t+3
__device__ __forceinline__ uint32_t crc_word_nib(const char *lds, uint32_t lb, uint32_t t, uint32_t x) {
    const uint32_t xl = x & 0x0f0f0f0fu, xh = (x >> 4) & 0x0f0f0f0fu;
    return X3(X3(NIB(t, 0, xl, 0), NIB(t, 1, xh, 0), NIB(t + 1, 0, xl, 1)),
              X3(NIB(t + 1, 1, xh, 1), NIB(t + 2, 0, xl, 2), NIB(t + 2, 1, xh, 2)),
              NIB(t + 3, 0, xl, 3) ^ NIB(t + 3, 1, xh, 3));
}

// A advanced over one 1 KiB row whose lane piece is p:
// crc_raw(shift(A, 1008 B), p) = shift(A, 1024 B) ^ crc_raw(0, p)
__device__ __forceinline__ uint32_t crc_row_nib(const char *lds, uint32_t lb, uint32_t A, uint4 p) {
    const uint32_t d = X3(crc_word_nib(lds, lb, 0, p.x), crc_word_nib(lds, lb, 4, p.y), crc_word_nib(lds, lb, 8, p.z)) ^
                       crc_word_nib(lds, lb, 12, p.w);
    return crc_word_nib(lds, lb, 16, A) ^ d;
}
#undef X3

// crc_raw(0, 16-byte piece p) through the LDS nibble tables U0..U15
__device__ __forceinline__ uint32_t crc_u16_nib(const char *lds, uint32_t lb, uint32_t x, uint32_t y, uint32_t z,
                                                uint32_t w) {
#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
    return X3(crc_word_nib(lds, lb, 0, x), crc_word_nib(lds, lb, 4, y), crc_word_nib(lds, lb, 8, z)) ^
           crc_word_nib(lds, lb, 12, w);
#undef X3
}

#ifndef JFSX_CRC_CHAINS
#define JFSX_CRC_CHAINS 2
#endif
#ifndef JFSX_CRC_XPOSE
#define JFSX_CRC_XPOSE 1
#endif
// the lane's 64-byte chunk of span r of a segment: piece j.  XPOSE = 0: lane l
// owns bytes 64l..64l+63 (each load instruction touches 32 cache lines, 32 B
// of each).  XPOSE = 1: instruction j loads the span's bytes 1024j + 16l
// (one fully coalesced 1 KiB row, 8 whole lines); after quad_xpose lane
// l = 4m + t holds the chunk at 64 (16t + m) of the span.
// JFSX_CRC_NT = 1: the loads carry the non-temporal hint (the data is read
// once; A/B in profiles/r4/ab_crc.txt)
#ifndef JFSX_CRC_NT
#define JFSX_CRC_NT 1
#endif
__device__ __forceinline__ uint4 crc_ld16(const uint8_t *p) { return JFSX_CRC_NT ? gld16_nt(p) : gld16(p); }
__device__ __forceinline__ uint4 crc_chunk_ld(const uint8_t *seg, uint32_t lane, int r, int j) {
    return JFSX_CRC_XPOSE ? crc_ld16(seg + 4096 * r + 1024 * j + 16 * lane) : crc_ld16(seg + 4096 * r + 64 * lane + 16 * j);
}
// lane chunk index within a span (the final shift to the segment end)
__device__ __forceinline__ uint32_t crc_chunk_idx(uint32_t lane) {
    return JFSX_CRC_XPOSE ? 16u * (lane & 3u) + (lane >> 2) : lane;
}
// 4 x 4 transpose of 16-byte pieces across the 4 lanes of a quad: afterwards
// v[i] of lane t is what v[t] of lane i held.  Two butterfly stages (lane bit
// 0, then bit 1), each a DPP quad swap of the piece the partner needs.
__device__ __forceinline__ uint32_t dpp_swap(uint32_t x, int ctrl) {
    return ctrl == 0xB1 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true)
                        : (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
}
__device__ __forceinline__ void xpose_stage(uint32_t &a, uint32_t &b, bool odd, int ctrl) {
    const uint32_t r = dpp_swap(odd ? a : b, ctrl);
    a = odd ? r : a;
    b = odd ? b : r;
}
__device__ __forceinline__ void quad_xpose(uint4 (&v)[4], uint32_t lane) {
    const bool o1 = lane & 1u, o2 = lane & 2u;
#define XS(f)                                 \
    xpose_stage(v[0].f, v[1].f, o1, 0xB1);    \
    xpose_stage(v[2].f, v[3].f, o1, 0xB1);    \
    xpose_stage(v[0].f, v[2].f, o2, 0x4E);    \
    xpose_stage(v[1].f, v[3].f, o2, 0x4E);
    XS(x) XS(y) XS(z) XS(w)
#undef XS
}
#if JFSX_CRC_BYTE
// byte k of x through U(12 + k): region k >> 1 (lb byte 2 = 1), half k & 1
#define BYT(x, k)                                                                                              \
    lds_u32(lds, __builtin_amdgcn_perm((x), lb, 0x0c000000u | ((k) >= 2 ? 0x00020000u : 0x000c0000u) |        \
                                                    ((4u + (k)) << 8)) +                                       \
                     ((k)&1) * 128u)
// 4096-B shift nibble tables in region 2 (lb byte 3 = 2)
#define NIBS(t, h, xm) lds_u32(lds, __builtin_amdgcn_perm((xm), lb, 0x0c030000u | ((4u + (t)) << 8)) + ((t)*4096u + (h)*128u))
#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
// one slice-by-4 step: crc_raw of the 4 bytes of x (= state ^ word)
__device__ __forceinline__ uint32_t crc_step4(const char *lds, uint32_t lb, uint32_t x) {
    return X3(BYT(x, 0), BYT(x, 1), BYT(x, 2)) ^ BYT(x, 3);
}
// crc_raw of the 4 bytes of x, XORed with w
__device__ __forceinline__ uint32_t crc_step4x(const char *lds, uint32_t lb, uint32_t x, uint32_t w) {
    return X3(X3(BYT(x, 0), BYT(x, 1), BYT(x, 2)), BYT(x, 3), w);
}
__device__ __forceinline__ uint32_t crc_shift4096(const char *lds, uint32_t lb, uint32_t A) {
    const uint32_t xl = A & 0x0f0f0f0fu, xh = (A >> 4) & 0x0f0f0f0fu;
    return X3(X3(NIBS(0, 0, xl), NIBS(0, 1, xh), NIBS(1, 0, xl)), X3(NIBS(1, 1, xh), NIBS(2, 0, xl), NIBS(2, 1, xh)),
              NIBS(3, 0, xl) ^ NIBS(3, 1, xh));
}
#undef X3
__device__ __forceinline__ uint32_t crc_u16_byte(const char *lds, uint32_t lb, uint4 p) {
    uint32_t c = crc_step4(lds, lb, p.x);
    c = crc_step4(lds, lb, c ^ p.y);
    c = crc_step4(lds, lb, c ^ p.z);
    return crc_step4(lds, lb, c ^ p.w);
}
#endif

// the guarded path's row step with the 1024-B shift from global byte tables
__device__ __forceinline__ uint32_t crc_row_g(const char *lds, const uint32_t *__restrict__ T, uint32_t lb, uint32_t A,
                                              uint4 p) {
    const uint32_t s = T[24 * 256 + (A & 0xffu)] ^ T[25 * 256 + ((A >> 8) & 0xffu)] ^
                       T[26 * 256 + ((A >> 16) & 0xffu)] ^ T[27 * 256 + (A >> 24)];
#if JFSX_CRC_BYTE
    return crc_u16_byte(lds, lb, p) ^ s;
#else
    return crc_u16_nib(lds, lb, p.x, p.y, p.z, p.w) ^ s;
#endif
}

// ragged tails (segment length not a multiple of 16 B: the last segment of an
// odd-sized block only) read the byte tables from global memory:
// crc_raw(shift(A, 1008 B), first n bytes of p)
__device__ __noinline__ uint32_t crc_partial_g(const uint32_t *__restrict__ T, uint32_t A, const uint32_t p[4], int n) {
    uint32_t c = T[16 * 256 + (A & 0xffu)] ^ T[17 * 256 + ((A >> 8) & 0xffu)] ^ T[18 * 256 + ((A >> 16) & 0xffu)] ^
                 T[19 * 256 + (A >> 24)];
    for (int i = 0; i < n; i++) {
        const uint32_t byte = (p[i >> 2] >> (8 * (i & 3))) & 0xffu;
        c = T[15 * 256 + ((c ^ byte) & 0xffu)] ^ (c >> 8);
    }
    return c;
}

#ifndef JFSX_CRC_WPE
#define JFSX_CRC_WPE (JFSX_CRC_BYTE ? 4 : 8)
#endif
__global__ __launch_bounds__(kCrcWaves * 64) __attribute__((amdgpu_waves_per_eu(JFSX_CRC_WPE))) void crc_segments_k(const Task *__restrict__ tasks,
                                                                const BlkDev *__restrict__ blks, DevTables tab) {
    __shared__ __attribute__((aligned(16))) char lds[kCrcLds];
    const Task task = tasks[blockIdx.x];
    const BlkDev blk = blks[task.blk];
    const uint32_t tid = threadIdx.x;
#if JFSX_CRC_BYTE
    // stage: byte tables U12..U15, i = (table t, entry e, replica quad rq)
    for (uint32_t i = tid; i < 4 * 256 * 8; i += kCrcWaves * 64) {
        const uint32_t rq = i & 7, e = (i >> 3) & 255, t = i >> 11;
        const uint32_t v = tab.crc[(12 + t) * 256 + e];
        *reinterpret_cast<uint4 *>(lds + (t >> 1) * 0x10000u + e * 256 + (t & 1) * 128 + 16 * rq) =
            make_uint4(v, v, v, v);
    }
    // the 4096-B shift as nibble tables in region 2: i = (table t, hi, nibble, rq)
    for (uint32_t i = tid; i < 4 * 2 * 16 * 8; i += kCrcWaves * 64) {
        const uint32_t rq = i & 7, nib = (i >> 3) & 15, hi = (i >> 7) & 1, t = i >> 8;
        const uint32_t v = tab.crc[(28 + t) * 256 + (hi ? nib << 4 : nib)];
        *reinterpret_cast<uint4 *>(lds + 0x20000u + t * 4096 + nib * 256 + hi * 128 + 16 * rq) =
            make_uint4(v, v, v, v);
    }
    __syncthreads();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const uint32_t lb = ((lane & 31) << 2) | 0x10000u | 0x2000000u;
#else
    // stage: i = (table t, hi, nibble, replica quad rq)
    for (uint32_t i = tid; i < 640 * 8; i += kCrcWaves * 64) {
        const uint32_t rq = i & 7, nib = (i >> 3) & 15, hi = (i >> 7) & 1, t = i >> 8;
        const uint32_t v = tab.crc[(t < 16 ? t : t + (JFSX_CRC_SPAN >= 64 ? 12 : 8)) * 256 + (hi ? nib << 4 : nib)];
        *reinterpret_cast<uint4 *>(lds + t * 4096 + nib * 256 + hi * 128 + 16 * rq) = make_uint4(v, v, v, v);
    }
    __syncthreads();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const uint32_t lb = ((lane & 31) << 2) | 0x10000u;
#endif
    const uint8_t *src = blk.src;
    for (uint64_t seg0 = task.c0 + (uint64_t)wave * kSeg; seg0 < task.c1; seg0 += (uint64_t)kCrcWaves * kSeg) {
        const uint64_t seg1 = seg0 + kSeg < task.c1 ? seg0 + kSeg : task.c1;
        uint32_t A = 0, lend = 0;
        const uint64_t nrows = (seg1 - seg0 + 1023) / 1024;
        if (JFSX_CRC_BYTE && seg1 - seg0 == (uint64_t)kSeg) {
#if JFSX_CRC_BYTE
            // full segment, 64-B lane chunks of the 8 spans of 4 KiB; CH spans
            // are CH independent slice-by-4 chains, and each piece's load for
            // the span CH further on is issued as soon as the piece is consumed
            constexpr int CH = JFSX_CRC_CHAINS;
            uint4 buf[CH][4];
#pragma unroll
            for (int k = 0; k < CH; k++)
#pragma unroll
                for (int j = 0; j < 4; j++) buf[k][j] = crc_chunk_ld(src + seg0, lane, k, j);
#pragma unroll
            for (int r = 0; r < 8; r += CH) {
                if (JFSX_CRC_XPOSE) {
#pragma unroll
                    for (int k = 0; k < CH; k++) quad_xpose(buf[k], lane);
                }
                // x = state ^ next word; each step folds the next word into
                // its 4-way XOR (two v_bitop3)
                uint32_t x[CH];
#pragma unroll
                for (int k = 0; k < CH; k++) x[k] = buf[k][0].x;
#pragma unroll
                for (int j = 0; j < 4; j++) {
#pragma unroll
                    for (int k = 0; k < CH; k++) x[k] = crc_step4x(lds, lb, x[k], buf[k][j].y);
#pragma unroll
                    for (int k = 0; k < CH; k++) x[k] = crc_step4x(lds, lb, x[k], buf[k][j].z);
                    if (j < 3) {
#pragma unroll
                        for (int k = 0; k < CH; k++) x[k] = crc_step4x(lds, lb, x[k], buf[k][j].w);
#pragma unroll
                        for (int k = 0; k < CH; k++) x[k] = crc_step4x(lds, lb, x[k], buf[k][j + 1].x);
                    } else {
#pragma unroll
                        for (int k = 0; k < CH; k++) x[k] = crc_step4x(lds, lb, x[k], buf[k][j].w);
                    }
                    // piece j of every chain consumed (its .x was read one step ago)
                    if (r + CH < 8 && j > 0) {
#pragma unroll
                        for (int k = 0; k < CH; k++) buf[k][j - 1] = crc_chunk_ld(src + seg0, lane, r + CH + k, j - 1);
                    }
                }
                if (r + CH < 8) {
#pragma unroll
                    for (int k = 0; k < CH; k++) buf[k][3] = crc_chunk_ld(src + seg0, lane, r + CH + k, 3);
                }
#pragma unroll
                for (int k = 0; k < CH; k++) A = crc_step4x(lds, lb, x[k], crc_shift4096(lds, lb, A));
            }
            lend = kSeg;
#endif
        } else if (!JFSX_CRC_BYTE && JFSX_CRC_SPAN >= 64 && seg1 - seg0 == (uint64_t)kSeg) {
            // full segment: spans of 64 x SPAN bytes, lane chunk SPAN bytes
            // (P pieces); each piece's load for the next span is issued as
            // soon as the piece is consumed
            constexpr int P = JFSX_CRC_SPAN / 16, NSP = 32768 / (64 * JFSX_CRC_SPAN);
            const uint8_t *q = src + seg0 + JFSX_CRC_SPAN * lane;
            static_assert(!JFSX_CRC_XPOSE || JFSX_CRC_SPAN == 64, "quad transpose needs 64-B lane chunks");
            uint4 buf[P];
#pragma unroll
            for (int j = 0; j < P; j++) buf[j] = JFSX_CRC_XPOSE ? crc_chunk_ld(src + seg0, lane, 0, j) : gld16(q + 16 * j);
#pragma unroll
            for (int r = 0; r < NSP; r++) {
                uint32_t c = 0;
#if JFSX_CRC_XPOSE
                quad_xpose(buf, lane);
#endif
#pragma unroll
                for (int j = 0; j < P; j++) {
                    const uint4 p = buf[j];
                    if (r + 1 < NSP)
                        buf[j] = JFSX_CRC_XPOSE ? crc_chunk_ld(src + seg0, lane, r + 1, j)
                                                : gld16(q + 64 * JFSX_CRC_SPAN * (r + 1) + 16 * j);
                    c = crc_u16_nib(lds, lb, p.x ^ c, p.y, p.z, p.w);
                }
                A = crc_word_nib(lds, lb, 16, A) ^ c;
            }
            lend = kSeg;  // marker: lane chunk ends at 32768 - SPAN * (63 - lane)
        } else if (JFSX_CRC_SPAN < 64 && seg1 - seg0 == (uint64_t)kSeg) {
            // full segment: 32 rows, kCrcPf loads in flight per wave (HBM
            // latency x 8 TB/s needs ~64 KiB in flight per CU)
            const uint8_t *q = src + seg0 + 16 * lane;
            uint4 buf[kCrcPf];
#pragma unroll
            for (int r = 0; r < kCrcPf; r++) buf[r] = gld16(q + 1024 * r);
#pragma unroll
            for (int r = 0; r < 32; r++) {
                const uint4 p = buf[r % kCrcPf];
                if (r + kCrcPf < 32) buf[r % kCrcPf] = gld16(q + 1024 * (r + kCrcPf));
                A = crc_row_nib(lds, lb, A, p);
            }
            lend = kSeg - 1024 + 16 * lane + 16;
        } else {
            for (uint64_t r = 0; r < nrows; r++) {
                const uint64_t o = seg0 + 1024 * r + 16 * lane;
                const uint4 p = load_piece(src, o, seg1);
                if (o + 16 <= seg1) {
                    A = JFSX_CRC_SPAN >= 64 ? crc_row_g(lds, tab.crc, lb, A, p) : crc_row_nib(lds, lb, A, p);
                    lend = (uint32_t)(o + 16 - seg0);
                } else if (o < seg1) {
                    const uint32_t pw[4] = {p.x, p.y, p.z, p.w};
                    A = crc_partial_g(tab.crc, A, pw, (int)(seg1 - o));
                    lend = (uint32_t)(seg1 - seg0);
                }
            }
        }
        const uint32_t Lseg = (uint32_t)(seg1 - seg0);
        uint32_t v, K;
        if (Lseg == (uint32_t)kSeg) {
            if (JFSX_CRC_SPAN >= 64) {
                // lane chunk end to segment end: SPAN * (63 - lane) bytes =
                // crcx[128 + lane] (64 * (63 - lane) bytes) squared SPAN / 64 - 1 times
                uint32_t x = tab.crcx[128 + crc_chunk_idx(lane)];
                for (int k = 64; k < JFSX_CRC_SPAN; k <<= 1) x = crc_mulmod(x, x);
                v = crc_mulmod(x, A);
            } else {
                v = crc_mulmod(tab.crcx[lane], A);
            }
            K = tab.crcx[96];
        } else {
            v = crc_mulmod(crc_xpow8(Lseg - lend, tab.crcx + 64), A);
            K = crc_mulmod(crc_xpow8(Lseg, tab.crcx + 64), 0xffffffffu);
        }
        const uint32_t raw = wave_xor(v);
        if (lane == 0) {
            const uint32_t crc = ~(K ^ raw);
            const uint64_t si = seg0 / kSeg;
            if (blk.crc_calc)
                blk.crc_calc[si] = crc;
            else
                *reinterpret_cast<uint32_t *>(blk.crc + 4 * si) = __builtin_bswap32(crc);
        }
    }
}

// zero-length ranges/blocks still produce one zero CRC (Go's checksum(): 4 bytes)
__global__ __launch_bounds__(64) void crc_finalize_k(const BlkDev *__restrict__ blks, int crc_mode,
                                                    BlkOut *__restrict__ out) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const BlkDev blk = blks[b];
    BlkOut o;
    for (int q = 0; q < 4; q++) o.tag[q] = 0;
    o.status = JFSX_OK;
    o.bad_seg = -1;
    o.got = o.expect = 0;
    if (crc_mode == JFSX_CRC_GEN && blk.len == 0 && lane == 0) *reinterpret_cast<uint32_t *>(blk.crc) = 0;
    if (crc_mode == JFSX_CRC_VERIFY) {
        crc_verify_block(blk, o, lane);
        if (o.bad_seg >= 0) o.status = JFSX_ECRC;
    }
    if (lane == 0) out[b] = o;
}

// SplitMix64 stream: word k of block b = mix64(seed + G*((b << 40) + k + 1))
// (identical to oracle/jfs_oracle.c orc_gen_block)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void gen_synthetic_k(uint8_t *__restrict__ dst, uint64_t len, uint64_t seed,
                                                      uint64_t block) {
    const uint64_t G = 0x9E3779B97F4A7C15ULL;
    const uint64_t nw2 = len / 16;
    const uint64_t base = seed + G * ((block << 40) + 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw2;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = mix64(base + G * (2 * i)), b = mix64(base + G * (2 * i + 1));
        *reinterpret_cast<ulonglong2 *>(dst + 16 * i) = make_ulonglong2(a, b);
    }
    if (blockIdx.x == 0 && threadIdx.x < 16) {
        const uint64_t i = nw2 * 16 + threadIdx.x;
        if (i < len) {
            const uint64_t w = mix64(base + G * (i / 8));
            dst[i] = (uint8_t)(w >> (8 * (i % 8)));
        }
    }
}

// batched generator: grid (x = workgroups per block, y = block), block i of
// the batch is the stream of global block block0 + i, lens[i] bytes at
// dst + i * stride (one launch for a whole bench batch)
__global__ __launch_bounds__(256) void gen_synthetic_batch_k(uint8_t *__restrict__ dst, uint64_t stride,
                                                            const uint64_t *__restrict__ lens, uint64_t seed,
                                                            uint64_t block0) {
    const uint64_t G = 0x9E3779B97F4A7C15ULL;
    const uint32_t bi = blockIdx.y;
    const uint64_t len = lens[bi];
    uint8_t *d = dst + stride * bi;
    const uint64_t nw2 = len / 16;
    const uint64_t base = seed + G * (((block0 + bi) << 40) + 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw2;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = mix64(base + G * (2 * i)), b = mix64(base + G * (2 * i + 1));
        *reinterpret_cast<ulonglong2 *>(d + 16 * i) = make_ulonglong2(a, b);
    }
    if (blockIdx.x == 0 && threadIdx.x < 16) {
        const uint64_t i = nw2 * 16 + threadIdx.x;
        if (i < len) {
            const uint64_t w = mix64(base + G * (i / 8));
            d[i] = (uint8_t)(w >> (8 * (i % 8)));
        }
    }
}

// dst[0, bytes) = src[0, bytes) for a small region (a pipeline group's
// descriptors) read by the GPU straight out of pinned host memory, which the
// host rewrote since the previous group: system-scope loads, so no cache level
// can hand back the previous group's words.  bytes is a multiple of 4.
__global__ __launch_bounds__(256) void pull_k(uint32_t *__restrict__ dst, uint32_t *__restrict__ src, uint32_t n4) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256)
        dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

void launch_pull(hipStream_t s, void *dst, const void *src, size_t bytes) {
    const uint32_t n4 = (uint32_t)(bytes / 4);
    if (!n4) return;
    const uint32_t grid = (n4 + 255) / 256 < 128 ? (n4 + 255) / 256 : 128;
    hipLaunchKernelGGL(pull_k, dim3(grid), dim3(256), 0, s, (uint32_t *)dst, (uint32_t *)src, n4);
}

void launch_gen_synthetic_batch(hipStream_t s, uint8_t *dst, uint64_t stride, int n, const uint64_t *lens,
                                uint64_t seed, uint64_t block0) {
    // y <= 65535 blocks per launch
    for (int i0 = 0; i0 < n; i0 += 65535) {
        const int m = n - i0 < 65535 ? n - i0 : 65535;
        hipLaunchKernelGGL(gen_synthetic_batch_k, dim3(16, (unsigned)m), dim3(256), 0, s, dst + stride * i0, stride,
                           lens + i0, seed, block0 + i0);
    }
}

void launch_crc_segments(hipStream_t s, int ntasks, const Task *tasks, const BlkDev *blks, DevTables t) {
    if (ntasks > 0) hipLaunchKernelGGL(crc_segments_k, dim3(ntasks), dim3(kCrcWaves * 64), 0, s, tasks, blks, t);
}

void launch_crc_finalize(hipStream_t s, int n, int crc_mode, const BlkDev *blks, BlkOut *out) {
    if (n > 0) hipLaunchKernelGGL(crc_finalize_k, dim3(n), dim3(64), 0, s, blks, crc_mode, out);
}

void launch_gen_synthetic(hipStream_t s, uint8_t *dst, uint64_t len, uint64_t seed, uint64_t block) {
    uint64_t nw2 = len / 16;
    uint64_t blocks = (nw2 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(gen_synthetic_k, dim3((unsigned)blocks), dim3(256), 0, s, dst, len, seed, block);
}

}  // namespace jfsx

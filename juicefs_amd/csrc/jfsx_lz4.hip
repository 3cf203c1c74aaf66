// jfsx_lz4.hip -- LZ4 block compression / decompression (gfx950), the
// compression stage of the compressed block path.
//
// Replaces, per block, LZ4.Compress = lz4.CompressDefault(src, dst) and
// LZ4.Decompress = lz4.DecompressSafe(src, dst) (pkg/compress/compress.go:
// 107-125, github.com/hungys/go-lz4 over the LZ4 C library), called by
// cachedStore.upload before the object is put (pkg/chunk/cached_store.go:
// 371-392: dst sized CompressBound(len)) and by cachedStore.load after the
// object is read (:680-745).  Output bytes are those of LZ4_compress_default
// (acceleration 1) and the accept/reject rules of LZ4_decompress_safe, as
// restated in oracle/jfs_lz4.c and pinned there against liblz4.
//
// The greedy LZ4 parse is sequential per block, so a block is one wave and
// the wave's 64 lanes work on the parse together (no MFMA, no cross-block
// state; blocks shard like the AEAD blocks):
//   * match search: the compressor probes positions ip, ip+1, ... with a step
//     that grows by one every 64 misses.  Those positions depend only on the
//     search start, so a wave evaluates 64 probes at once (lane j = probe
//     k0 + j): hash, hash-table read, distance check, 4-byte compare.  Probes
//     of the same batch that share a hash bucket see each other's table
//     writes in probe order (13 ballots give each lane the lanes of its
//     bucket); the first succeeding probe ends the search and only the probes
//     before it write the table, last writer per bucket.
//   * backward extension, match-length count, literal and 255-run copies:
//     64 (or 256) bytes per step with a ballot for the first difference.
//   * the 16 KiB hash table (4096 x u32 for inputs >= 64 KiB + 11 B, else
//     8192 x u16) lives in LDS: 10 waves per CU.
// The decompressor parses tokens from a 256-byte window of the input held in
// the wave's VGPRs (one dword per lane, read back with v_readlane) and copies
// literals / matches 64 bytes per step into an LDS ring of the recent output,
// which leaves for global memory in coalesced 1 KiB wave stores; a match reads
// only output written before it (overlapping matches are expanded as
// out[op+i] = out[op-off+i%off]), from the ring, or from global memory once
// the wave's stores of it have completed (s_waitcnt vmcnt(0)).
#include <string.h>

#include "jfsx_dev.h"

// TabL::put as one masked LDS write (ds_mskor_b32) instead of an and / or
// atomic pair; -DJFSX_LZ4_MSKOR=0 builds the pair (A/B)
#ifndef JFSX_LZ4_MSKOR
#define JFSX_LZ4_MSKOR 1
#endif

namespace jfsx {

namespace {

constexpr uint32_t kMinMatch = 4, kMfLimit = 12, kLastLit = 5, kLimit64K = 65536 + kMfLimit - 1;

typedef __attribute__((address_space(1))) const uint32_t gcu32;
typedef __attribute__((address_space(1))) const uint8_t gcu8;
typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ uint32_t ld32a(const uint8_t *p) { return *(gcu32 *)p; }
__device__ __forceinline__ uint32_t ld8(const uint8_t *p) { return *(gcu8 *)p; }
__device__ __forceinline__ void st8(uint8_t *p, uint32_t v) { *(gu8 *)p = (uint8_t)v; }

// 4 bytes at any address: two aligned dword loads, each holding at least one
// of the requested bytes (so neither touches a page the bytes are not on)
__device__ __forceinline__ uint32_t ld32u(const uint8_t *a) {
    const uintptr_t x = (uintptr_t)a;
    const uint8_t *b = (const uint8_t *)(x & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(x & 3);
    const uint32_t w0 = ld32a(b), w1 = ld32a(sh ? b + 4 : b);
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
}

__device__ __forceinline__ uint32_t lz_hash(const uint8_t *p, bool small) {
    const uint32_t w = ld32u(p);
    if (small) return (w * 2654435761u) >> (32 - 13);
    const uint64_t v = (uint64_t)w | ((uint64_t)ld8(p + 4) << 32);  // LZ4_hash5: the read's low 5 bytes
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - 12));
}

// offset of probe k from the search start: steps 1 (probes 0..64), then
// (63 + t) >> 6 for probe t (LZ4_skipTrigger = 6)
__device__ __forceinline__ uint32_t probe_off(uint32_t k) {
    if (k == 0) return 0;
    const uint32_t m = 62 + k, q = m >> 6, r = m & 63;
    return 1 + 32 * q * (q - 1) + (r + 1) * q;
}

__device__ __forceinline__ uint64_t ballot(bool b) { return __ballot(b); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// lanes below / above this one
__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// dst[0, len) = src[0, len); src and dst do not overlap.  16-byte stores on
// 16-byte aligned destination units (head and tail byte-wise), each unit from
// one dword-aligned 16-byte load plus, when src and dst disagree modulo 4,
// the next dword (never a dword without a source byte: page-safe); four
// 1 KiB wave steps in flight per round.
__device__ void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t len, uint32_t lane) {
    typedef __attribute__((address_space(1))) v4u gv4;
    typedef __attribute__((address_space(1))) const v4u gcv4;
    uint32_t head = (uint32_t)(-(uintptr_t)dst & 15);
    if (head > len) head = len;
    if (lane < head) st8(dst + lane, ld8(src + lane));
    uint32_t i = head;
    const uintptr_t sx = (uintptr_t)(src + i);
    const uint32_t sh = (uint32_t)(sx & 3);
    const uint8_t *sa = (const uint8_t *)(sx & ~(uintptr_t)3);  // src + i - sh
    uint8_t *d = dst + i;
    auto unit = [&](uint32_t o) {  // 16 bytes at d + o from sa + o
        const v4u v = *(gcv4 *)(sa + o);
        v4u r;
        if (sh) {
            const uint32_t e = ld32a(sa + o + 16);
            r.x = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
            r.y = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
            r.z = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
            r.w = __builtin_amdgcn_alignbyte(e, v.w, sh);
        } else {
            r = v;
        }
        *(gv4 *)(d + o) = r;
    };
    const uint32_t body = len - i;
    uint32_t o = 0;
    for (; o + 4096 <= body; o += 4096) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) unit(o + 1024 * k + 16 * lane);
    }
    for (; o + 16 <= body; o += 1024)
        if (o + 16 * lane + 16 <= body) unit(o + 16 * lane);
    o = body & ~15u;
    if (lane < body - o) st8(d + o + lane, ld8(src + i + o + lane));
}

__device__ void wave_fill255(uint8_t *dst, uint32_t cnt, uint32_t lane) {
    for (uint32_t j = lane; j < cnt; j += 64) st8(dst + j, 255u);
}

// literal or match length continuation: (v - 15) as 255-runs plus the rest
__device__ __forceinline__ uint32_t put_len(uint8_t *dst, uint32_t op, uint32_t v, uint32_t lane) {
    const uint32_t runs = v / 255;
    wave_fill255(dst + op, runs, lane);
    if (lane == 0) st8(dst + op + runs, v % 255);
    return op + runs + 1;
}

}  // namespace

namespace {

// The block as an aligned image: input byte pos sits at image offset pos + sh
// of al = src rounded down to 4 (all offsets 32-bit scalars).
struct Img {
    const uint8_t *al;
    uint32_t sh, n;
};

// 256 bytes of the input in the wave's VGPRs: lane L holds the image dword at
// w0 + 4L (zero past the block end).  Reads inside it cost a v_readlane
// (uniform position) or a ds_bpermute (per-lane position), not a memory trip.
struct IWin {
    uint32_t w0;
    uint32_t w;
};

__device__ __forceinline__ void iwin_load(IWin &W, const Img &I, uint32_t pos, uint32_t lane) {
    W.w0 = (pos + I.sh) & ~3u;
    const uint32_t o = W.w0 + 4 * lane;
    W.w = o < I.n + I.sh ? ld32a(I.al + o) : 0u;
}
// [pos, pos + len) inside the window (uniform)
__device__ __forceinline__ bool iwin_has(const IWin &W, const Img &I, uint32_t pos, uint32_t len) {
    const uint32_t x = pos + I.sh;
    return x >= W.w0 && x + len <= W.w0 + 256u;
}
// 4 bytes at pos and the byte at pos + 4, uniform pos inside the window
__device__ __forceinline__ uint32_t iwin_u32(const IWin &W, const Img &I, uint32_t pos, uint32_t &b4) {
    const uint32_t r = pos + I.sh - W.w0, i = r >> 2, sh = r & 3;
    const uint32_t d0 = __builtin_amdgcn_readlane(W.w, i), d1 = __builtin_amdgcn_readlane(W.w, i + 1);
    b4 = (d1 >> (8 * sh)) & 255u;
    return __builtin_amdgcn_alignbyte(d1, d0, sh);
}
// the same for a per-lane pos (ds_bpermute)
__device__ __forceinline__ uint32_t iwin_u32_lane(const IWin &W, const Img &I, uint32_t pos, uint32_t &b4) {
    const uint32_t r = pos + I.sh - W.w0, i = r >> 2, sh = r & 3;
    const uint32_t d0 = __shfl(W.w, (int)i, 64), d1 = __shfl(W.w, (int)(i + 1), 64);
    b4 = (d1 >> (8 * sh)) & 255u;
    return __builtin_amdgcn_alignbyte(d1, d0, sh);
}

__device__ __forceinline__ uint32_t hash_of(uint32_t w, uint32_t b4, bool small) {
    if (small) return (w * 2654435761u) >> (32 - 13);
    const uint64_t v = (uint64_t)w | ((uint64_t)b4 << 32);
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - 12));
}

// dst[0, len) = input [pos, pos + len) from the window (len <= 256)
__device__ __forceinline__ void iwin_copy(uint8_t *dst, const IWin &W, const Img &I, uint32_t pos, uint32_t len,
                                          uint32_t lane) {
    const uint32_t r = pos + I.sh - W.w0;
    for (uint32_t k = 0; k < 4 && 64 * k < len; k++) {  // literal runs are short: one pass, mostly
        const uint32_t j = lane + 64 * k, q = r + j;
        const uint32_t d = __shfl(W.w, (int)((q >> 2) & 63), 64);
        if (j < len) st8(dst + j, (d >> (8 * (q & 3))) & 255u);
    }
}

// Match length beyond MINMATCH at (ip, match): LZ4_count(ip + 4, match + 4,
// matchlimit).  Loads the window C at ip + 4 (input side) and, in the same
// round of loads, the catch-up bytes before ip / match (limc <= 64 of them;
// back = equal bytes found, 64 when all were equal).  Returns mc.  With
// skip = 0 the count starts at ip itself: the result is the number of equal
// bytes from (ip, match), so the 4-byte test read32(match) == read32(ip) and
// the count share one round of loads (result >= 4 <=> the test holds).
__device__ uint32_t count_and_back(IWin &C, const Img &I, const uint8_t *src, uint32_t ip, uint32_t match,
                                   uint32_t matchlimit, uint32_t limc, uint32_t &back, uint32_t lane,
                                   uint32_t skip = kMinMatch) {
    const uint32_t aa = ip + skip, off = ip - match;
    iwin_load(C, I, aa, lane);
    const uint32_t lp = C.w0 + 4 * lane - I.sh;  // input position of this lane's first window byte (may wrap below 0 on lane 0)
    const uint32_t mp = lp - off;
    // with skip = 0 and a match in the block's first 3 bytes, lane 0's match
    // dword starts before byte 0: read the block's first dword shifted up
    // (the bytes below 0 face input bytes before aa and are not compared)
    const int32_t mps = (int32_t)mp;
    const uint32_t mw = mps < 0 ? ld32u(src) << (8 * (uint32_t)(-mps)) : ld32u(src + (mp + 4 <= I.n ? mp : I.n - 4));
    bool ceq = false;
    if (lane < limc) ceq = ld8(src + ip - 1 - lane) == ld8(src + match - 1 - lane);
    const uint64_t cst = ballot(!ceq);
    back = cst ? (uint32_t)__builtin_ctzll(cst) : 64u;
    // first byte i of this lane's 4 that stops the count: at or after aa, and
    // differing or at or past matchlimit (k: bytes before aa, lane 0 only, <= 3)
    const int32_t k = (int32_t)(aa - lp), m = (int32_t)(matchlimit - lp);
    const uint32_t pre = k > 0 ? (0xffffffffu << (8 * (uint32_t)k)) : 0xffffffffu;
    const uint32_t lim = m >= 4 ? 0u : (m <= 0 ? 0xffffffffu : (0xffffffffu << (8 * (uint32_t)m)));
    const uint32_t y = ((C.w ^ mw) | lim) & pre;
    const uint32_t si = y ? (uint32_t)__builtin_ctz(y) >> 3 : 4u;
    const uint64_t sm = ballot(si < 4);
    if (sm) {
        const int L = __builtin_ctzll(sm);
        return uni(C.w0 + 4 * L - I.sh + __builtin_amdgcn_readlane(si, L) - aa);
    }
    // a long match: continue 256 bytes per step from the window's end
    const uint32_t avail = matchlimit > aa ? matchlimit - aa : 0u;
    uint32_t mc = C.w0 + 256 - I.sh - aa;
    const uint8_t *a2 = src + aa, *m2 = src + match + skip;
    for (;;) {
        if (mc >= avail) return avail;
        const uint32_t t = mc + 4 * lane;
        uint32_t stop = 0;
        if (t < avail) {
            const uint32_t y = ld32u(a2 + t) ^ ld32u(m2 + t);
            stop = min(y ? (uint32_t)__builtin_ctz(y) >> 3 : 4u, avail - t);
        }
        const uint64_t s2 = ballot(stop < 4);
        if (s2) {
            const int L = __builtin_ctzll(s2);
            return uni(mc + 4 * L + __builtin_amdgcn_readlane(stop, L));
        }
        mc += 256;
    }
}

}  // namespace

#ifdef JFSX_LZ4_STAMP
// diagnostic build only: cycles per compressor section, summed over waves
__device__ unsigned long long g_lz4_stamps[8];
#define LZ_STAMP(t)                                                                   \
    do {                                                                              \
        __builtin_amdgcn_sched_barrier(0);                                            \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");   \
        __builtin_amdgcn_sched_barrier(0);                                            \
    } while (0)
#define LZ_SEC(k)                      \
    do {                               \
        unsigned long long t_;         \
        LZ_STAMP(t_);                  \
        st_acc[k] += t_ - st_last;     \
        st_last = t_;                  \
    } while (0)
#else
#define LZ_SEC(k) \
    do {          \
    } while (0)
#endif

// The compressor's hash table.  Positions are absolute input offsets; get()
// takes the reference position p of the probe (every entry was written at a
// position <= p) and step(lo, hi) is called, wave-uniform, before each step
// whose table accesses lie at positions in [lo, hi] (steps advance
// monotonically).
//
// TabG: the table in global memory (16 KiB per block: 4096 x u32 for inputs
// >= 64 KiB + 11 B, else 8192 x u16 as LZ4_compress_default), L2/MALL
// resident; occupancy is then set by VGPRs (8 waves per SIMD).
struct TabG {
    typedef __attribute__((address_space(1))) uint32_t gtu32;
    typedef __attribute__((address_space(1))) uint16_t gtu16;
    gtu32 *T;
    bool small;
    __device__ __forceinline__ uint32_t get(uint32_t h, uint32_t) const {
        return small ? (uint32_t)((gtu16 *)T)[h] : T[h];
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
        if (small) ((gtu16 *)T)[h] = (uint16_t)v;
        else T[h] = v;
    }
    __device__ __forceinline__ void step(uint32_t, uint32_t, uint32_t) {}
};

// TabL: the 4096-entry table of inputs >= 64 KiB + 11 B in 9 KiB of LDS, each
// entry the low 18 bits of its position (u16 + a 2-bit field), so 16 blocks
// fit a CU (the 16 GiB / 4096-block batch is one wave per block on 16 waves per
// CU: the global table's L2/MALL round trips are then the parse's latency).
// A position is recovered relative to the probe, x = p - ((p - v) mod 2^18);
// that is exact while every entry is younger than 2^18.  The only thing LZ4
// asks of an entry older than 65535 bytes is that it fails the distance test
// (LZ4_compress_generic: match + LZ4_DISTANCE_MAX < ip), so step() sweeps the
// table whenever the parse has moved 64 KiB past the last sweep point and
// rewrites every entry older than 65535 bytes as s - 65536 (still too far from
// any later probe, and young enough to stay unambiguous until the next sweep).
// Bounds (s_k sweep points, hi the highest position of the previous steps):
// a live entry is <= 65535 + 96 KiB old at any read, a rewritten one between
// 64 KiB and 160 KiB, both below 2^18.
struct TabL {
    uint16_t *lo;  // [4096]
    uint32_t *hb;  // [256]: bits 16-17 of entry h at 2 * (h & 15) of word h >> 4
    uint32_t sw, whi;  // last sweep point, highest position of the previous steps (wave-uniform)
    __device__ __forceinline__ uint32_t get(uint32_t h, uint32_t p) const {
        const uint32_t v = (uint32_t)lo[h] | (((hb[h >> 4] >> (2 * (h & 15))) & 3u) << 16);
        return p - ((p - v) & 0x3FFFFu);
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
        lo[h] = (uint16_t)v;
        const uint32_t sh = 2 * (h & 15);
#if JFSX_LZ4_MSKOR
        // one LDS op: word = (word & ~mask) | bits (ds_mskor_b32, atomic in
        // LDS like the and / or pair it replaces; a wave's LDS ops complete
        // in order, so a later read of the word sees it)
        const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)&hb[h >> 4];
        asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(a), "v"(3u << sh), "v"(((v >> 16) & 3u) << sh) : "memory");
#else
        atomicAnd(&hb[h >> 4], ~(3u << sh));
        atomicOr(&hb[h >> 4], ((v >> 16) & 3u) << sh);
#endif
    }
    __device__ void sweep(uint32_t s, uint32_t lane) {
        // lane owns words 4 lane .. 4 lane + 3 and their 64 entries
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t w = 4 * lane + k;
            const uint32_t hw = hb[w];
            uint32_t nw = 0;
            for (uint32_t e = 0; e < 16; e++) {
                const uint32_t i = 16 * w + e;
                uint32_t v = (uint32_t)lo[i] | (((hw >> (2 * e)) & 3u) << 16);
                if (((s - v) & 0x3FFFFu) > 65535u) v = (s - 65536u) & 0x3FFFFu;
                lo[i] = (uint16_t)v;
                nw |= ((v >> 16) & 3u) << (2 * e);
            }
            hb[w] = nw;
        }
    }
    __device__ __forceinline__ void step(uint32_t lo_pos, uint32_t hi_pos, uint32_t lane) {
        while (lo_pos - sw >= 65536u) {
            const uint32_t s = min(lo_pos, max(sw + 65536u, whi));
            sweep(s, lane);
            sw = s;
        }
        whi = max(whi, hi_pos);
    }
};

// One wave per block.  ZDev.len = input bytes, ZDev.cap >= LZ4_compressBound
// (checked on the host); ZOut.out_len = compressed bytes.
#ifndef JFSX_LZ4_K0
#define JFSX_LZ4_K0 4
#endif
template <class Tab>
__device__ __forceinline__ void lz4c_block(Tab &T, const uint8_t *src, uint8_t *dst, const uint32_t n,
                                           const Img &I, const bool small, const uint32_t lane, ZOut *out) {
    uint32_t op = 0, anchor = 0;
    if (n >= kMfLimit + 1) {
        const uint32_t mflimit1 = n - kMfLimit + 1, matchlimit = n - kLastLit;
        T.step(0u, 0u, lane);
        if (lane == 0) T.put(lz_hash(src, small), 0u);
        uint32_t ip = 1;
#ifdef JFSX_LZ4_STAMP
        unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_last;
        LZ_STAMP(st_last);
#endif
        IWin W;  // input window; a search starts with it holding [anchor, anchor + 253)
        W.w0 = 0xfffff000u;  // empty
        W.w = 0;
        for (;;) {
            // ---- find a match: 64 probes per step ----
            uint32_t match = 0;
            bool found = false;
            {
                const uint32_t q0 = ip;
                if (!iwin_has(W, I, anchor, q0 - anchor + 72)) iwin_load(W, I, anchor, lane);
                // speculation width: a step runs the next K probes (a prefix of
                // the serial search, so the output is unchanged); a search
                // starts with JFSX_LZ4_K0 lanes and doubles K on each step
                // without a match -- on text the first match comes within a few
                // probes, and every probe costs a random table read and a random
                // candidate read
                uint32_t K = JFSX_LZ4_K0;
                for (uint32_t k0 = 0;; k0 += K, K = K < 32 ? 2 * K : 64) {
                    const uint32_t k = k0 + lane;
                    const uint32_t p = q0 + probe_off(k);
                    const bool valid = lane < K && q0 + probe_off(k + 1) <= mflimit1;  // else this probe ends the search
                    const uint64_t amask = K >= 64 ? ~0ull : ((1ull << K) - 1ull);
                    const uint32_t pc = valid ? p : q0;
                    const uint32_t pf = q0 + probe_off(k0), pl = q0 + probe_off(k0 + K - 1);
                    uint32_t cur, b4;
                    if (iwin_has(W, I, pf, pl - pf + 8)) {
                        cur = iwin_u32_lane(W, I, pc, b4);
                    } else {
                        cur = ld32u(src + pc);
                        b4 = small ? 0u : ld8(src + pc + 4);
                    }
                    const uint32_t h = hash_of(cur, b4, small);
                    const uint64_t vmask = ballot(valid);  // a prefix of the lanes
                    T.step(pf, pl, lane);
                    // probes against the table as it stood before this step
                    const uint32_t mi0 = T.get(h, pc);
                    const bool ok0 = valid && (small || mi0 + 65535u >= p) && ld32u(src + mi0) == cur;
                    const uint64_t okm0 = ballot(ok0);
                    uint32_t mi = mi0;
                    uint64_t okm;
                    bool writer;
                    if (okm0 & 1ull) {
                        // the first probe matches: it alone ran, nothing shares its bucket
                        okm = 1ull;
                        writer = lane == 0;
                    } else {
                        // lanes of the same bucket: bit i of eq is set when lane
                        // i's hash equals this lane's
                        uint64_t eq = ~0ull;
                        if (K <= 16) {
                            // a narrow step: compare with each active lane's hash
                            eq = 0ull;
                            for (uint32_t i = 0; i < K; i++)
                                eq |= h == __builtin_amdgcn_readlane(h, (int)i) ? 1ull << i : 0ull;
                        } else {
                            // 13 ballots over the hash bits
#pragma unroll
                            for (int bit = 0; bit < 13; bit++) {
                                const bool hb = (h >> bit) & 1u;
                                const uint64_t bl = ballot(hb);
                                eq &= hb ? bl : ~bl;
                            }
                        }
                        const uint64_t below = lanes_below(lane);
                        const uint64_t prev = eq & below & vmask;
                        okm = okm0;
                        if (ballot(prev != 0ull)) {
                            // a probe after another of its bucket reads that probe's position
                            const uint32_t plv = __shfl(p, prev ? 63 - __builtin_clzll(prev) : lane, 64);
                            bool ok = ok0;
                            if (prev) {
                                mi = plv;
                                ok = valid && (small || mi + 65535u >= p) && ld32u(src + mi) == cur;
                            }
                            okm = ballot(ok);
                        }
                        const uint64_t ex = okm ? ((okm & (0ull - okm)) << 1) - 1ull : vmask;  // probes that ran
                        writer = ((ex >> lane) & 1ull) && !(eq & ex & ~below & ~(1ull << lane));
                    }
                    if (writer) T.put(h, p);
                    if (okm) {
                        const int j = __builtin_ctzll(okm);
                        ip = uni(__builtin_amdgcn_readlane(p, j));
                        match = uni(__builtin_amdgcn_readlane(mi, j));
                        found = true;
                        break;
                    }
                    if (vmask != amask) break;
                }
            }
            LZ_SEC(0);  // search
            if (!found) break;
            // ---- catch-up and match length in one round of loads ----
            // (bytes [ip', ip + 4) are equal after the catch-up, so the length
            // counted from ip + 4 plus the catch-up distance is LZ4_count from ip' + 4)
            IWin C;
            uint32_t back;
            const uint32_t limc = min(min(ip - anchor, match), 64u);
            uint32_t mc = count_and_back(C, I, src, ip, match, matchlimit, limc, back, lane);
            back = uni(back);
            if (back == 64 && limc == 64) {
                // a longer backward run: continue 64 bytes per step
                const uint32_t lim = min(ip - anchor, match);
                for (;;) {
                    const uint32_t t = back + lane;
                    const bool same = t < lim && ld8(src + ip - 1 - t) == ld8(src + match - 1 - t);
                    const uint64_t stop = ballot(!same);
                    if (stop) {
                        back += __builtin_ctzll(stop);
                        break;
                    }
                    back += 64;
                }
                back = uni(back);
            }
            ip -= back;
            match -= back;
            mc += back;
            LZ_SEC(1);  // catch-up + count
            // ---- literals ----
            uint32_t tokpos = op, tok;
            {
                const uint32_t ll = ip - anchor;
                op++;
                if (ll >= 15) {
                    tok = 15u << 4;
                    op = put_len(dst, op, ll - 15, lane);
                } else {
                    tok = ll << 4;
                }
                if (iwin_has(W, I, anchor, ll))
                    iwin_copy(dst + op, W, I, anchor, ll, lane);
                else
                    wave_copy(dst + op, src + anchor, ll, lane);
                op += ll;
            }
            LZ_SEC(2);  // literals
            // ---- match, then as long as the next position matches at once ----
            for (;;) {
                const uint32_t off = ip - match;
                if (lane == 0) {
                    st8(dst + op, off & 255u);
                    st8(dst + op + 1, off >> 8);
                }
                op += 2;
                ip += mc + kMinMatch;
                if (mc >= 15) {
                    tok += 15;
                    op = put_len(dst, op, mc - 15, lane);
                } else {
                    tok += mc;
                }
                if (lane == 0) st8(dst + tokpos, tok);
                anchor = ip;
                if (ip >= mflimit1) break;
                LZ_SEC(3);  // emit match
                // fill the table at ip - 2, then test ip itself (bytes from the
                // count window when it holds them)
                uint32_t wm2, bm2, w0, b0;
                if (iwin_has(C, I, ip - 2, 10)) {
                    wm2 = iwin_u32(C, I, ip - 2, bm2);
                    w0 = iwin_u32(C, I, ip, b0);
                } else {
                    wm2 = uni(ld32u(src + ip - 2));
                    bm2 = uni(ld8(src + ip + 2));
                    w0 = uni(ld32u(src + ip));
                    b0 = uni(ld8(src + ip + 4));
                }
                const uint32_t hm2 = uni(hash_of(wm2, bm2, small));
                const uint32_t h = uni(hash_of(w0, b0, small));
                T.step(ip - 2, ip, lane);
                if (lane == 0) T.put(hm2, ip - 2);
                const uint32_t mi = uni(T.get(h, ip));
                if (lane == 0) T.put(h, ip);
                if (small || mi + 65535u >= ip) {
                    // the 4-byte test and the match length in one round of loads
                    uint32_t nb;
                    LZ_SEC(4);  // table + hash
                    const uint32_t t = count_and_back(C, I, src, ip, mi, matchlimit, 0u, nb, lane, 0u);
                    LZ_SEC(5);  // next-position count
                    if (t >= kMinMatch) {
                        tokpos = op++;
                        tok = 0;
                        match = mi;
                        mc = t - kMinMatch;
                        continue;
                    }
                }
                break;
            }
            if (anchor >= mflimit1) break;
            ip++;
            W = C;  // the next search starts inside the count window
            LZ_SEC(6);  // next-test tail
        }
#ifdef JFSX_LZ4_STAMP
        if (lane == 0)
            for (int k = 0; k < 7; k++) atomicAdd(&g_lz4_stamps[k], st_acc[k]);
#endif
    }
    // ---- last literals ----
    {
        const uint32_t run = n - anchor;
        const uint32_t tokpos = op++;
        if (run >= 15) {
            if (lane == 0) st8(dst + tokpos, 15u << 4);
            op = put_len(dst, op, run - 15, lane);
        } else if (lane == 0) {
            st8(dst + tokpos, run << 4);
        }
        wave_copy(dst + op, src + anchor, run, lane);
        op += run;
    }
    if (lane == 0) {
        out->out_len = op;
        out->status = JFSX_OK;
    }
}

__global__ __launch_bounds__(64) void lz4_compress_k(const ZDev *__restrict__ blks, ZOut *__restrict__ outs,
                                                     uint32_t *__restrict__ tabs) {
    const uint32_t lane = threadIdx.x;
    const ZDev b = blks[blockIdx.x];
    const uint32_t n = uni((uint32_t)b.len);
    const Img I{(const uint8_t *)((uintptr_t)b.src & ~(uintptr_t)3), (uint32_t)((uintptr_t)b.src & 3), n};
    TabG T{(TabG::gtu32 *)(tabs + (size_t)blockIdx.x * 4096), n < kLimit64K};
    for (uint32_t i = 4 * lane; i < 4096; i += 256) *(__attribute__((address_space(1))) v4u *)(T.T + i) = v4u{0, 0, 0, 0};
    lz4c_block(T, b.src, b.dst, n, I, T.small, lane, outs + blockIdx.x);
}

// the same with the large-input table in LDS (TabL); inputs below 64 KiB + 11 B
// keep the u16 table in global memory
__global__ __launch_bounds__(64) void lz4_compress_lds_k(const ZDev *__restrict__ blks, ZOut *__restrict__ outs,
                                                         uint32_t *__restrict__ tabs) {
    __shared__ uint16_t tlo[4096];
    __shared__ uint32_t thb[256];
    const uint32_t lane = threadIdx.x;
    const ZDev b = blks[blockIdx.x];
    const uint32_t n = uni((uint32_t)b.len);
    const Img I{(const uint8_t *)((uintptr_t)b.src & ~(uintptr_t)3), (uint32_t)((uintptr_t)b.src & 3), n};
    if (n < kLimit64K) {
        TabG T{(TabG::gtu32 *)(tabs + (size_t)blockIdx.x * 4096), true};
        for (uint32_t i = 4 * lane; i < 4096; i += 256)
            *(__attribute__((address_space(1))) v4u *)(T.T + i) = v4u{0, 0, 0, 0};
        lz4c_block(T, b.src, b.dst, n, I, true, lane, outs + blockIdx.x);
        return;
    }
    for (uint32_t i = lane; i < 2048; i += 64) reinterpret_cast<uint32_t *>(tlo)[i] = 0u;
    for (uint32_t i = lane; i < 256; i += 64) thb[i] = 0u;
    TabL T{tlo, thb, 0u, 0u};
    lz4c_block(T, b.src, b.dst, n, I, false, lane, outs + blockIdx.x);
}


namespace {

// 256-byte window of the compressed input in the wave's VGPRs
struct DWin {
    uint32_t n;
    uint32_t w0;   // window start (multiple of 4, relative to src's dword-aligned base)
    uint32_t w;    // this lane's dword
    uintptr_t al;  // src rounded down to 4
    uint32_t sh;   // src - al
};

__device__ __forceinline__ void win_load(DWin &W, uint32_t pos, uint32_t lane) {
    // dword d of the aligned image covers src bytes [4d - sh, 4d - sh + 4)
    W.w0 = (pos + W.sh) & ~3u;
    const uint32_t o = W.w0 + 4 * lane;  // aligned-image offset
    const bool in = o < W.n + W.sh;        // the dword holds at least one input byte
    W.w = in ? ld32a((const uint8_t *)(W.al + o)) : 0u;
}

// input bytes [pos, pos + 4) as a little-endian word (uniform; reloads the
// window at pos when it does not hold them).  Two v_readlane and one 64-bit
// scalar shift: the parse stays in SGPRs.
__device__ __forceinline__ uint32_t win_u32(DWin &W, uint32_t pos, uint32_t lane) {
    const uint32_t x = pos + W.sh;
    if (x < W.w0 || x + 4u > W.w0 + 256u) win_load(W, pos, lane);
    const uint32_t r = x - W.w0;
    const uint64_t d = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(W.w, r >> 2) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(W.w, ((r >> 2) + 1) & 63) << 32);
    return (uint32_t)(d >> (8 * (r & 3)));
}

__device__ __forceinline__ uint32_t win_byte(DWin &W, uint32_t pos, uint32_t lane) {
    const uint32_t x = pos + W.sh;
    if (x - W.w0 >= 256u) win_load(W, pos, lane);
    const uint32_t r = x - W.w0;
    return (__builtin_amdgcn_readlane(W.w, r >> 2) >> (8 * (r & 3))) & 255u;
}

typedef __attribute__((address_space(1))) v4u gv4u;

}  // namespace

// The decoder writes its output into an LDS ring and from there to global
// memory in coalesced 16-byte stores (one 1 KiB wave store per step).  Output
// position p sits at ring[(p + s) & (R - 1)], s = dst & 15, so a ring slot and
// the global address of its byte agree modulo 16.
#ifndef JFSX_LZ4_RING
#define JFSX_LZ4_RING 8192
#endif
constexpr uint32_t kDRing = JFSX_LZ4_RING;  // decoder ring: the most recent output bytes
#ifndef JFSX_LZ4_FLUSH
#define JFSX_LZ4_FLUSH 4096
#endif
constexpr uint32_t kDFlush = JFSX_LZ4_FLUSH;  // flush once this many unflushed bytes are in the ring

namespace {

// global image bytes [a, b) (image coordinate = position + s; dal = dst - s,
// 16-byte aligned) from the ring: aligned 16-byte units as 1 KiB wave stores,
// the partial units at either end byte-wise
template <uint32_t R>
__device__ void ring_flush(uint8_t *dal, const uint8_t *ring, uint32_t a, uint32_t b, uint32_t lane) {
    constexpr uint32_t RM = R - 1;
    if (a >= b) return;
    const uint32_t u0 = (a + 15) & ~15u, u1 = b & ~15u;
    if (u0 >= u1) {
        if (lane < b - a) st8(dal + a + lane, ring[(a + lane) & RM]);
        return;
    }
    if (lane < u0 - a) st8(dal + a + lane, ring[(a + lane) & RM]);
    for (uint32_t u = u0; u < u1; u += 1024) {
        const uint32_t x = u + 16 * lane;
        if (x < u1) *(gv4u *)(dal + x) = *(const v4u *)(ring + (x & RM));
    }
    if (lane < b - u1) st8(dal + u1 + lane, ring[(u1 + lane) & RM]);
}

// ring bytes of positions [p, p + cnt) from global bytes g[0, cnt)
template <uint32_t R>
__device__ void ring_fill(uint8_t *ring, uint32_t s, uint32_t p, uint32_t cnt, const uint8_t *g, uint32_t lane) {
    constexpr uint32_t RM = R - 1;
#pragma unroll 1
    for (uint32_t j = lane; j < cnt; j += 64) ring[(p + s + j) & RM] = (uint8_t)ld8(g + j);
}

}  // namespace

// Lane L decodes the sequence that would start at input position base + L
// (the window holds [base, base + 96)) for the fast path.  A sequence is
// "short" when none of LZ4_decompress_safe's input-side checks can reject it:
// literal run < 15, match nibble < 15, no overlap (off >= match length), and
// it ends at least 8 bytes before the input end.
//   c.f  bit 0: short and its successor token lies within the 64 lanes;
//        bit 1: off > near (the source is farther back than the ring keeps);
//        bit 2: short, but the successor lies past lane 63 (refresh first);
//        bits 8-13: the successor's lane
//   c.ll literal length, c.tot literal + match length, c.off offset
struct SeqCand {
    uint32_t f, ll, tot, off;
};
template <uint32_t NEAR>
__device__ __forceinline__ SeqCand seq_candidates(const DWin &W, uint32_t base, uint32_t n, uint32_t lane) {
    const uint32_t p = base + lane, r = p + W.sh - W.w0;
    const uint32_t t = (__shfl(W.w, (int)(r >> 2), 64) >> (8 * (r & 3))) & 255u;
    const uint32_t ll = t >> 4, mn = t & 15u, q = r + 1 + ll;
    const uint32_t d0 = __shfl(W.w, (int)(q >> 2), 64), d1 = __shfl(W.w, (int)((q >> 2) + 1), 64);
    const uint32_t off = __builtin_amdgcn_alignbyte(d1, d0, q & 3) & 0xffffu;
    const uint32_t ml = mn + kMinMatch, next = lane + 3 + ll;
    const bool shrt = ll < 15 && mn < 15 && off >= ml && p + 9 + ll <= n;
    SeqCand c;
    c.f = (uint32_t)(shrt && next < 64) | ((uint32_t)(off > NEAR) << 1) | ((uint32_t)(shrt && next >= 64) << 2) |
          ((next & 63) << 8);
    c.ll = ll;
    c.tot = ll + ml;
    c.off = off;
    return c;
}

// One wave per block.  ZDev.len = compressed bytes, ZDev.cap = dst capacity
// (< 2^32, checked on the host); ZOut.out_len = decoded bytes; status
// JFSX_EFORMAT for a malformed stream.  The control flow is wave-uniform
// 32-bit scalar code: a sequence's token, offset and first length byte come
// from one 4-byte read of the register window.  Output is assembled in the
// LDS ring and leaves it in 4 KiB coalesced flushes, so a match whose source
// lies in the ring reads LDS, and only a source farther back than the ring
// (already flushed) is read from global memory.  Long literal runs and long
// or far overlapping matches copy global to global after a flush.
template <uint32_t R>
__global__ __launch_bounds__(64) void lz4_decompress_k(const ZDev *__restrict__ blks, ZOut *__restrict__ outs) {
    // ring room: a flush leaves < kDFlush + 16 unflushed bytes; then a literal
    // run of <= 256 bytes and a 64-byte copy; a far source (off > R - 64) is
    // flushed when kDFlush + 142 <= R
    static_assert(R >= kDFlush + 16 + 256 + 64 && (R & (R - 1)) == 0, "ring size");
    __shared__ __attribute__((aligned(16))) uint8_t ring[R];
    constexpr uint32_t RM = R - 1;
    // a ring source must lie within the last R - 64 bytes: the fast path's
    // 64-lane copies may overwrite the 64 slots after the write position
    constexpr uint32_t NR = R - 64;
    const uint32_t lane = threadIdx.x;
    const ZDev b = blks[blockIdx.x];
    const uint8_t *src = b.src;
    uint8_t *dst = b.dst;
    const uint32_t n = uni((uint32_t)b.len);
    const uint32_t cap = uni((uint32_t)b.cap);
    const uint32_t s = (uint32_t)((uintptr_t)dst & 15);
    uint8_t *dal = dst - s;
    uint32_t op = 0, fl = 0, fenced = 0;  // [0, fl) flushed to dst; [0, fenced) visible to this wave's loads
    bool bad = false;
    // everything up to op to dst (the bulk paths write dst directly after it)
    auto flush_all = [&]() {
        ring_flush<R>(dal, ring, fl + s, op + s, lane);
        fl = op;
    };
    // make dst bytes below need visible to this wave's loads
    auto fence = [&](uint32_t need) {
        if (need > fenced) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            fenced = fl;
        }
    };
    if (cap == 0) {
        bad = !(n == 1 && ld8(src) == 0);
    } else if (n == 0) {
        bad = true;
    } else {
        DWin W;
        W.n = n;
        W.al = (uintptr_t)src & ~(uintptr_t)3;
        W.sh = (uint32_t)((uintptr_t)src & 3);
        win_load(W, 0, lane);
        uint32_t ip = 0, base = 0, litq = 0;
        SeqCand cand{0, 0, 0, 0};
        bool stale = true;
        const uint32_t lane_s = lane + s;
        // literals [ip, ip + len) to output position op.  A run the window
        // holds goes to the ring; a longer one is copied global to global
        // (and its last R bytes to the ring unless it ends the block).
        auto literals = [&](uint32_t len, bool last) {
            const uint32_t xl = ip + W.sh;
            if (len <= 253u && (xl < W.w0 || xl + len > W.w0 + 256u)) win_load(W, ip, lane);
            if (xl >= W.w0 && xl + len <= W.w0 + 256u) {
                const uint32_t rl = xl - W.w0;
#pragma unroll
                for (uint32_t k = 0; k < 4; k++) {
                    if (64 * k >= len) break;
                    const uint32_t j = lane + 64 * k, q = rl + j;
                    const uint32_t d = __shfl(W.w, (int)((q >> 2) & 63), 64);
                    if (j < len) ring[(op + s + j) & RM] = (uint8_t)(d >> (8 * (q & 3)));
                }
            } else {
                flush_all();
                wave_copy(dst + op, src + ip, len, lane);
                if (!last) {
                    const uint32_t k = len > R ? len - R : 0u;
                    ring_fill<R>(ring, s, op + k, len - k, src + ip + k, lane);
                }
                fl = op + len;
            }
        };
        for (;;) {
            if (op - fl >= kDFlush) {
                // flush whole 16-byte units only, so the next flush starts aligned
                const uint32_t e = (op + s) & ~15u;
                ring_flush<R>(dal, ring, fl + s, e, lane);
                fl = e - s;
            }
            // ---- fast path: sequences decoded in advance by the lanes ----
            if (stale || ip - base >= 64u) {
                base = ip;
                const uint32_t x = base + W.sh;
                if (x < W.w0 || x + 96u > W.w0 + 256u) win_load(W, base, lane);
                cand = seq_candidates<NR>(W, base, n, lane);
                litq = base + 1 + W.sh - W.w0 + lane;  // window byte of literal lane for kk = 0
                stale = false;
            }
            {
                // Every check of a sequence comes before its first write, so an
                // exit leaves (ip, op) at a sequence start for the general path.
                // Copies run on all 64 lanes: the bytes past a literal run or
                // match land on output positions written again before they are
                // flushed, and on ring slots no near match (off <= R - 64) reads.
                uint32_t kk = ip - base;
                const uint32_t fstop = fl + kDFlush;
                const uint32_t opstop = cap >= 44u ? min(fstop, cap - 43u) : 0u;
                uint32_t info = __builtin_amdgcn_readlane(cand.f, kk);
                auto run = [&](auto early) {
                    while ((info & 1u) && op < opstop) {
                        const uint32_t ll = __builtin_amdgcn_readlane(cand.ll, kk);
                        const uint32_t off = __builtin_amdgcn_readlane(cand.off, kk);
                        if (decltype(early)::value && op + ll < off) break;  // the general path rejects it
                        // the literal run (64 window bytes) at op, then the match at op + ll
                        const uint32_t q = kk + litq;
                        const uint32_t d = __shfl(W.w, (int)((q >> 2) & 63), 64);
                        ring[(op + lane_s) & RM] = (uint8_t)(d >> (8 * (q & 3)));
                        const uint32_t dp = op + ll + lane_s;
                        if (!(info & 2u)) {
#ifdef JFSX_ABLATE_NEAR
                            ring[dp & RM] = (uint8_t)off;
#else
                            ring[dp & RM] = ring[(dp - off) & RM];
#endif
                        } else {
#ifdef JFSX_ABLATE_FAR
                            ring[dp & RM] = (uint8_t)off;
#else
                            // farther back than the ring: flushed, read dst
                            const uint32_t srcp = op + ll - off;
                            fence(srcp + 64u);
                            ring[dp & RM] = (uint8_t)ld8(dst + srcp + lane);
#endif
                        }
                        op += __builtin_amdgcn_readlane(cand.tot, kk);
                        kk = (info >> 8) & 63u;
                        info = __builtin_amdgcn_readlane(cand.f, kk);
                    }
                };
                if (op >= 65536u)
                    run(std::false_type{});
                else
                    run(std::true_type{});
                ip = base + kk;
                if (op >= fstop) continue;  // flush, then on
                if (!(info & 1u) && (info & 4u)) {
                    stale = true;  // the next token is past the candidates
                    continue;
                }
            }
            // ---- general path: one sequence with every LZ4_decompress_safe check ----
            stale = true;
            if (ip >= n) { bad = true; break; }
            const uint32_t D = win_u32(W, ip, lane);  // token and the next 3 bytes
            const uint32_t token = D & 255u;
            ip++;
            uint32_t len = token >> 4;
            if (len == 15) {
                uint32_t sb;
                do {
                    if (ip + 15 >= n) { bad = true; break; }
                    sb = win_byte(W, ip++, lane);
                    len += sb;
                } while (sb == 255);
                if (bad) break;
            }
            if (len > cap - op || len > n - ip) { bad = true; break; }
            if ((uint64_t)op + len + kMfLimit > cap || (uint64_t)ip + len + (2 + 1 + kLastLit) > n) {
                // the last sequence: it must end the input exactly
                if (ip + len != n) { bad = true; break; }
                literals(len, true);
                op += len;
                break;
            }
            uint32_t off, ml = token & 15u, e1;  // e1: the byte after the offset
            if (len == 0) {
                off = (D >> 8) & 0xffffu;
                e1 = D >> 24;
            } else {
                literals(len, false);
                ip += len;
                op += len;
                const uint32_t w = win_u32(W, ip, lane);
                off = w & 0xffffu;
                e1 = (w >> 16) & 255u;
            }
            ip += 2;
            if (off > op) { bad = true; break; }
            if (ml == 15) {
                if (ip + kLastLit > n) { bad = true; break; }
                uint32_t sb = e1;
                ip++;
                ml += sb;
                while (sb == 255) {
                    if (ip + kLastLit > n) { bad = true; break; }
                    sb = win_byte(W, ip++, lane);
                    ml += sb;
                }
                if (bad) break;
            }
            ml += kMinMatch;
            if (ml > cap - op || (uint64_t)op + ml + kLastLit > cap) { bad = true; break; }
            if (ml <= 64 && ml <= off && off <= NR) {
                // one step, the source in the ring (all of this step's reads
                // happen before its writes)
#ifdef JFSX_ABLATE_NEAR
                if (lane < ml) ring[(op + s + lane) & RM] = (uint8_t)off;
#else
                if (lane < ml) ring[(op + s + lane) & RM] = ring[(op - off + s + lane) & RM];
#endif
                op += ml;
                continue;
            }
            if (op + ml > fl + R) flush_all();  // ring room for the match
            if (ml <= R && off == 0) {
                // an offset of 0 copies the bytes being written: LZ4 1.9 zero-fills them
                for (uint32_t j = lane; j < ml; j += 64) ring[(op + s + j) & RM] = 0;
            } else if (ml <= R && ml <= off && off <= NR) {
                // disjoint, in the ring: step k's source lies above every slot
                // steps < k overwrote
                for (uint32_t j0 = 0; j0 < ml; j0 += 64) {
                    const uint32_t j = j0 + lane;
                    if (j < ml) ring[(op + s + j) & RM] = ring[(op - off + s + j) & RM];
                }
            } else if (ml <= 64 && ml <= off) {
                // disjoint and farther back than the ring: flushed, read dst
#ifdef JFSX_ABLATE_FAR
                if (lane < ml) ring[(op + s + lane) & RM] = (uint8_t)off;
#else
                if (op - off + ml > fl) flush_all();
                fence(op - off + ml);
                if (lane < ml) ring[(op + s + lane) & RM] = (uint8_t)ld8(dst + op - off + lane);
#endif
            } else if (off != 0 && off <= 64 && ml <= R && ml <= (1u << 24)) {
                // short period: the off source bytes, read once, repeat.  j % off
                // by a float reciprocal (j < 2^24: the quotient is off by at most one)
                const float rcp = 1.0f / (float)off;
                auto mod = [&](uint32_t j) {
                    uint32_t q = (uint32_t)((float)j * rcp);
                    int32_t rr = (int32_t)(j - q * off);
                    rr += rr < 0 ? (int32_t)off : 0;
                    rr -= rr >= (int32_t)off ? (int32_t)off : 0;
                    return (uint32_t)rr;
                };
                const uint32_t pat = ring[(op - off + s + mod(lane)) & RM];
                for (uint32_t j0 = 0; j0 < ml; j0 += 64) {
                    // every lane joins the ds_bpermute (a disabled source lane reads 0)
                    const uint32_t j = j0 + lane;
                    const uint32_t v = __shfl(pat, (int)mod(j), 64);
                    if (j < ml) ring[(op + s + j) & RM] = (uint8_t)v;
                }
            } else if (off != 0 && off <= NR && off + ml <= R) {
                // overlapping, period > 64: the first off bytes repeat
                for (uint32_t j = lane; j < ml; j += 64)
                    ring[(op + s + j) & RM] = ring[(op - off + s + (j < off ? j : j % off)) & RM];
            } else {
                // long: global to global after a flush, then the last R bytes to the ring
                flush_all();
                fence(op);
                uint8_t *o = dst + op;
                const uint8_t *m = o - off;
                if (off == 0)
                    for (uint32_t j = lane; j < ml; j += 64) st8(o + j, 0u);
                else if (ml <= off)
                    wave_copy(o, m, ml, lane);  // disjoint
                else  // overlapping: the first off bytes repeat
                    for (uint32_t j = lane; j < ml; j += 64) st8(o + j, ld8(m + j % off));
#pragma unroll 1
                for (uint32_t j = (ml > R ? ml - R : 0) + lane; j < ml; j += 64)
                    ring[(op + s + j) & RM] = off == 0 ? 0 : (uint8_t)ld8(m + (j < off ? j : j % off));
                fl = op + ml;
            }
            op += ml;
        }
    }
    if (!bad) ring_flush<R>(dal, ring, fl + s, op + s, lane);
    if (lane == 0) {
        outs[blockIdx.x].out_len = bad ? 0 : (uint64_t)op;
        outs[blockIdx.x].status = bad ? JFSX_EFORMAT : JFSX_OK;
    }
}

#ifdef JFSX_LZ4_STAMP
}  // namespace jfsx
extern "C" int jfsx_debug_lz4_stamps(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(jfsx::g_lz4_stamps), sizeof(unsigned long long) * 8) != hipSuccess)
        return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(jfsx::g_lz4_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
namespace jfsx {
#endif

// LDS table while every block of the batch is resident at once (up to 16
// blocks per CU: the parse is then latency-bound), global-memory table for
// bigger batches (32 waves per CU).  JFSX_LZ4_TABLE=lds|global overrides.
void launch_lz4_compress(hipStream_t s, int n, int ncu, const ZDev *blks, ZOut *outs, uint32_t *tabs) {
    if (n <= 0) return;
    const char *e = getenv("JFSX_LZ4_TABLE");  // read per launch (tests switch it)
    const int mode = !e ? 0 : !strcmp(e, "lds") ? 1 : !strcmp(e, "global") ? 2 : 0;
    const bool lds = mode == 1 || (mode == 0 && n <= 16 * ncu);
    if (lds) hipLaunchKernelGGL(lz4_compress_lds_k, dim3(n), dim3(64), 0, s, blks, outs, tabs);
    else hipLaunchKernelGGL(lz4_compress_k, dim3(n), dim3(64), 0, s, blks, outs, tabs);
}

void launch_lz4_decompress(hipStream_t s, int n, const ZDev *blks, ZOut *outs) {
    if (n > 0) hipLaunchKernelGGL(lz4_decompress_k<kDRing>, dim3(n), dim3(64), 0, s, blks, outs);
}

}  // namespace jfsx

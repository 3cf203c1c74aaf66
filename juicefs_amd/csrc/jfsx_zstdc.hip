// jfsx_zstdc.hip -- Zstandard level-1 compression on gfx950 (the upload side
// of --compress zstd volumes).
//
// Replaces ZStandard.Compress = zstd.CompressLevel(dst, src, 1)
// (pkg/compress/compress.go:82-91; DataDog/zstd v1.5.0 -> ZSTD_compress) as
// called by cachedStore.upload (pkg/chunk/cached_store.go:371-392, :387).
// The frame bytes are those of the zstd library's level-1 one-shot path
// (jfsx_zstdc.h restates it; tests compare with the system libzstd 1.4.8).
//
// Decomposition: the greedy parse of a frame is sequential from its first
// byte to its last (one hash table and one set of repcodes and entropy
// tables carried over all 128 KiB blocks), so one wave owns one object.
// Persistent waves take objects w, w + W, ... (W waves; a ticket queue is an
// A/B switch); each has a global scratch (hash table, sequences, literals,
// codes) and its entropy tables in LDS.
//
// The parser (ZSTD_compressBlock_fast_generic) runs on the 64 lanes:
//   * a search step evaluates 64 consecutive iterations of the serial loop at
//     once -- lane j the positions p_j, p_j + 1 (hashes, table reads, 4-byte
//     compares) and the repcode at p_j + 2.  The positions of a miss run are
//     known in advance (step = (p - anchor) / 128 + 2).
//   * iterations see the table writes of the iterations before them: when
//     the first iteration does not already succeed on its own, 2 x hashLog
//     ballots give every lane the lanes whose writes share its buckets; reads
//     take the latest earlier writer, and only the last writer of a bucket
//     (up to the first success) stores.
//   * backward catch-up and the match-length count run 64 / 256 bytes per
//     step with a ballot for the first difference.
//   * the input bytes a step, a match's catch-up and length, its literal copy
//     and its hash inserts need come from 256-byte register windows where
//     they fall inside one (parse_fast_wave_w, JFSX_ZC_WIN bits), so most
//     sequences cost two or three memory round trips, not eight.
// The entropy stage of a block (literal Huffman coding, sequence FSE coding)
// builds its tables on one lane (the library's serial code, jfsx_zstdc.h) and
// spreads the per-symbol work over the lanes.
//
// The parser is bound by memory latency (a chain of dependent random reads
// per sequence), so occupancy is what buys throughput: 16 waves per CU (LDS
// 9.3 KiB and <= 128 VGPRs per wave) -- a 4096-object batch in one pass.
#include "jfsx_dev.h"
#include "jfsx_zstdc.h"

// 0: parse_fast_wave (every read from memory); else parse_fast_wave_w with
// the window features named below (287: windows for everything + candidate
// extensions; A/B in profiles/r4/ab_zstdc_win.txt)
#ifndef JFSX_ZC_WIN
#define JFSX_ZC_WIN 287
#endif
// lanes of the first search step after a match (doubling on each miss)
#ifndef JFSX_ZC_K0
#define JFSX_ZC_K0 2
#endif
// the entropy stage's byte loops and the block copies with several loads in
// flight per lane (bits: 1 block copies, 2 histograms, 4 Huffman emission,
// 8 FSE state chains, 16 sequence emission and codes; 0: one load per loop
// iteration, the round-3 code; A/B in profiles/r4/ab_zstdc_win.txt)
#ifndef JFSX_ZC_MLP
#define JFSX_ZC_MLP 31
#endif

namespace jfsx {

namespace {
constexpr size_t kZcHtab = (size_t)4 << jzc::kHashLogMax;             // 128 KiB
constexpr size_t kZcSeq = (size_t)jzc::kMaxSeq * sizeof(jzc::SeqDef);  // 256 KiB
constexpr size_t kZcLit = (size_t)jzc::kBlockMax + 256;                // literals
constexpr size_t kZcCodes = (size_t)3 * jzc::kMaxSeq;                  // ll / ml / of codes
constexpr size_t kZcBody = (size_t)jzc::kBodyCap;                      // one block body
constexpr size_t kZcRec = (size_t)6 * jzc::kMaxSeq;                    // FSE state-chain outputs (3 x u16)
static_assert(kZcHtab + kZcSeq + kZcLit + kZcCodes + kZcBody + kZcRec <= kZstdcScratch, "zstd compress scratch");

typedef __attribute__((address_space(1))) const uint32_t gcu32z;
typedef __attribute__((address_space(1))) const uint8_t gcu8c;
typedef __attribute__((address_space(1))) uint8_t gu8c;
typedef __attribute__((address_space(1))) uint32_t gu32c;

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int32_t unis(int32_t v) { return (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)v); }
__device__ __forceinline__ uint64_t ballot(bool b) { return __ballot(b); }
__device__ __forceinline__ uint32_t ld8(const uint8_t *p) { return *(gcu8c *)p; }
__device__ __forceinline__ uint32_t ld32a(const uint8_t *p) { return *(gcu32z *)p; }
// 4 bytes at any address: two aligned dword loads, each holding at least one
// of the requested bytes (neither touches a page the bytes are not on)
__device__ __forceinline__ uint32_t ld32u(const uint8_t *a) {
    const uintptr_t x = (uintptr_t)a;
    const uint8_t *b = (const uint8_t *)(x & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(x & 3);
    const uint32_t w0 = ld32a(b), w1 = ld32a(sh ? b + 4 : b);
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
}
__device__ __forceinline__ uint32_t readlane(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int32_t readlanes(int32_t v, int l) { return (int32_t)__builtin_amdgcn_readlane((uint32_t)v, l); }

// jzc::hash_ptr of the 8 bytes w (little-endian) at a position
__device__ __forceinline__ uint32_t hash_w(uint64_t w, uint32_t hlog, uint32_t mls) {
    if (mls == 5) return (uint32_t)(((w << 24) * 889523592379ull) >> (64 - hlog));
    if (mls == 6) return (uint32_t)(((w << 16) * 227718039650203ull) >> (64 - hlog));
    if (mls == 7) return (uint32_t)(((w << 8) * 58295818150454627ull) >> (64 - hlog));
    return ((uint32_t)w * 2654435761u) >> (32 - hlog);
}

// bytes [p, p + 8) and [p + 1, p + 9) from three aligned dwords (p + 8 must
// lie inside the input)
__device__ __forceinline__ void load9(const uint8_t *src, int32_t p, uint64_t &w0, uint64_t &w1) {
    const uintptr_t x = (uintptr_t)(src + p);
    const uint8_t *b = (const uint8_t *)(x & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(x & 3);
    const uint32_t d0 = ld32a(b), d1 = ld32a(b + 4), d2 = ld32a(b + 8);
    w0 = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
    if (sh == 3) {
        w1 = (uint64_t)d1 | ((uint64_t)d2 << 32);
    } else {
        w1 = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh + 1) |
             ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh + 1) << 32);
    }
}

__device__ __forceinline__ uint64_t ld64u(const uint8_t *p) {
    return (uint64_t)ld32u(p) | ((uint64_t)ld32u(p + 4) << 32);
}

// ZSTD_count(a, b, lim) on the wave: 256 bytes per step (a > b)
__device__ uint32_t count_wave(const uint8_t *a, const uint8_t *b, const uint8_t *lim, uint32_t lane) {
    const uint32_t avail = (uint32_t)(lim - a);
    for (uint32_t c = 0;; c += 256) {
        if (c >= avail) return avail;
        const uint32_t t = c + 4 * lane;
        uint32_t stop = 0xffffffffu;
        if (t + 4 <= avail) {
            const uint32_t x = ld32u(a + t) ^ ld32u(b + t);
            if (x) stop = t + ((uint32_t)__builtin_ctz(x) >> 3);
        } else if (t < avail) {
            stop = avail;
            for (uint32_t k = t; k < avail; k++)
                if (ld8(a + k) != ld8(b + k)) {
                    stop = k;
                    break;
                }
        }
        const uint64_t sm = ballot(stop != 0xffffffffu);
        if (sm) return uni(readlane(stop, __builtin_ctzll(sm)));
    }
}

// how many of the bytes before a and b (at most lim) are equal, 64 per step
__device__ uint32_t back_wave(const uint8_t *a, const uint8_t *b, uint32_t lim, uint32_t lane) {
    for (uint32_t c = 0;; c += 64) {
        if (c >= lim) return lim;
        const uint32_t t = c + lane;
        const bool diff = t < lim && ld8(a - 1 - t) != ld8(b - 1 - t);
        const uint64_t sm = ballot(diff || t >= lim);
        if (sm) return uni(c + (uint32_t)__builtin_ctzll(sm));
    }
}

__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
__device__ __forceinline__ uint64_t lanes_above(uint32_t lane) { return lane == 63 ? 0ull : (~0ull << (lane + 1)); }

struct WSeq {  // the wave's view of the block's sequence store
    jzc::SeqDef *seq;
    uint8_t *lit;
    uint32_t nseq, nlit, long_id, long_pos;
};

// ZSTD_storeSeq: literals copied by the lanes, the record by lane 0
__device__ __forceinline__ void store_seq_wave(WSeq &ss, const uint8_t *lits, uint32_t litLen, uint32_t offCode,
                                               uint32_t mlBase, uint32_t lane) {
    for (uint32_t o = lane; o < litLen; o += 64) *(gu8c *)(ss.lit + ss.nlit + o) = (uint8_t)ld8(lits + o);
    if (litLen > 0xFFFF) ss.long_id = 1, ss.long_pos = ss.nseq;
    if (mlBase > 0xFFFF) ss.long_id = 2, ss.long_pos = ss.nseq;
    if (lane == 0) {
        jzc::SeqDef d;
        d.offset = offCode + 1;
        d.ll = (uint16_t)litLen;
        d.ml = (uint16_t)mlBase;
        ss.seq[ss.nseq] = d;
    }
    ss.nseq++;
    ss.nlit += litLen;
}

// ---------------------------------------------------------------------------
// Register windows (JFSX_ZC_WIN): 256 input bytes in the wave's VGPRs, lane L
// holding the image dword at w0 + 4L (zero past the object's end).  A read
// inside a window is a ds_bpermute (per-lane position) or v_readlane (uniform
// position), not a memory round trip; the search steps, the literal copies and
// the hash inserts after a match read from them, and the catch-up bytes and
// the match length come from one round of loads (count_back).
// ---------------------------------------------------------------------------
struct ZImg {  // the object as an aligned image: byte pos at offset pos + sh of al
    const uint8_t *al;
    uint32_t sh, n;
};
struct ZWin {
    uint32_t w0, w;
};
__device__ __forceinline__ void zw_load(ZWin &W, const ZImg &I, uint32_t pos, uint32_t lane) {
    W.w0 = (pos + I.sh) & ~3u;
    const uint32_t o = W.w0 + 4 * lane;
    W.w = o < I.n + I.sh ? ld32a(I.al + o) : 0u;
}
// [pos, pos + len) inside the window (pos may be any int)
__device__ __forceinline__ bool zw_has(const ZWin &W, const ZImg &I, int32_t pos, uint32_t len) {
    const int64_t x = (int64_t)pos + I.sh;
    return x >= (int64_t)W.w0 && x + len <= (int64_t)W.w0 + 256;
}
// 4 bytes at a per-lane position inside the window (zw_has(pos, 8))
__device__ __forceinline__ uint32_t zw_u32_lane(const ZWin &W, const ZImg &I, int32_t pos) {
    const uint32_t r = (uint32_t)pos + I.sh - W.w0, i = r >> 2, sh = r & 3;
    const uint32_t d0 = __shfl(W.w, (int)(i & 63), 64), d1 = __shfl(W.w, (int)((i + 1) & 63), 64);
    return __builtin_amdgcn_alignbyte(d1, d0, sh);
}
// 8 bytes at a uniform position inside the window (zw_has(pos, 12))
__device__ __forceinline__ uint64_t zw_u64(const ZWin &W, const ZImg &I, int32_t pos) {
    const uint32_t r = (uint32_t)pos + I.sh - W.w0, i = r >> 2, sh = r & 3;
    const uint32_t d0 = readlane(W.w, (int)i), d1 = readlane(W.w, (int)i + 1), d2 = readlane(W.w, (int)i + 2);
    return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
}
// load9 from the window: bytes [p, p + 8) and [p + 1, p + 9) (zw_has(p, 12))
__device__ __forceinline__ void zw_load9(const ZWin &W, const ZImg &I, int32_t p, uint64_t &w0, uint64_t &w1) {
    const uint32_t r = (uint32_t)p + I.sh - W.w0, i = r >> 2, sh = r & 3;
    const uint32_t d0 = __shfl(W.w, (int)(i & 63), 64), d1 = __shfl(W.w, (int)((i + 1) & 63), 64),
                   d2 = __shfl(W.w, (int)((i + 2) & 63), 64);
    w0 = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
    if (sh == 3) {
        w1 = (uint64_t)d1 | ((uint64_t)d2 << 32);
    } else {
        w1 = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh + 1) |
             ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh + 1) << 32);
    }
}
// Candidate extensions (bit 256): with its 4-byte check a lane loads the 24
// image bytes from the dword at or below m - 4 (m the candidate), so the
// winner's catch-up (up to 4 bytes) and first 12 match bytes are in registers
// when the step's ballot names it and a short match needs no count_back.
typedef unsigned int zv4u __attribute__((ext_vector_type(4), aligned(4)));
typedef unsigned int zv2u __attribute__((ext_vector_type(2), aligned(4)));
struct ZExt {
    uint32_t e[6];
    bool in;  // the 24 bytes lie inside the object image (else e is not loaded)
};
__device__ __forceinline__ void zx_load(ZExt &X, const ZImg &I, int32_t m) {
    const int32_t o = ((m + (int32_t)I.sh) & ~3) - 4;
    X.in = o >= 0 && o + 24 <= (int32_t)(I.n + I.sh);
    // lanes whose 24 bytes are not inside the image load nothing (an object
    // shorter than 24 bytes has no in-bounds 24-byte window at all)
    zv4u v = {0u, 0u, 0u, 0u};
    zv2u w = {0u, 0u};
    if (X.in) {
        const uint8_t *a = I.al + o;
        v = *(__attribute__((address_space(1))) const zv4u *)a;
        w = *(__attribute__((address_space(1))) const zv2u *)(a + 16);
    }
    X.e[0] = v.x, X.e[1] = v.y, X.e[2] = v.z, X.e[3] = v.w, X.e[4] = w.x, X.e[5] = w.y;
}

// ZSTD_storeSeq with the literals [pos, pos + litLen) taken from the window
__device__ __forceinline__ void store_seq_win(WSeq &ss, const ZWin &W, const ZImg &I, int32_t pos, uint32_t litLen,
                                              uint32_t offCode, uint32_t mlBase, uint32_t lane) {
    const uint32_t r = (uint32_t)pos + I.sh - W.w0;
    for (uint32_t k = 0; k < 4 && 64 * k < litLen; k++) {  // literal runs are short: one pass, mostly
        const uint32_t j = lane + 64 * k, q = r + j;
        const uint32_t dw = __shfl(W.w, (int)((q >> 2) & 63), 64);
        if (j < litLen) *(gu8c *)(ss.lit + ss.nlit + j) = (uint8_t)(dw >> (8 * (q & 3)));
    }
    if (litLen > 0xFFFF) ss.long_id = 1, ss.long_pos = ss.nseq;
    if (mlBase > 0xFFFF) ss.long_id = 2, ss.long_pos = ss.nseq;
    if (lane == 0) {
        jzc::SeqDef d;
        d.offset = offCode + 1;
        d.ll = (uint16_t)litLen;
        d.ml = (uint16_t)mlBase;
        ss.seq[ss.nseq] = d;
    }
    ss.nseq++;
    ss.nlit += litLen;
}
// ZSTD_count(ipX + 4, mX + 4, limit) and, in the same round of loads, the
// catch-up: how many of the limc (<= 64) bytes before ipX and mX are equal
// (back; 64 when all 64 were).  C receives the window at ipX + 4.
__device__ uint32_t count_back(ZWin &C, const ZImg &I, const uint8_t *src, int32_t ipX, int32_t mX, int32_t limit,
                               uint32_t limc, uint32_t &back, uint32_t lane) {
    const int32_t aa = ipX + 4, off = ipX - mX;
    zw_load(C, I, (uint32_t)aa, lane);
    const int32_t lp = (int32_t)(C.w0 + 4 * lane) - (int32_t)I.sh;  // input position of this lane's window dword
    const int32_t mp = lp - off;                                      // >= 1: mX >= 0 and lp >= aa - 3
    const uint32_t mw = ld32u(src + (mp + 4 <= (int32_t)I.n ? mp : (int32_t)I.n - 4));
    bool ceq = false;
    if (lane < limc) ceq = ld8(src + ipX - 1 - (int32_t)lane) == ld8(src + mX - 1 - (int32_t)lane);
    const uint64_t cst = ballot(!ceq);
    back = cst ? (uint32_t)__builtin_ctzll(cst) : 64u;
    // first byte of this lane's 4 that stops the count: at or after aa, and
    // differing or at or past limit
    const int32_t k = aa - lp, m = limit - lp;
    const uint32_t pre = k > 0 ? (0xffffffffu << (8 * (uint32_t)k)) : 0xffffffffu;
    const uint32_t lim = m >= 4 ? 0u : (m <= 0 ? 0xffffffffu : (0xffffffffu << (8 * (uint32_t)m)));
    const uint32_t y = ((C.w ^ mw) | lim) & pre;
    const uint32_t si = y ? (uint32_t)__builtin_ctz(y) >> 3 : 4u;
    const uint64_t sm = ballot(si < 4);
    if (sm) {
        const int L = __builtin_ctzll(sm);
        return uni((uint32_t)((int32_t)(C.w0 + 4 * L) - (int32_t)I.sh + (int32_t)readlane(si, L) - aa));
    }
    // a long match: continue 256 bytes per step from the window's end
    const uint32_t avail = limit > aa ? (uint32_t)(limit - aa) : 0u;
    uint32_t mc = (uint32_t)((int32_t)(C.w0 + 256) - (int32_t)I.sh - aa);
    return uni(mc >= avail ? avail : mc + count_wave(src + aa + mc, src + mX + 4 + mc, src + limit, lane));
}

// jzc::parse_fast on the wave: same sequences, same table, same repcodes.
__device__ uint32_t parse_fast_wave(const uint8_t *src, int32_t istart, int32_t iend, uint32_t *htab, jzc::Params P,
                                    uint32_t rep[2], WSeq &ss, uint32_t lane) {
    const uint32_t hlog = P.hlog, mls = P.mls;
    const int32_t endIndex = iend + 1;
    const int32_t prefixStartIndex = jzc::prefix_start_index(endIndex, P.wlog);
    const int32_t prefixStart = prefixStartIndex - 1;
    const int32_t ilimit = iend - 8;
    int32_t ip0 = istart, anchor = istart;
    uint32_t offset_1 = rep[0], offset_2 = rep[1], offsetSaved = 0;
    ip0 += (ip0 == prefixStart);
    {
        const int32_t cur = ip0 + 1;
        const int32_t windowLow = jzc::prefix_start_index(cur, P.wlog);
        const uint32_t maxRep = (uint32_t)(cur - windowLow);
        if (offset_2 > maxRep) offsetSaved = offset_2, offset_2 = 0;
        if (offset_1 > maxRep) offsetSaved = offset_1, offset_1 = 0;
    }
    const uint8_t *const iendp = src + iend;
    gu32c *const T = (gu32c *)htab;
    // speculation width: a step evaluates the next K iterations of the serial
    // loop (a prefix, so the semantics are unchanged).  Each iteration costs a
    // random hash-table read and a random candidate read; on text the first
    // success comes within a few iterations, so after every match a step starts
    // with JFSX_ZC_K0 lanes and doubles K on each step without a success.
    uint32_t K = JFSX_ZC_K0;
    while (ip0 + 1 < ilimit) {
        // ---- one search step: iterations j = 0..K-1 of the serial loop ----
        const int32_t d0 = ip0 - anchor;
        int32_t d;
        if (d0 < 2) {
            d = d0 + 2 * (int32_t)lane;  // every step is 2 while d < 128
        } else {
            int32_t x = d0;
            d = d0;
            for (uint32_t j = 0; j < K; j++) {
                if (lane == j) d = x;
                x += (x >> 7) + 2;
            }
        }
        const int32_t p = anchor + d;
        const uint64_t amask = K >= 64 ? ~0ull : ((1ull << K) - 1ull);
        const bool valid = lane < K && p + 1 < ilimit;
        const uint64_t vmask = ballot(valid);
        const int32_t pc = valid ? p : ip0;
        uint64_t w0, w1;
        load9(src, pc, w0, w1);
        const uint32_t A = hash_w(w0, hlog, mls), B = hash_w(w1, hlog, mls);
        const int32_t tA0 = (int32_t)T[A], tB0 = (int32_t)T[B];
        const uint32_t v0 = (uint32_t)w0, v1 = (uint32_t)w1, r2 = (uint32_t)(w0 >> 16);
        const bool okr = valid && offset_1 > 0 && ld32u(src + pc + 2 - (int32_t)offset_1) == r2;
        bool ok0 = valid && tA0 > prefixStartIndex && ld32u(src + tA0 - 1) == v0;
        bool ok1 = valid && tB0 > prefixStartIndex && ld32u(src + tB0 - 1) == v1;
        int32_t tA = tA0, tB = tB0;
        uint64_t sm = ballot(okr || ok0 || ok1);
        uint64_t commit;
        bool wA, wB;
        if (sm & 1ull) {
            // the first iteration succeeds on its own: it alone ran
            commit = 1ull;
            wA = lane == 0 && A != B;
            wB = lane == 0;
        } else {
            // lanes whose writes share this lane's buckets: bit i of eqXY is
            // set when lane i's hash Y equals this lane's hash X
            uint64_t eqAA = ~0ull, eqBA = ~0ull, eqAB = ~0ull, eqBB = ~0ull;
            if (K <= 16) {
                // a narrow step: compare with each active lane's hashes directly
                eqAA = eqBA = eqAB = eqBB = 0ull;
                for (uint32_t i = 0; i < K; i++) {
                    const uint32_t Ai = readlane(A, (int)i), Bi = readlane(B, (int)i);
                    const uint64_t bit = 1ull << i;
                    eqAA |= A == Ai ? bit : 0ull;
                    eqBA |= A == Bi ? bit : 0ull;
                    eqAB |= B == Ai ? bit : 0ull;
                    eqBB |= B == Bi ? bit : 0ull;
                }
            } else {
                // hashLog x 2 ballots
                for (uint32_t bit = 0; bit < hlog; bit++) {
                    const bool a = (A >> bit) & 1u, b = (B >> bit) & 1u;
                    const uint64_t bA = ballot(a), bB = ballot(b);
                    eqAA &= a ? bA : ~bA;
                    eqBA &= a ? bB : ~bB;
                    eqAB &= b ? bA : ~bA;
                    eqBB &= b ? bB : ~bB;
                }
            }
            eqAA &= vmask;
            eqBA &= vmask;
            eqAB &= vmask;
            eqBB &= vmask;
            const uint64_t below = lanes_below(lane), above = lanes_above(lane);
            // reads: the latest earlier write to the bucket (B after A within an iteration)
            {
                const uint64_t ea = eqAA & below, eb = eqBA & below;
                const int ia = ea ? 63 - __builtin_clzll(ea) : -1, ib = eb ? 63 - __builtin_clzll(eb) : -1;
                const int src_l = ib >= ia ? ib : ia;
                const int32_t pv = __shfl(p, src_l < 0 ? (int)lane : src_l, 64);
                if (src_l >= 0) tA = pv + (ib >= ia ? 2 : 1);
            }
            {
                const uint64_t ea = eqAB & below, eb = eqBB & below;
                const int ia = ea ? 63 - __builtin_clzll(ea) : -1, ib = eb ? 63 - __builtin_clzll(eb) : -1;
                const int src_l = ib >= ia ? ib : ia;
                const int32_t pv = __shfl(p, src_l < 0 ? (int)lane : src_l, 64);
                if (src_l >= 0) tB = pv + (ib >= ia ? 2 : 1);
            }
            if (tA != tA0) ok0 = valid && tA > prefixStartIndex && ld32u(src + tA - 1) == v0;
            if (tB != tB0) ok1 = valid && tB > prefixStartIndex && ld32u(src + tB - 1) == v1;
            sm = ballot(okr || ok0 || ok1);
            commit = sm ? ((sm & (0ull - sm)) << 1) - 1ull : vmask;  // iterations that ran
            const bool in = (commit >> lane) & 1ull;
            wA = in && A != B && !((eqAA | eqBA) & above & commit);
            wB = in && !((eqAB | eqBB) & above & commit);
        }
        if (wA) T[A] = (uint32_t)(p + 1);
        if (wB) T[B] = (uint32_t)(p + 2);
        if (!sm) {
            if (vmask != amask) break;  // the serial loop ends inside this step
            ip0 = anchor + unis(readlanes(d + (d >> 7) + 2, (int)K - 1));
            K = K < 32 ? 2 * K : 64;  // any K0: never past 64
            continue;
        }
        K = JFSX_ZC_K0;
        // ---- the match of the first successful iteration f ----
        const int f = __builtin_ctzll(sm);
        const int32_t pf = unis(readlanes(p, f));
        const bool fr = (readlane((uint32_t)okr, f) & 1u) != 0, f0 = (readlane((uint32_t)ok0, f) & 1u) != 0;
        const int32_t current0 = pf + 1;
        int32_t match0;
        uint32_t mLength, offcode;
        if (fr) {
            const int32_t ip2 = pf + 2, repMatch = ip2 - (int32_t)offset_1;
            mLength = ld8(src + ip2 - 1) == ld8(src + repMatch - 1) ? 1u : 0u;
            ip0 = ip2 - (int32_t)mLength;
            match0 = repMatch - (int32_t)mLength;
            mLength += 4;
            offcode = 0;
        } else {
            if (f0) {
                ip0 = pf;
                match0 = unis(readlanes(tA, f)) - 1;
            } else {
                ip0 = pf + 1;
                match0 = unis(readlanes(tB, f)) - 1;
            }
            offset_2 = offset_1;
            offset_1 = (uint32_t)(ip0 - match0);
            offcode = offset_1 + 2;
            mLength = 4;
            const uint32_t lim = (uint32_t)min(ip0 - anchor, match0 - prefixStart);
            const uint32_t back = lim ? back_wave(src + ip0, src + match0, lim, lane) : 0u;
            ip0 -= (int32_t)back;
            match0 -= (int32_t)back;
            mLength += back;
        }
        mLength += count_wave(src + ip0 + mLength, src + match0 + mLength, iendp, lane);
        mLength = uni(mLength);
        store_seq_wave(ss, src + anchor, (uint32_t)(ip0 - anchor), offcode, mLength - 3, lane);
        ip0 += (int32_t)mLength;
        anchor = ip0;
        if (ip0 <= ilimit) {
            if (lane == 0) {
                T[hash_w(ld64u(src + current0 + 1), hlog, mls)] = (uint32_t)(current0 + 2);
                T[hash_w(ld64u(src + ip0 - 2), hlog, mls)] = (uint32_t)(ip0 - 1);
            }
            while (ip0 <= ilimit && offset_2 > 0 && uni(ld32u(src + ip0)) == uni(ld32u(src + ip0 - (int32_t)offset_2))) {
                const uint32_t rLength = uni(count_wave(src + ip0 + 4, src + ip0 + 4 - offset_2, iendp, lane)) + 4;
                const uint32_t t = offset_2;
                offset_2 = offset_1;
                offset_1 = t;
                if (lane == 0) T[hash_w(ld64u(src + ip0), hlog, mls)] = (uint32_t)(ip0 + 1);
                ip0 += (int32_t)rLength;
                store_seq_wave(ss, src + anchor, 0, 0, rLength - 3, lane);
                anchor = ip0;
            }
        }
    }
    rep[0] = offset_1 ? offset_1 : offsetSaved;
    rep[1] = offset_2 ? offset_2 : offsetSaved;
    return (uint32_t)(iend - anchor);
}

// parse_fast_wave with the input reads served from register windows where
// they fall inside one (JFSX_ZC_WIN): the same sequences, table and repcodes.
// W covers the search step's positions; C, loaded by count_back at the
// match, covers the match's end, the next anchor and often the next step.
// ZWF (JFSX_ZC_WIN bits): 1 search positions, 2 count_back, 4 literal copies,
// 8 hash inserts and repcode loop, 16 the match window as the next search window,
// 256 candidate extensions (ZExt): a short match needs no count_back.  (Bits
// 32, 64 and 128 -- everything after a match from one round of loads, the
// next step's table reads in that round, repcode windows -- were measured
// slower or equal and removed: profiles/r4/ab_zstdc_win.txt.)
constexpr int ZWF = JFSX_ZC_WIN == 1 ? 31 : JFSX_ZC_WIN;
__device__ uint32_t parse_fast_wave_w(const uint8_t *src, const ZImg I, int32_t istart, int32_t iend, uint32_t *htab,
                                      jzc::Params P, uint32_t rep[2], WSeq &ss, uint32_t lane) {
    const uint32_t hlog = P.hlog, mls = P.mls;
    const int32_t endIndex = iend + 1;
    const int32_t prefixStartIndex = jzc::prefix_start_index(endIndex, P.wlog);
    const int32_t prefixStart = prefixStartIndex - 1;
    const int32_t ilimit = iend - 8;
    int32_t ip0 = istart, anchor = istart;
    uint32_t offset_1 = rep[0], offset_2 = rep[1], offsetSaved = 0;
    ip0 += (ip0 == prefixStart);
    {
        const int32_t cur = ip0 + 1;
        const int32_t windowLow = jzc::prefix_start_index(cur, P.wlog);
        const uint32_t maxRep = (uint32_t)(cur - windowLow);
        if (offset_2 > maxRep) offsetSaved = offset_2, offset_2 = 0;
        if (offset_1 > maxRep) offsetSaved = offset_1, offset_1 = 0;
    }
    const uint8_t *const iendp = src + iend;
    gu32c *const T = (gu32c *)htab;
    // speculation width: a step evaluates the next K iterations of the serial
    // loop (a prefix, so the semantics are unchanged).  Each iteration costs a
    // random hash-table read and a random candidate read; on text the first
    // success comes within a few iterations, so after every match a step starts
    // with JFSX_ZC_K0 lanes and doubles K on each step without a success.
    uint32_t K = JFSX_ZC_K0;
    ZWin W, C;
    W.w0 = C.w0 = 0xfffff000u;  // empty
    W.w = C.w = 0;
    while (ip0 + 1 < ilimit) {
        // ---- one search step: iterations j = 0..K-1 of the serial loop ----
        const int32_t d0 = ip0 - anchor;
        int32_t d;
        if (d0 < 2) {
            d = d0 + 2 * (int32_t)lane;  // every step is 2 while d < 128
        } else {
            int32_t x = d0;
            d = d0;
            for (uint32_t j = 0; j < K; j++) {
                if (lane == j) d = x;
                x += (x >> 7) + 2;
            }
        }
        const int32_t p = anchor + d;
        const uint64_t amask = K >= 64 ? ~0ull : ((1ull << K) - 1ull);
        const bool valid = lane < K && p + 1 < ilimit;
        const uint64_t vmask = ballot(valid);
        const int32_t pc = valid ? p : ip0;
        // the step's positions [ip0, p of lane K-1] (+ 8 bytes each, + the
        // hash insert at pf + 2) from W, reloaded at ip0 when it does not cover them
        const int32_t phi = unis(readlanes(p, (int)K - 1));
        const uint32_t span = (uint32_t)(phi - ip0) + 16u;
        bool win = (ZWF & 1) && zw_has(W, I, ip0, span);
        if ((ZWF & 1) && !win && span <= 240u) {
            zw_load(W, I, (uint32_t)ip0, lane);
            win = true;
        }
        uint64_t w0, w1;
        if (win)
            zw_load9(W, I, pc, w0, w1);
        else
            load9(src, pc, w0, w1);
        const uint32_t A = hash_w(w0, hlog, mls), B = hash_w(w1, hlog, mls);
        const int32_t tA0 = (int32_t)T[A], tB0 = (int32_t)T[B];
        const uint32_t v0 = (uint32_t)w0, v1 = (uint32_t)w1, r2 = (uint32_t)(w0 >> 16);
        // the repcode candidate: from W when every active lane's lies inside it
        const int32_t q = pc + 2 - (int32_t)offset_1;
        const bool rq = valid && offset_1 > 0;
        bool okr;
        if (win && !ballot(rq && !zw_has(W, I, q, 8))) {
            // every lane takes part in the ds_bpermute (a lane masked off
            // would hand 0 to the lanes reading its dword); lanes without a
            // repcode candidate read their own position
            const uint32_t qv = zw_u32_lane(W, I, rq ? q : pc);
            okr = rq && qv == r2;
        } else
            okr = rq && ld32u(src + q) == r2;
        ZExt XA, XB;
        bool ok0, ok1;
        if (ZWF & 256) {
            zx_load(XA, I, tA0 - 1);
            zx_load(XB, I, tB0 - 1);
            const uint32_t sA = (uint32_t)(tA0 - 1 + (int32_t)I.sh) & 3u, sB = (uint32_t)(tB0 - 1 + (int32_t)I.sh) & 3u;
            ok0 = valid && tA0 > prefixStartIndex &&
                  (XA.in ? __builtin_amdgcn_alignbyte(XA.e[2], XA.e[1], sA) : ld32u(src + tA0 - 1)) == v0;
            ok1 = valid && tB0 > prefixStartIndex &&
                  (XB.in ? __builtin_amdgcn_alignbyte(XB.e[2], XB.e[1], sB) : ld32u(src + tB0 - 1)) == v1;
        } else {
            ok0 = valid && tA0 > prefixStartIndex && ld32u(src + tA0 - 1) == v0;
            ok1 = valid && tB0 > prefixStartIndex && ld32u(src + tB0 - 1) == v1;
        }
        int32_t tA = tA0, tB = tB0;
        uint64_t sm = ballot(okr || ok0 || ok1);
        uint64_t commit;
        bool wA, wB;
        if (sm & 1ull) {
            // the first iteration succeeds on its own: it alone ran
            commit = 1ull;
            wA = lane == 0 && A != B;
            wB = lane == 0;
        } else {
            // lanes whose writes share this lane's buckets: bit i of eqXY is
            // set when lane i's hash Y equals this lane's hash X
            uint64_t eqAA = ~0ull, eqBA = ~0ull, eqAB = ~0ull, eqBB = ~0ull;
            if (K <= 16) {
                // a narrow step: compare with each active lane's hashes directly
                eqAA = eqBA = eqAB = eqBB = 0ull;
                for (uint32_t i = 0; i < K; i++) {
                    const uint32_t Ai = readlane(A, (int)i), Bi = readlane(B, (int)i);
                    const uint64_t bit = 1ull << i;
                    eqAA |= A == Ai ? bit : 0ull;
                    eqBA |= A == Bi ? bit : 0ull;
                    eqAB |= B == Ai ? bit : 0ull;
                    eqBB |= B == Bi ? bit : 0ull;
                }
            } else {
                // hashLog x 2 ballots
                for (uint32_t bit = 0; bit < hlog; bit++) {
                    const bool a = (A >> bit) & 1u, b = (B >> bit) & 1u;
                    const uint64_t bA = ballot(a), bB = ballot(b);
                    eqAA &= a ? bA : ~bA;
                    eqBA &= a ? bB : ~bB;
                    eqAB &= b ? bA : ~bA;
                    eqBB &= b ? bB : ~bB;
                }
            }
            eqAA &= vmask;
            eqBA &= vmask;
            eqAB &= vmask;
            eqBB &= vmask;
            const uint64_t below = lanes_below(lane), above = lanes_above(lane);
            // reads: the latest earlier write to the bucket (B after A within an iteration)
            {
                const uint64_t ea = eqAA & below, eb = eqBA & below;
                const int ia = ea ? 63 - __builtin_clzll(ea) : -1, ib = eb ? 63 - __builtin_clzll(eb) : -1;
                const int src_l = ib >= ia ? ib : ia;
                const int32_t pv = __shfl(p, src_l < 0 ? (int)lane : src_l, 64);
                if (src_l >= 0) tA = pv + (ib >= ia ? 2 : 1);
            }
            {
                const uint64_t ea = eqAB & below, eb = eqBB & below;
                const int ia = ea ? 63 - __builtin_clzll(ea) : -1, ib = eb ? 63 - __builtin_clzll(eb) : -1;
                const int src_l = ib >= ia ? ib : ia;
                const int32_t pv = __shfl(p, src_l < 0 ? (int)lane : src_l, 64);
                if (src_l >= 0) tB = pv + (ib >= ia ? 2 : 1);
            }
            if (tA != tA0) ok0 = valid && tA > prefixStartIndex && ld32u(src + tA - 1) == v0;
            if (tB != tB0) ok1 = valid && tB > prefixStartIndex && ld32u(src + tB - 1) == v1;
            sm = ballot(okr || ok0 || ok1);
            commit = sm ? ((sm & (0ull - sm)) << 1) - 1ull : vmask;  // iterations that ran
            const bool in = (commit >> lane) & 1ull;
            wA = in && A != B && !((eqAA | eqBA) & above & commit);
            wB = in && !((eqAB | eqBB) & above & commit);
        }
        if (wA) T[A] = (uint32_t)(p + 1);
        if (wB) T[B] = (uint32_t)(p + 2);
        if (!sm) {
            if (vmask != amask) break;  // the serial loop ends inside this step
            ip0 = anchor + unis(readlanes(d + (d >> 7) + 2, (int)K - 1));
            K = K < 32 ? 2 * K : 64;  // any K0: never past 64
            continue;
        }
        K = JFSX_ZC_K0;
        // ---- the match of the first successful iteration f ----
        const int f = __builtin_ctzll(sm);
        const int32_t pf = unis(readlanes(p, f));
        const bool fr = (readlane((uint32_t)okr, f) & 1u) != 0, f0 = (readlane((uint32_t)ok0, f) & 1u) != 0;
        const int32_t current0 = pf + 1;
        int32_t match0;
        uint32_t mLength, offcode;
        uint32_t back;
        if (fr) {
            // the repcode match extends one byte back when ip2[-1] == repMatch[-1]
            const int32_t ip2 = pf + 2, repMatch = ip2 - (int32_t)offset_1;
            uint32_t mc;
            if (ZWF & 2) {
                mc = count_back(C, I, src, ip2, repMatch, iend, 1u, back, lane);
            } else {
                back = ld8(src + ip2 - 1) == ld8(src + repMatch - 1) ? 1u : 0u;
                mc = uni(count_wave(src + ip2 + 4, src + repMatch + 4, src + iend, lane));
                C.w0 = 0xfffff000u;
            }
            ip0 = ip2 - (int32_t)back;
            match0 = repMatch - (int32_t)back;
            mLength = 4 + back + mc;
            offcode = 0;
        } else {
            int32_t ipX;
            if (f0) {
                ipX = pf;
                match0 = unis(readlanes(tA, f)) - 1;
            } else {
                ipX = pf + 1;
                match0 = unis(readlanes(tB, f)) - 1;
            }
            offset_2 = offset_1;
            offset_1 = (uint32_t)(ipX - match0);
            offcode = offset_1 + 2;
            const uint32_t lim = (uint32_t)min(ipX - anchor, match0 - prefixStart);
            uint32_t mc = 0;
            bool fast = false;
            if (ZWF & 256) {
                // a short match from the winner's extension and W: catch-up
                // (<= 4 bytes) and ZSTD_count's first 12 bytes
                const int32_t t0 = unis(readlanes(f0 ? tA0 : tB0, f));
                const bool inf = (readlane((uint32_t)(f0 ? XA.in : XB.in), f) & 1u) != 0;
                if (t0 - 1 == match0 && inf) {
                    uint32_t u[6];
#pragma unroll
                    for (int k = 0; k < 6; k++) u[k] = uni(readlane(f0 ? XA.e[k] : XB.e[k], f));
                    const uint32_t s = (uint32_t)(match0 + (int32_t)I.sh) & 3u;
                    const uint32_t L = (uint32_t)(iend - (ipX + 4));
                    bool okf = false, okb = false;
                    uint32_t mcf = 0, bk = 0;
                    if (zw_has(W, I, ipX + 4, 20)) {
                        const uint64_t c1 = zw_u64(W, I, ipX + 4);
                        const uint32_t c2 = (uint32_t)zw_u64(W, I, ipX + 12);
                        const uint64_t m1 = (uint64_t)__builtin_amdgcn_alignbyte(u[3], u[2], s) |
                                            ((uint64_t)__builtin_amdgcn_alignbyte(u[4], u[3], s) << 32);
                        const uint32_t m2 = __builtin_amdgcn_alignbyte(u[5], u[4], s);
                        const uint64_t x1 = c1 ^ m1;
                        const uint32_t x2 = c2 ^ m2;
                        const uint32_t j = x1 ? (uint32_t)__builtin_ctzll(x1) >> 3
                                              : x2 ? 8u + ((uint32_t)__builtin_ctz(x2) >> 3) : 12u;
                        if (j < 12u || L <= 12u) {
                            mcf = j < L ? j : L;
                            okf = true;
                        }
                    }
                    if (lim == 0) {
                        okb = true;
                    } else if (zw_has(W, I, ipX - 4, 12)) {
                        const uint32_t y = (uint32_t)zw_u64(W, I, ipX - 4) ^ __builtin_amdgcn_alignbyte(u[1], u[0], s);
                        const uint32_t eq = y ? (uint32_t)__builtin_clz(y) >> 3 : 4u;
                        if (eq < 4u || lim <= 4u) {
                            bk = eq < lim ? eq : lim;
                            okb = true;
                        }
                    }
                    if (okf && okb) {
                        mc = mcf;
                        back = bk;
                        fast = true;
                        C = W;
                    }
                }
            }
            if (fast) {
            } else if (ZWF & 2) {
                mc = count_back(C, I, src, ipX, match0, iend, lim < 64u ? lim : 64u, back, lane);
                if (back == 64u && lim > 64u) back = 64u + back_wave(src + ipX - 64, src + match0 - 64, lim - 64u, lane);
            } else {
                back = lim ? back_wave(src + ipX, src + match0, lim, lane) : 0u;
                mc = uni(count_wave(src + ipX + 4, src + match0 + 4, src + iend, lane));
                C.w0 = 0xfffff000u;
            }
            ip0 = ipX - (int32_t)back;
            match0 -= (int32_t)back;
            mLength = 4 + back + mc;
        }
        mLength = uni(mLength);
        if ((ZWF & 4) && zw_has(W, I, anchor, (uint32_t)(ip0 - anchor)))
            store_seq_win(ss, W, I, anchor, (uint32_t)(ip0 - anchor), offcode, mLength - 3, lane);
        else
            store_seq_wave(ss, src + anchor, (uint32_t)(ip0 - anchor), offcode, mLength - 3, lane);
        ip0 += (int32_t)mLength;
        anchor = ip0;
        if (ip0 <= ilimit) {
            {
                const uint64_t h1 = (ZWF & 8) && zw_has(W, I, current0 + 1, 12) ? zw_u64(W, I, current0 + 1)
                                                                              : ld64u(src + current0 + 1);
                const uint64_t h2 = (ZWF & 8) && zw_has(C, I, ip0 - 2, 12) ? zw_u64(C, I, ip0 - 2) : ld64u(src + ip0 - 2);
                if (lane == 0) {
                    T[hash_w(h1, hlog, mls)] = (uint32_t)(current0 + 2);
                    T[hash_w(h2, hlog, mls)] = (uint32_t)(ip0 - 1);
                }
            }
            for (;;) {
                if (!(ip0 <= ilimit && offset_2 > 0)) break;
                const uint32_t a = (ZWF & 8) && zw_has(C, I, ip0, 8) ? (uint32_t)zw_u64(C, I, ip0) : uni(ld32u(src + ip0));
                const int32_t rp = ip0 - (int32_t)offset_2;
                const uint32_t bq = (ZWF & 8) && zw_has(C, I, rp, 12) ? (uint32_t)zw_u64(C, I, rp) : uni(ld32u(src + rp));
                if (a != bq) break;
                const uint64_t h3 = (ZWF & 8) && zw_has(C, I, ip0, 12) ? zw_u64(C, I, ip0) : ld64u(src + ip0);
                uint32_t b0;
                const uint32_t rLength =
                    ((ZWF & 2) ? count_back(C, I, src, ip0, rp, iend, 0u, b0, lane)
                               : uni(count_wave(src + ip0 + 4, src + rp + 4, src + iend, lane))) + 4;
                const uint32_t t = offset_2;
                offset_2 = offset_1;
                offset_1 = t;
                if (lane == 0) T[hash_w(h3, hlog, mls)] = (uint32_t)(ip0 + 1);
                ip0 += (int32_t)rLength;
                store_seq_wave(ss, src + anchor, 0, 0, rLength - 3, lane);
                anchor = ip0;
            }
        }
        // the next search starts at anchor: C often covers it already
        if ((ZWF & 16) && zw_has(C, I, anchor, 2 * JFSX_ZC_K0 + 16)) W = C;
    }
    rep[0] = offset_1 ? offset_1 : offsetSaved;
    rep[1] = offset_2 ? offset_2 : offsetSaved;
    return (uint32_t)(iend - anchor);
}

// the entropy stage of one block, on one lane (called by lane 0 only)
__device__ __noinline__ uint64_t block_body_lane(jzc::Work *W, jzc::SeqDef *seqs, uint8_t *lits, uint8_t *codes,
                                                 uint32_t nseq, uint32_t nlit, uint32_t long_id, uint32_t long_pos,
                                                 uint8_t *body, uint32_t bs) {
    jzc::SeqStore ss;
    ss.seq = seqs;
    ss.lit = lits;
    ss.llc = codes;
    ss.mlc = codes + jzc::kMaxSeq;
    ss.ofc = codes + 2 * jzc::kMaxSeq;
    ss.nseq = nseq;
    ss.nlit = nlit;
    ss.long_id = long_id;
    ss.long_pos = long_pos;
    return jzc::compress_block_body(W->prev, W->next, ss, body, jzc::kBodyCap, bs, W->litCount, W->hufScratch, W->hw,
                                    W->sw);
}

__device__ __noinline__ uint32_t frame_header_lane(uint8_t *dst, uint64_t n, jzc::Params P) {
    return jzc::write_frame_header(dst, n, P);
}

// ---------------------------------------------------------------------------
// The entropy stage on the wave.  Table building (Huffman tree, FSE
// normalisation and spreads: a few hundred entries) stays on lane 0 with the
// library's serial code; the per-symbol work is spread over the lanes:
// histograms (LDS atomics), the sequence codes, the Huffman streams and the
// sequence bit stream.  A bit stream is the concatenation, in emission order,
// of fixed bit strings, so each lane emits its own run of symbols at an
// offset from a suffix scan of the runs' lengths, OR-ing 32-bit words into a
// zeroed destination.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) uint16_t gu16c;

// exclusive suffix sum within groups of w lanes: sum of x over the group's
// higher lanes
__device__ __forceinline__ uint32_t suffix_excl(uint32_t x, uint32_t lane, uint32_t w) {
    uint32_t v = x;
    for (uint32_t d = 1; d < w; d <<= 1) {
        const uint32_t y = __shfl_down(v, d, (int)w);
        if ((lane % w) + d < w) v += y;
    }
    return v - x;
}

// OR the low nb bits of v into the bit stream at bit q (words of base)
__device__ __forceinline__ void or_bits(uint32_t *base, uint64_t q, uint64_t v, uint32_t nb) {
    if (!nb) return;
    v &= nb >= 64 ? ~0ull : ((1ull << nb) - 1);
    const uint32_t sh = (uint32_t)(q & 31);
    uint32_t *w = base + (q >> 5);
    const uint64_t lo = v << sh;
    atomicOr(w, (uint32_t)lo);
    if (sh + nb > 32) atomicOr(w + 1, (uint32_t)(lo >> 32));
    if (sh + nb > 64) atomicOr(w + 2, (uint32_t)(v >> (64 - sh)));
}

// zero exactly the bytes [a, b) of the word-aligned body (the bytes around
// belong to headers already written)
__device__ __forceinline__ void zero_range(uint8_t *body, uint32_t a, uint32_t b, uint32_t lane) {
    const uint32_t wa = min((a + 3) & ~3u, b), wb = max(b & ~3u, wa);
    if (lane < wa - a) *(gu8c *)(body + a + lane) = 0;
    if (lane < b - wb) *(gu8c *)(body + wb + lane) = 0;
    for (uint32_t i = wa + 4 * lane; i < wb; i += 256) *(gu32c *)(body + i) = 0;
}

__device__ __forceinline__ void wave_sync() { __syncthreads(); }

// ---------------------------------------------------------------------------
// Byte runs and bulk copies with several loads in flight per lane.  A loop
// that loads a byte and then stores or ORs it pays a memory round trip per
// iteration: the stores may alias the next iteration's load, so the load
// waits.  Here each lane loads 16 bytes per step and a step's loads go out
// before its stores (and before the previous step's work where that helps).
// ---------------------------------------------------------------------------
typedef unsigned int zv4a __attribute__((ext_vector_type(4)));
// 16 bytes at byte offset off of the 4-byte aligned image a; dwords past
// dlast (the last one holding a wanted byte) read as 0, so no dword without
// a wanted byte is touched
__device__ __forceinline__ void ld16r(const uint8_t *a, uint32_t off, uint32_t dlast, uint32_t r[4]) {
    const uint32_t d = off >> 2, sh = off & 3;
    uint32_t w[5];
#pragma unroll
    for (int k = 0; k < 5; k++) w[k] = d + k <= dlast ? ld32a(a + 4 * (d + k)) : 0u;
#pragma unroll
    for (int k = 0; k < 4; k++) r[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
}
__device__ __forceinline__ uint32_t byte_of(const uint32_t r[4], int k) { return (r[k >> 2] >> (8 * (k & 3))) & 255u; }

// dst[0, n) = src[0, n), global to global, any alignment, no overlap: 16 bytes
// per lane, 4 KiB per wave step, a step's loads before its stores
__device__ __noinline__ void copy_run(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t lane) {
    if (!n) return;
    const uintptr_t sx = (uintptr_t)src;
    const uint8_t *sa = (const uint8_t *)(sx & ~(uintptr_t)3);
    const uint32_t ssh = (uint32_t)(sx & 3), dlast = (ssh + n - 1) >> 2;
    const bool dal = ((uintptr_t)dst & 3) == 0;
    for (uint32_t base = 0; base < n; base += 4096) {
        uint32_t r[4][4];
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint32_t o = base + 1024 * g + 16 * lane;
            if (o < n) ld16r(sa, ssh + o, dlast, r[g]);
        }
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint32_t o = base + 1024 * g + 16 * lane;
            if (o < n) {
                const uint32_t c = min(16u, n - o);
                uint8_t *d = dst + o;
                if (c == 16 && dal) {
#pragma unroll
                    for (int k = 0; k < 4; k++) *(gu32c *)(d + 4 * k) = r[g][k];
                } else {
#pragma unroll
                    for (int k = 0; k < 16; k++)
                        if ((uint32_t)k < c) *(gu8c *)(d + k) = (uint8_t)byte_of(r[g], k);
                }
            }
        }
    }
}
// the same, one byte per lane per iteration (the round-3 loop; A/B)
__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src, uint32_t n, uint32_t lane) {
#if JFSX_ZC_MLP & 1
    copy_run(dst, src, n, lane);
#else
    for (uint32_t o = lane; o < n; o += 64) *(gu8c *)(dst + o) = (uint8_t)ld8(src + o);
#endif
}

// histogram of the bytes p[0, n) (p 4-byte aligned, readable up to the next
// dword) into LDS counters by atomics
__device__ __forceinline__ void hist_bytes(uint32_t *cnt, const uint8_t *p, uint32_t n, uint32_t lane) {
#if JFSX_ZC_MLP & 2
#pragma unroll 4
    for (uint32_t i = 4 * lane; i < n; i += 256) {
        const uint32_t w = ld32a(p + i);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (i + k < n) atomicAdd(&cnt[(w >> (8 * k)) & 255u], 1u);
    }
#else
    for (uint32_t i = lane; i < n; i += 64) atomicAdd(&cnt[ld8(p + i)], 1u);
#endif
}
// diagnostic build (-DJFSX_ZC_TRACE): lane 0 prints each stage of the entropy
// stage as it is reached (device printf is a hostcall: lines appear while the
// kernel runs, so a hang shows its last stage)
#ifdef JFSX_ZC_TRACE
#define ZT(...)                                    \
    do {                                           \
        if (threadIdx.x == 0) printf(__VA_ARGS__); \
    } while (0)
#else
#define ZT(...) \
    do {        \
    } while (0)
#endif

// HUF_compress_internal without the encoding: 0 not compressible, 1 RLE,
// 2 encode with the old table (W->next.ct), 3 encode with the new table
// (header of *hSize bytes written at hdr; W->next.ct = the new table)
__device__ __noinline__ uint32_t huf_plan_lane(jzc::Work *W, uint8_t *hdr, uint64_t cap, uint32_t n, uint32_t maxSym,
                                               uint32_t largest, bool preferRepeat, uint32_t *hSizeOut,
                                               uint32_t *repeatOut) {
    uint32_t repeat = W->prev.repeat;
    *repeatOut = repeat;
    *hSizeOut = 0;
    if (preferRepeat && repeat == jzc::kHufValid) return 2;
    if (largest == n) return 1;
    if (largest <= (n >> 7) + 4) return 0;
    if (repeat == jzc::kHufCheck) {
        bool bad = false;
        for (uint32_t s = 0; s <= maxSym; s++) bad |= (W->litCount[s] != 0) & (W->next.ct.nb[s] == 0);
        if (bad) repeat = jzc::kHufNone;
    }
    *repeatOut = repeat;
    if (preferRepeat && repeat != jzc::kHufNone) return 2;
    uint32_t huffLog = jzc::fse_optimal_table_log(jzc::kHufLogDefault, n, maxSym, 1);
    huffLog = jzc::huf_build_ctable(W->hufScratch, W->litCount, maxSym, huffLog, W->hw);
    const uint64_t hSize = jzc::huf_write_ctable(hdr, cap, W->hufScratch, maxSym, huffLog, W->hw);
    if (hSize == 0) return 0;
    if (repeat != jzc::kHufNone) {
        uint64_t oldBits = 0, newBits = 0;
        for (uint32_t s = 0; s <= maxSym; s++) {
            oldBits += (uint64_t)W->next.ct.nb[s] * W->litCount[s];
            newBits += (uint64_t)W->hufScratch.nb[s] * W->litCount[s];
        }
        if ((oldBits >> 3) <= hSize + (newBits >> 3) || hSize + 12 >= n) return 2;
    }
    if (hSize + 12 >= n) return 0;
    *repeatOut = jzc::kHufNone;
    W->next.ct = W->hufScratch;
    *hSizeOut = (uint32_t)hSize;
    return 3;
}

// The Huffman streams of n literals (HUF_compress1X / 4X_usingCTable):
// returns their size in bytes (4X: with the 6-byte jump table), or 0 when
// they would not fit in cap.  out is byte offset `o` of the word-aligned body.
__device__ uint32_t huf_streams_wave(uint8_t *body, uint32_t o, uint32_t cap, const uint8_t *lit, uint32_t n, bool single,
                                     const jzc::HufCT &ct, uint32_t lane) {
    __shared__ uint32_t sz[4];
    const uint32_t w = single ? 64 : 16;  // lanes per stream
    const uint32_t s = lane / w, j = lane % w;
    const uint32_t seg = single ? n : (n + 3) / 4;
    const uint32_t s0 = s * seg, slen = single ? n : (s < 3 ? seg : n - 3 * seg);
    const uint32_t per = (slen + w - 1) / w;
    const uint32_t c0 = min(j * per, slen), c1 = min(c0 + per, slen);
    uint32_t bits = 0;
#pragma unroll 8
    for (uint32_t i = c0; i < c1; i++) bits += ct.nb[ld8(lit + s0 + i)];
    const uint32_t before = suffix_excl(bits, lane, w);  // symbols after this run come first
    const uint32_t total = __shfl(before + bits, (int)(s * w), 64);  // the stream's bits (group lane 0)
    if (j == 0) sz[s] = (total + 1 + 7) >> 3;  // with the end mark
    wave_sync();
    const uint32_t nstreams = single ? 1 : 4;
    uint32_t start = o + (single ? 0 : 6), end = start;
    uint32_t my0 = start;
    for (uint32_t k = 0; k < nstreams; k++) {
        if (k == s) my0 = end;
        end += sz[k];
    }
    my0 = single ? start : my0;
    if (end + 16 > cap) return 0;  // the library's bit streams would overflow their buffers
    zero_range(body, start, end, lane);
    wave_sync();
    // this lane's run, last symbol first, from bit `before` of its stream
    uint64_t q = 8ull * my0 + before;
#if JFSX_ZC_MLP & 4
    if (c1 > c0) {
        // the run backwards in 16-byte groups, the next group loaded before
        // this one's ORs
        const uintptr_t lx = (uintptr_t)(lit + s0 + c0);
        const uint8_t *la = (const uint8_t *)(lx & ~(uintptr_t)3);
        const uint32_t lsh = (uint32_t)(lx & 3), m = c1 - c0, dlast = (lsh + m - 1) >> 2;
        int32_t gs = (int32_t)((m - 1) & ~15u);
        uint32_t r[4], rn[4];
        ld16r(la, lsh + (uint32_t)gs, dlast, r);
        for (; gs >= 0; gs -= 16) {
            if (gs >= 16) ld16r(la, lsh + (uint32_t)gs - 16, dlast, rn);
#pragma unroll
            for (int k = 15; k >= 0; k--) {
                if ((uint32_t)(gs + k) < m) {
                    const uint32_t b = byte_of(r, k);
                    or_bits((uint32_t *)body, q, ct.val[b], ct.nb[b]);
                    q += ct.nb[b];
                }
            }
#pragma unroll
            for (int k = 0; k < 4; k++) r[k] = rn[k];
        }
    }
#else
    for (int32_t i = (int32_t)c1 - 1; i >= (int32_t)c0; i--) {
        const uint32_t b = ld8(lit + s0 + i);
        or_bits((uint32_t *)body, q, ct.val[b], ct.nb[b]);
        q += ct.nb[b];
    }
#endif
    if (j == 0) or_bits((uint32_t *)body, 8ull * my0 + total, 1, 1);  // end mark
    if (!single && lane == 0) {
        jzc::wr16(body + o, sz[0]);
        jzc::wr16(body + o + 2, sz[1]);
        jzc::wr16(body + o + 4, sz[2]);
    }
    wave_sync();
    return end - o;
}

// literal histogram into W.litCount; returns (maxSym, largest) on every lane
__device__ void hist_literals(jzc::Work &W, const uint8_t *lit, uint32_t n, uint32_t lane, uint32_t &maxSym,
                              uint32_t &largest) {
    for (uint32_t i = lane; i < 256; i += 64) W.litCount[i] = 0;
    wave_sync();
    hist_bytes(W.litCount, lit, n, lane);
    wave_sync();
    uint32_t mx = 0, ms = 0;
    for (uint32_t k = 0; k < 4; k++) {
        const uint32_t sym = 4 * lane + k, c = W.litCount[sym];
        if (c > mx) mx = c;
        if (c) ms = sym;
    }
    for (int d = 32; d > 0; d >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
        ms = max(ms, (uint32_t)__shfl_xor(ms, d, 64));
    }
    maxSym = ms;
    largest = mx;
}

__device__ void copy_huf_state(jzc::HufState &d, const jzc::HufState &s, uint32_t lane) {
    for (uint32_t i = lane; i < 256; i += 64) d.ct.nb[i] = s.ct.nb[i], d.ct.val[i] = s.ct.val[i];
    if (lane == 0) d.repeat = s.repeat;
}

// ZSTD_compressLiterals on the wave: the literal section at body[0..),
// returns its size; W.next as the library leaves nextHuf
__device__ uint32_t literals_wave(jzc::Work &W, uint8_t *body, const uint8_t *lit, uint32_t n, uint32_t lane) {
    __shared__ uint32_t bc[3];
    const uint32_t lhSize = 3 + (n >= 1024) + (n >= 16384);
    bool single = n < 256;
    copy_huf_state(W.next, W.prev, lane);
    const uint32_t fl = 1 + (n > 31) + (n > 4095);
    uint32_t mode = 0, cLit = 0, hType = jzc::kSetCompressed;
    wave_sync();
    if (n > 63) {  // COMPRESS_LITERALS_SIZE_MIN (no table is ever "valid" without a dictionary)
        uint32_t maxSym, largest;
        hist_literals(W, lit, n, lane, maxSym, largest);
        if (lane == 0) {
            uint32_t hs = 0, rep = 0;
            bc[0] = huf_plan_lane(&W, body + lhSize, jzc::kBodyCap - lhSize, n, maxSym, largest, n <= 1024, &hs, &rep);
            bc[1] = hs;
            bc[2] = rep;
        }
        wave_sync();
        mode = uni(bc[0]);
        const uint32_t hSize = uni(bc[1]), repeat = uni(bc[2]);
        if (mode == 1) cLit = 1;
        if (mode >= 2) {
            // mode 2: the old table (W.next = prev); mode 3: the new one, now in W.next
            const uint32_t c = huf_streams_wave(body, lhSize + hSize, jzc::kBodyCap, lit, n, single, W.next.ct, lane);
            cLit = (c == 0 || hSize + c >= n - 1) ? 0u : hSize + c;
        }
        if (repeat != jzc::kHufNone) hType = jzc::kSetRepeat;
    }
    if (n <= 63 || cLit == 0 || cLit >= n - jzc::min_gain(n) || cLit == 1) {
        copy_huf_state(W.next, W.prev, lane);
        wave_sync();
        if (n > 63 && cLit == 1) {
            if (lane == 0) jzc::lit_rle(body, ld8(lit), n);
            wave_sync();
            return fl + 1;
        }
        if (lane == 0) {
            if (fl == 1) body[0] = (uint8_t)(jzc::kSetBasic + (n << 3));
            else if (fl == 2) jzc::wr16(body, jzc::kSetBasic + (1u << 2) + (n << 4));
            else jzc::wr24(body, jzc::kSetBasic + (3u << 2) + (n << 4));
        }
        copy_bytes(body + fl, lit, n, lane);
        wave_sync();
        return fl + n;
    }
    if (lane == 0) {
        if (hType == jzc::kSetCompressed) W.next.repeat = jzc::kHufCheck;
        const uint32_t c = cLit;
        if (lhSize == 3) jzc::wr24(body, hType + ((uint32_t)(!single) << 2) + (n << 4) + (c << 14));
        else if (lhSize == 4) jzc::wr32(body, hType + (2u << 2) + (n << 4) + (c << 18));
        else {
            jzc::wr32(body, hType + (3u << 2) + (n << 4) + (c << 22));
            body[4] = (uint8_t)(c >> 10);
        }
    }
    wave_sync();
    return lhSize + cLit;
}

// code histogram of one kind (HIST_countFast): returns (max present, most frequent)
__device__ void hist_codes_wave(jzc::Work &W, const uint8_t *codes, uint32_t n, uint32_t maxIn, uint32_t lane,
                                uint32_t &maxSym, uint32_t &mostFreq) {
    W.sw.count[lane] = 0;
    wave_sync();
    hist_bytes(W.sw.count, codes, n, lane);
    wave_sync();
    const uint32_t c = lane <= maxIn ? W.sw.count[lane] : 0u;
    uint32_t mx = c, ms = c ? lane : 0u;
    for (int d = 32; d > 0; d >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor(mx, d, 64));
        ms = max(ms, (uint32_t)__shfl_xor(ms, d, 64));
    }
    maxSym = ms;
    mostFreq = mx;
}

__device__ __noinline__ uint32_t build_table_lane(jzc::Work *W, uint8_t *op, uint32_t kind, uint32_t type, uint32_t max,
                                                  const uint8_t *codes, uint32_t nbSeq) {
    if (kind == 0)
        return jzc::build_ctable(op, W->sw.ll, jzc::kLLLog, type, W->sw.count, max, codes, nbSeq, jzc::kLLDef, 6,
                                 jzc::kMaxLL, W->sw);
    if (kind == 1)
        return jzc::build_ctable(op, W->sw.of, jzc::kOffLog, type, W->sw.count, max, codes, nbSeq, jzc::kOFDef, 5,
                                 jzc::kDefaultMaxOff, W->sw);
    return jzc::build_ctable(op, W->sw.ml, jzc::kMLLog, type, W->sw.count, max, codes, nbSeq, jzc::kMLDef, 6,
                             jzc::kMaxML, W->sw);
}

// ZSTD_encodeSequences on the wave.  Lanes 0..2 run the OF / ML / LL state
// chains (serial by nature) recording each transition's output bits; then
// every lane emits a run of sequences.  Returns the stream's size, 0 if it
// would not fit.
__device__ uint32_t sequences_wave(jzc::Work &W, uint8_t *body, uint32_t o, uint32_t cap, const jzc::SeqDef *seq,
                                   const uint8_t *llc, const uint8_t *mlc, const uint8_t *ofc, uint16_t *rec,
                                   uint32_t n, uint32_t lane) {
    __shared__ uint32_t fin[3];
    ZT("zc: seq chains n %u\n", n);
    if (lane < 3) {
        const jzc::FseCT &ct = lane == 0 ? W.sw.of : lane == 1 ? W.sw.ml : W.sw.ll;
        const uint8_t *cd = lane == 0 ? ofc : lane == 1 ? mlc : llc;
        gu16c *r = (gu16c *)(rec + (size_t)lane * jzc::kMaxSeq);
        jzc::FseState st;
        jzc::fse_init_state2(st, ct, ld8(cd + n - 1));
#if JFSX_ZC_MLP & 8
        // the codes in aligned 16-byte groups (cd is 16-byte aligned), the
        // next group's load in flight while this one's 16 steps run
        const int32_t top = (int32_t)n - 2;
        if (top >= 0) {
            typedef __attribute__((address_space(1))) const zv4a gzv4;
            int32_t G = top >> 4;
            zv4a v = *(gzv4 *)(cd + 16 * G), vn = v;
            for (; G >= 0; G--) {
                if (G > 0) vn = *(gzv4 *)(cd + 16 * (G - 1));
                const uint32_t rr[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int k = 15; k >= 0; k--) {
                    const int32_t i = 16 * G + k;
                    if (i <= top) {
                        const uint32_t c = byte_of(rr, k);
                        const uint32_t nb = (st.value + ct.dnb[c]) >> 16;
                        r[i] = (uint16_t)((nb << 12) | (st.value & ((1u << nb) - 1)));
                        st.value = ct.state[(int32_t)(st.value >> nb) + ct.dfs[c]];
                    }
                }
                v = vn;
            }
        }
#else
        for (int32_t i = (int32_t)n - 2; i >= 0; i--) {
            const uint32_t c = ld8(cd + i);
            const uint32_t nb = (st.value + ct.dnb[c]) >> 16;
            r[i] = (uint16_t)((nb << 12) | (st.value & ((1u << nb) - 1)));
            st.value = ct.state[(int32_t)(st.value >> nb) + ct.dfs[c]];
        }
#endif
        fin[lane] = st.value;
    }
    wave_sync();
    // per-sequence bits, runs of sequences per lane (emission: n - 1 first)
    const uint32_t per = (n + 63) / 64;
    const uint32_t c0 = min(lane * per, n), c1 = min(c0 + per, n);
    const gu16c *rOF = (const gu16c *)rec, *rML = rOF + jzc::kMaxSeq, *rLL = rML + jzc::kMaxSeq;
    uint32_t bits = 0;
#pragma unroll 8
    for (uint32_t i = c0; i < c1; i++) {
        const uint32_t l = ld8(llc + i), m = ld8(mlc + i), f = ld8(ofc + i);
        bits += jzc::kLLBits[l] + jzc::kMLBits[m] + f;
        if (i + 1 < n) bits += (rOF[i] >> 12) + (rML[i] >> 12) + (rLL[i] >> 12);
    }
    ZT("zc: seq bits\n");
    const uint32_t before = suffix_excl(bits, lane, 64);
    const uint32_t total = __shfl(before + bits, 0, 64);
    ZT("zc: seq total %u\n", total);
    const uint32_t tl = W.sw.ml.tableLog + W.sw.of.tableLog + W.sw.ll.tableLog;
    const uint32_t bytes = (total + tl + 1 + 7) >> 3;
    if (o + bytes + 16 > cap) return 0;
    zero_range(body, o, o + bytes, lane);
    wave_sync();
    uint64_t q = 8ull * o + before;
    uint32_t *base = (uint32_t *)body;
#if JFSX_ZC_MLP & 16
    constexpr int kG = 4;  // sequences whose inputs are loaded before their ORs
    for (int32_t i0 = (int32_t)c1 - 1; i0 >= (int32_t)c0; i0 -= kG) {
        uint32_t L[kG], M[kG], F[kG], RA[kG], RB[kG], RC[kG];
        jzc::SeqDef D[kG];
#pragma unroll
        for (int k = 0; k < kG; k++) {
            const int32_t i = i0 - k;
            if (i >= (int32_t)c0) {
                L[k] = ld8(llc + i), M[k] = ld8(mlc + i), F[k] = ld8(ofc + i);
                D[k] = seq[i];
                const bool has = (uint32_t)i + 1 < n;
                RA[k] = has ? rOF[i] : 0u, RB[k] = has ? rML[i] : 0u, RC[k] = has ? rLL[i] : 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < kG; k++) {
            if (i0 - k >= (int32_t)c0) {
                const uint32_t a = RA[k], b = RB[k], c = RC[k];
                or_bits(base, q, a & 0xfff, a >> 12);
                q += a >> 12;
                or_bits(base, q, b & 0xfff, b >> 12);
                q += b >> 12;
                or_bits(base, q, c & 0xfff, c >> 12);
                q += c >> 12;
                or_bits(base, q, D[k].ll, jzc::kLLBits[L[k]]);
                q += jzc::kLLBits[L[k]];
                or_bits(base, q, D[k].ml, jzc::kMLBits[M[k]]);
                q += jzc::kMLBits[M[k]];
                or_bits(base, q, D[k].offset, F[k]);
                q += F[k];
            }
        }
    }
#else
    for (int32_t i = (int32_t)c1 - 1; i >= (int32_t)c0; i--) {
        const uint32_t l = ld8(llc + i), m = ld8(mlc + i), f = ld8(ofc + i);
        const jzc::SeqDef d = seq[i];
        if ((uint32_t)i + 1 < n) {
            const uint32_t a = rOF[i], b = rML[i], c = rLL[i];
            or_bits(base, q, a & 0xfff, a >> 12);
            q += a >> 12;
            or_bits(base, q, b & 0xfff, b >> 12);
            q += b >> 12;
            or_bits(base, q, c & 0xfff, c >> 12);
            q += c >> 12;
        }
        or_bits(base, q, d.ll, jzc::kLLBits[l]);
        q += jzc::kLLBits[l];
        or_bits(base, q, d.ml, jzc::kMLBits[m]);
        q += jzc::kMLBits[m];
        or_bits(base, q, d.offset, f);
        q += f;
    }
#endif
    if (lane == 0) {
        uint64_t e = 8ull * o + total;
        or_bits(base, e, fin[1], W.sw.ml.tableLog);
        e += W.sw.ml.tableLog;
        or_bits(base, e, fin[0], W.sw.of.tableLog);
        e += W.sw.of.tableLog;
        or_bits(base, e, fin[2], W.sw.ll.tableLog);
        e += W.sw.ll.tableLog;
        or_bits(base, e, 1, 1);  // end mark
    }
    wave_sync();
    return bytes;
}

// ZSTD_entropyCompressSequences on the wave: the block body in body[0..),
// 0 when the block is stored raw
__device__ uint64_t block_body_wave(jzc::Work &W, const WSeq &ss, uint8_t *codes, uint16_t *rec, uint8_t *body,
                                    uint32_t bs, uint32_t lane) {
    __shared__ uint32_t bc[2];
    ZT("zc: block body nlit %u nseq %u bs %u\n", ss.nlit, ss.nseq, bs);
    uint32_t op = literals_wave(W, body, ss.lit, ss.nlit, lane);
    ZT("zc: literals -> %u\n", op);
    const uint32_t nbSeq = ss.nseq;
    if (lane == 0) {
        if (nbSeq < 128) {
            body[op] = (uint8_t)nbSeq;
        } else if (nbSeq < jzc::kLongNbSeq) {
            body[op] = (uint8_t)((nbSeq >> 8) + 0x80);
            body[op + 1] = (uint8_t)nbSeq;
        } else {
            body[op] = 0xFF;
            jzc::wr16(body + op + 1, nbSeq - jzc::kLongNbSeq);
        }
    }
    op += nbSeq < 128 ? 1 : nbSeq < jzc::kLongNbSeq ? 2 : 3;
    if (nbSeq != 0) {
        uint8_t *llc = codes, *mlc = codes + jzc::kMaxSeq, *ofc = codes + 2 * jzc::kMaxSeq;
#if JFSX_ZC_MLP & 16
        for (uint32_t i0 = lane; i0 < nbSeq; i0 += 256) {
            jzc::SeqDef D[4];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++)
                if (i0 + 64 * k < nbSeq) D[k] = ss.seq[i0 + 64 * k];
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t i = i0 + 64 * k;
                if (i < nbSeq) {
                    *(gu8c *)(llc + i) = (uint8_t)jzc::ll_code(D[k].ll);
                    *(gu8c *)(ofc + i) = (uint8_t)jzc::highbit32(D[k].offset);
                    *(gu8c *)(mlc + i) = (uint8_t)jzc::ml_code(D[k].ml);
                }
            }
        }
#else
        for (uint32_t i = lane; i < nbSeq; i += 64) {
            const jzc::SeqDef d = ss.seq[i];
            *(gu8c *)(llc + i) = (uint8_t)jzc::ll_code(d.ll);
            *(gu8c *)(ofc + i) = (uint8_t)jzc::highbit32(d.offset);
            *(gu8c *)(mlc + i) = (uint8_t)jzc::ml_code(d.ml);
        }
#endif
        wave_sync();
        if (lane == 0) {
            if (ss.long_id == 1) llc[ss.long_pos] = jzc::kMaxLL;
            if (ss.long_id == 2) mlc[ss.long_pos] = jzc::kMaxML;
        }
        wave_sync();
        const uint32_t seqHead = op++;
        int32_t lastNCount = -1;
        uint32_t types[3];
        const uint8_t *cds[3] = {llc, ofc, mlc};
        const uint32_t maxIn[3] = {jzc::kMaxLL, jzc::kMaxOff, jzc::kMaxML};
        for (uint32_t k = 0; k < 3; k++) {
            uint32_t max, mf;
            hist_codes_wave(W, cds[k], nbSeq, maxIn[k], lane, max, mf);
            ZT("zc: hist %u max %u mf %u\n", k, max, mf);
            const uint32_t type = k == 1 ? jzc::select_type(mf, nbSeq, 5, max <= jzc::kDefaultMaxOff)
                                         : jzc::select_type(mf, nbSeq, 6, true);
            if (lane == 0) bc[0] = build_table_lane(&W, body + op, k, type, max, cds[k], nbSeq);
            wave_sync();
            const uint32_t t = uni(bc[0]);
            ZT("zc: table %u type %u size %u\n", k, type, t);
            if (type == jzc::kSetCompressed) lastNCount = (int32_t)op;
            op += t;
            types[k] = type;
        }
        if (lane == 0) body[seqHead] = (uint8_t)((types[0] << 6) + (types[1] << 4) + (types[2] << 2));
        if (op + 16 >= jzc::kBodyCap) return 0;
        ZT("zc: sequences at %u\n", op);
        const uint32_t b = sequences_wave(W, body, op, jzc::kBodyCap, ss.seq, llc, mlc, ofc, rec, nbSeq, lane);
        ZT("zc: sequences -> %u\n", b);
        if (b == 0) return 0;
        op += b;
        if (lastNCount >= 0 && (int32_t)op - lastNCount < 4) return 0;
    }
    if (op >= bs - jzc::min_gain(bs)) return 0;
    return op;
}

// ZSTD_compress(level 1) of one object by the wave
#ifdef JFSX_ZC_STAMP
// diagnostic build only: the wave's wall-clock ticks (100 MHz) in the parse
// and the entropy stage, and the sequences found (one wave per workgroup, so
// LDS words are per wave); waves 0..1 print them per object
__shared__ uint64_t g_zc_parse, g_zc_entropy, g_zc_nseq;
#endif
__device__ uint64_t compress_object(const uint8_t *src, uint64_t n, uint8_t *dst, uint32_t *htab,
                                    jzc::SeqDef *seqs, uint8_t *lits, uint8_t *codes, uint8_t *body, uint16_t *rec,
                                    jzc::Work &W, uint32_t lane) {
    const jzc::Params P = jzc::level1_params(n);
    ZT("zc: params %u %u %u\n", P.wlog, P.hlog, P.mls);
    __shared__ uint32_t bcast;
    if (lane == 0) bcast = frame_header_lane(dst, n, P);
    ZT("zc: header %u\n", bcast);
    __syncthreads();
    uint64_t op = uni(bcast);
    ZT("zc: op %lu\n", (unsigned long)op);
    if (n == 0) {
        if (lane == 0) jzc::wr24(dst + op, 1);
        return op + 3;
    }
    for (uint32_t i = 4 * lane; i < (1u << P.hlog); i += 256)
        htab[i] = htab[i + 1] = htab[i + 2] = htab[i + 3] = 0;
    for (uint32_t i = lane; i < 256; i += 64) W.prev.ct.nb[i] = 0, W.prev.ct.val[i] = 0;
    if (lane == 0) W.prev.repeat = jzc::kHufNone;
    uint32_t rep[2] = {1, 4};
    const uint32_t blockMax = (1u << P.wlog) < jzc::kBlockMax ? (1u << P.wlog) : jzc::kBlockMax;
    bool first = true;
    for (uint64_t pos = 0; pos < n;) {
        const uint32_t bs = (uint32_t)((n - pos) < blockMax ? (n - pos) : blockMax);
        const uint32_t last = (pos + bs == n);
        const uint8_t *ip = src + pos;
        uint64_t cSize = 0;
        if (bs >= 7) {
            WSeq ss{seqs, lits, 0, 0, 0, 0};
            uint32_t nrep[2] = {rep[0], rep[1]};
            __syncthreads();  // the table clear / last block's work has landed
            ZT("zc: parse block at %lu bs %u\n", (unsigned long)pos, bs);
#ifdef JFSX_ZC_STAMP
            const uint64_t t_p0 = wall_clock64();
#endif
#if JFSX_ZC_WIN
            const ZImg I{(const uint8_t *)((uintptr_t)src & ~(uintptr_t)3), (uint32_t)((uintptr_t)src & 3), (uint32_t)n};
            const uint32_t lastLL =
                parse_fast_wave_w(src, I, (int32_t)pos, (int32_t)(pos + bs), htab, P, nrep, ss, lane);
#else
            const uint32_t lastLL = parse_fast_wave(src, (int32_t)pos, (int32_t)(pos + bs), htab, P, nrep, ss, lane);
#endif
#ifdef JFSX_ZC_STAMP
            const uint64_t t_p1 = wall_clock64();
            if (lane == 0) g_zc_parse += t_p1 - t_p0, g_zc_nseq += ss.nseq;
#endif
            ZT("zc: parsed nseq %u lastLL %u\n", ss.nseq, lastLL);
            copy_bytes(lits + ss.nlit, src + pos + bs - lastLL, lastLL, lane);
            ss.nlit += lastLL;
            __syncthreads();  // sequences and literals visible to every lane
#ifdef JFSX_ZC_LANE0_ENTROPY
            if (lane == 0)
                bcast = (uint32_t)block_body_lane(&W, seqs, lits, codes, ss.nseq, ss.nlit, ss.long_id, ss.long_pos,
                                                  body, bs);
            __syncthreads();
            cSize = uni(bcast);
#else
            cSize = block_body_wave(W, ss, codes, rec, body, bs, lane);
            __syncthreads();
#endif
#ifdef JFSX_ZC_STAMP
            if (lane == 0) g_zc_entropy += wall_clock64() - t_p1;
#endif
            if (!first && cSize < jzc::kRleMaxLength) {
                const uint32_t b0 = ld8(ip);
                bool diff = false;
                for (uint32_t o = lane; o < bs; o += 64) diff |= ld8(ip + o) != b0;
                if (!ballot(diff)) cSize = 1;
            }
            if (cSize > 1) {
                rep[0] = uni(nrep[0]);
                rep[1] = uni(nrep[1]);
                // ZSTD_confirmRepcodesAndEntropyTables
                for (uint32_t i = lane; i < 256; i += 64) W.prev.ct.nb[i] = W.next.ct.nb[i], W.prev.ct.val[i] = W.next.ct.val[i];
                if (lane == 0) W.prev.repeat = W.next.repeat;
            }
        }
        if (cSize == 0) {
            if (lane == 0) jzc::wr24(dst + op, last + (bs << 3));
            copy_bytes(dst + op + 3, ip, bs, lane);
            op += 3 + bs;
        } else if (cSize == 1) {
            if (lane == 0) {
                jzc::wr24(dst + op, last + (1u << 1) + (bs << 3));
                dst[op + 3] = ip[0];
            }
            op += 4;
        } else {
            if (lane == 0) jzc::wr24(dst + op, last + (2u << 1) + ((uint32_t)cSize << 3));
            copy_bytes(dst + op + 3, body, (uint32_t)cSize, lane);
            op += 3 + cSize;
        }
        pos += bs;
        first = false;
    }
    return op;
}
}  // namespace

// Wave w compresses objects w, w + W, w + 2W, ... (W = gridDim.x): a loop
// whose trip count lives in SGPRs, so every lane runs it in lock-step.  (The
// first version took objects from an atomic queue through an LDS word; the
// compiler nested that loop so that lanes 1..63 re-ran the object loop
// waiting for lane 0's next queue read while lane 0 was masked off -- a hang on
// the first object, GPU-traced in round 3.)  ZDev.len = input bytes,
// ZDev.cap >= ZSTD_compressBound.
// queue != nullptr: after its first object (blockIdx.x) a wave takes the next
// object index from a ticket counter (lane 0's vector atomic, made wave-uniform
// by readfirstlane before the loop test), so a batch of more objects than
// waves finishes in about n / W object times instead of ceil(n / W).
// 4 waves per SIMD (<= 128 VGPRs): with the 9.3 KiB Work, 16 objects per CU
// are in flight, which is what a latency-bound parser needs
#ifndef JFSX_ZC_WPE
#define JFSX_ZC_WPE 4
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(JFSX_ZC_WPE))) void zstd_compress_k(const ZDev *__restrict__ blks, ZOut *__restrict__ outs,
                                                      uint8_t *__restrict__ scratch, int n,
                                                      uint32_t *__restrict__ queue) {
    __shared__ jzc::Work W;
    const uint32_t lane = threadIdx.x;
    uint8_t *const sc = scratch + (size_t)blockIdx.x * kZcScratchStride;
    uint32_t *const htab = (uint32_t *)sc;
    jzc::SeqDef *const seqs = (jzc::SeqDef *)(sc + kZcHtab);
    uint8_t *const lits = sc + kZcHtab + kZcSeq;
    uint8_t *const codes = lits + kZcLit;
    uint8_t *const body = codes + kZcCodes;
    uint16_t *const rec = (uint16_t *)(body + kZcBody);
    for (int obj = (int)blockIdx.x; obj < n;) {
        const ZDev b = blks[obj];
        ZT("zc: object %d len %lu\n", obj, (unsigned long)b.len);
#ifdef JFSX_ZC_SCALAR
        uint64_t r = 0;
        if (lane == 0) r = jzc::compress_frame(b.src, b.len, b.dst, htab, seqs, lits, codes, body, W);
#else
#ifdef JFSX_ZC_STAMP
        if (lane == 0) g_zc_parse = g_zc_entropy = g_zc_nseq = 0;
        const uint64_t t_o0 = wall_clock64();
#endif
        const uint64_t r = compress_object(b.src, b.len, b.dst, htab, seqs, lits, codes, body, rec, W, lane);
#ifdef JFSX_ZC_STAMP
        if (lane == 0 && blockIdx.x < 2)
            printf("zc-stamp wave %u obj %d len %lu out %lu total %lu parse %lu entropy %lu nseq %lu (100 MHz ticks)\n",
                   blockIdx.x, obj, (unsigned long)b.len, (unsigned long)r, (unsigned long)(wall_clock64() - t_o0),
                   (unsigned long)g_zc_parse, (unsigned long)g_zc_entropy, (unsigned long)g_zc_nseq);
#endif
#endif
        ZT("zc: object %d -> %lu\n", obj, (unsigned long)r);
        if (lane == 0) {
            outs[obj].out_len = r;
            outs[obj].status = JFSX_OK;
        }
        __syncthreads();  // W and the scratch are reused by the next object
        if (queue) {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(queue, 1u);
            obj = (int)gridDim.x + (int)__builtin_amdgcn_readfirstlane(t);
        } else {
            obj += (int)gridDim.x;
        }
    }
}

void launch_zstd_compress(hipStream_t s, int n, int waves, const ZDev *blks, ZOut *outs, uint8_t *scratch,
                          uint32_t *queue) {
    if (n <= 0) return;
    if (queue) (void)hipMemsetAsync(queue, 0, 4, s);
    hipLaunchKernelGGL(zstd_compress_k, dim3(waves), dim3(64), 0, s, blks, outs, scratch, n, queue);
}

}  // namespace jfsx

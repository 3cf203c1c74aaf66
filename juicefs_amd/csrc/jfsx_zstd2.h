// jfsx_zstd2.h -- block-parallel Zstandard frame decoding on gfx950 (device
// only; included by jfsx_zstd.hip after its DevEnv).
//
// Same contract as jzd::decompress (ZSTD_decompress, pkg/compress/compress.go:
// 93-100 as cachedStore.load calls it, pkg/chunk/cached_store.go:680-745), for
// the frames the level-1 compressor writes: one frame, up to kMaxBlk blocks,
// Huffman tables up to log 11.  The serial decoder spends most of its time in
// work that is serial only inside a block (FSE state chains, Huffman streams);
// here one wave decodes one object in four phases:
//   1. scan (wave-uniform, the serial decoder's own header / table code): block
//      headers, literal and sequence section headers; every Huffman and FSE
//      table the frame builds is copied to a per-block slot of the wave's
//      arena, so repeat modes are slot references;
//   2. entropy decode, one LANE per Huffman stream (up to 4 per block) and then
//      one lane per block's sequence stream, each lane with its own backward
//      bit reader and table gathers; sequences are stored as (ll, ml, offset)
//      with repeat offsets kept symbolic in the block's initial repeat state
//      (an offset is a value or max(rep_i - d, 1) of the block's entry state);
//   3. the repeat states chained over the blocks (one step per block);
//   4. execution in frame order, 64 sequences per step, one lane per sequence:
//      output and literal positions by wave prefix sums, literal runs copied
//      by their lanes, then match copies in rounds: a lane goes once its
//      source lies below the first unfinished lane's match (everything below
//      that is written), so no match reads bytes not yet final.
// Every check of the serial decoder is kept; anything it would reject, and any
// frame outside the fast path's shape, returns kFallback and the object is
// decoded again by jzd::decompress, which then produces the exact status.
#pragma once
#include "jfsx_zstd.h"

namespace jzd2 {
using namespace jzd;

// decompress_par results below 0: the object goes to the serial decoder; the
// value says why (jfsx_zblk.reserved = -value - 2 after the batch)
constexpr int32_t kFallback = -3;   // frame shape or header (scan)
constexpr int32_t kFbHuf = -4, kFbSeq = -5, kFbExec = -6, kFbRaw = -7, kFbLast = -8, kFbFcs = -9, kFbSum = -10;
constexpr uint32_t kMaxBlk = 64;                    // blocks per frame (8 MiB of full blocks)
constexpr uint32_t kSlot = 9216;                   // per-block table slot in the arena
constexpr uint32_t kSlotLL = 4096, kSlotML = 6144, kSlotOF = 8192;  // Huffman at 0 (2048 x u16)
constexpr size_t kTabBytes = (size_t)kMaxBlk * kSlot;               // 576 KiB
constexpr size_t kLitCap = ((size_t)4 << 20) + ((size_t)1 << 18);    // literal bytes per object (4 MiB blocks + table rounding)
constexpr uint32_t kSeqCap = 768u << 10;                            // sequences per object (4 MiB of 5-byte matches)
constexpr size_t kLitOff = kTabBytes, kLLMLOff = kLitOff + kLitCap, kOffOff = kLLMLOff + 8ull * kSeqCap;
constexpr size_t kArena = kOffOff + 4ull * kSeqCap;                 // 13.8 MiB per wave
static_assert(kArena == jfsx::kZstdArena, "arena size");
constexpr uint32_t kSym = 0x80000000u;  // symbolic offset: kSym | rep index << 29 | d

// diagnostic counters of -DJFSX_ZSTD_STAMP builds: 0 windows, 1 match rounds,
// 2 far matches fetched before the rounds, 3 sequence output bytes
#ifdef JFSX_ZSTD_STAMP
__device__ unsigned long long g_zstd_counts[4];
#define ZSTAT(k, v) atomicAdd(&g_zstd_counts[k], (unsigned long long)(v))
#else
#define ZSTAT(k, v) ((void)0)
#endif

struct BDesc {
    uint8_t type, ltype, nstreams, hlog;  // type 0 raw, 1 RLE, 2 compressed; ltype as the literal block type
    uint8_t llLog, mlLog, ofLog, pad;
    uint16_t hufSlot, llSlot, mlSlot, ofSlot;
    int32_t in;         // raw / RLE block: input offset of the content
    uint32_t size;      // raw / RLE block: decoded size
    uint32_t litSize;
    int32_t litSrc;     // raw literals: input offset; RLE literals: the byte
    uint32_t litOff;    // Huffman literals: arena literal offset
    int32_t s1, l[4];   // Huffman streams: first stream's input offset, stream lengths
    uint32_t seg;       // 4 streams: bytes per stream (the last gets litSize - 3 seg)
    int32_t seqIn, seqLen;
    uint32_t nbSeq, seqBase;
    uint32_t rep[3];    // repeat offsets on entry (phase 3)
    uint32_t fin[3];    // repeat offsets on exit, symbolic in rep[] (phase 2)
};

// output ring of the execution phase: output position p at ring slot
// (p + (dst mod 16)) mod kRing, so flushes are aligned 16-byte stores
constexpr uint32_t kRing = 8192, kRingMask = kRing - 1, kWinMax = 4096;
constexpr uint32_t kWinBytes = 1024;  // byte-parallel windows: 64 lanes x 16 output bytes
constexpr uint16_t kDone = 0xffff;
constexpr uint32_t kLitStage = 512;  // literal bytes a byte-parallel window stages in LDS

struct Shared {
    union {
        Tables t;  // scan: table building
        struct {   // execution: recent output, and the byte-parallel window
            __attribute__((aligned(16))) uint8_t ring[kRing];
            uint16_t ptr[kWinBytes];  // window byte -> earlier window byte it copies, or kDone
        };
    };
    uint4 seqtab[65];  // byte-parallel window: per sequence (start, match start, offset, literal index)
    uint32_t litst[kLitStage / 4 + 1];  // byte-parallel window: its literal bytes (from an aligned dword)
    BDesc d[kMaxBlk];
    uint8_t smap[4 * kMaxBlk];  // Huffman stream -> block | stream index << 6
    uint8_t qmap[kMaxBlk];      // sequence stream -> block
};

static_assert(sizeof(Tables) >= kRing + 2 * kWinBytes, "ring and pointers overlay the tables");

struct Frame {
    uint32_t nblk, nstreams, nseqblk;
    uint32_t hasFcs, checksum, want;
    uint64_t fcs;
};

// ---------------------------------------------------------------------------
// per-lane input reads (bytes outside [0, n) read as zero)
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const uint32_t gcu32;
typedef __attribute__((address_space(1))) const uint8_t gcu8;
typedef __attribute__((address_space(1))) uint8_t gu8;

__device__ __forceinline__ uint32_t lin8(const uint8_t *src, int32_t n, int32_t i) {
    return (i < 0 || i >= n) ? 0u : (uint32_t) * (gcu8 *)(src + i);
}
// bytes [i, i + 8), all inside the input: aligned dword loads (the third only
// when unaligned, and then it holds byte i + 7)
__device__ __forceinline__ uint64_t lin64u(const uint8_t *src, int32_t i) {
    const uintptr_t a = (uintptr_t)src + (uint32_t)i;
    const uintptr_t al = a & ~(uintptr_t)3;
    const uint32_t sh = 8 * (uint32_t)(a & 3);
    const uint64_t lo = (uint64_t) * (gcu32 *)al | ((uint64_t) * (gcu32 *)(al + 4) << 32);
    if (!sh) return lo;
    const uint64_t hi = *(gcu32 *)(al + 8);
    return (lo >> sh) | (hi << (64 - sh));
}
__device__ __forceinline__ uint64_t lin64(const uint8_t *src, int32_t n, int32_t i) {
    if (i >= 0 && i + 8 <= n) return lin64u(src, i);
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v |= (uint64_t)lin8(src, n, i + k) << (8 * k);
    return v;
}

// backward bit reader of one lane: the serial decoder's Bwd (jfsx_zstd.h) with
// per-lane state, same over-read rules
struct LBwd {
    const uint8_t *src;
    int32_t n, base, rem, cb;
    uint64_t cont;
    __device__ __forceinline__ void fill() {
        const int32_t top = (rem - 1) >> 3;
        if (top >= 7) {
            cb = top - 7;
            cont = lin64u(src, base + cb);
        } else {
            cb = 0;
            cont = lin64(src, n, base);
        }
    }
    __device__ __forceinline__ bool init(const uint8_t *s, int32_t insize, int32_t b, int32_t len) {
        src = s;
        n = insize;
        if (len <= 0) return false;
        const uint32_t last = lin8(s, insize, b + len - 1);
        if (last == 0) return false;
        base = b;
        rem = 8 * (len - 1) + (int32_t)highbit(last);
        cb = 1 << 30;
        cont = 0;
        fill();
        return true;
    }
    __device__ __forceinline__ uint32_t peek(uint32_t k) {
        const int32_t lo = rem - (int32_t)k;
        if (rem > cb * 8 + 64 || (lo < cb * 8 && cb > 0)) fill();
        const int32_t sh = lo - cb * 8;
        if (sh >= 0) return (uint32_t)((cont >> sh) & ((1ull << k) - 1));
        if (rem <= 0) return 0;
        return (uint32_t)((cont << (uint32_t)(-sh)) & ((1ull << k) - 1));
    }
    __device__ __forceinline__ uint32_t read(uint32_t k) {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        rem -= (int32_t)k;
        return v;
    }
    __device__ __forceinline__ bool ensure(uint32_t t) {
        if (rem - (int32_t)t >= cb * 8) return true;
        if (cb == 0) return false;
        fill();
        return rem - (int32_t)t >= cb * 8;
    }
    __device__ __forceinline__ uint32_t take(uint32_t k) {
        rem -= (int32_t)k;
        return (uint32_t)(cont >> ((uint32_t)(rem - cb * 8) & 63u)) & ((1u << k) - 1u);
    }
};

template <uint32_t KIND>
__device__ __forceinline__ SeqDec seq_dec(uint32_t w) {
    SeqDec d;
    d.next = w & 511u;
    d.nbBits = (w >> 9) & 15u;
    d.addBits = (w >> 13) & 31u;
    d.base = KIND == 2 ? 1u << d.addBits : (((w >> 18) & 63u) << ((w >> 24) & 15u)) + (KIND == 1 ? 3u : 0u);
    return d;
}

__device__ __forceinline__ uint32_t resolve(uint32_t v, uint32_t r0, uint32_t r1, uint32_t r2) {
    if (!(v & kSym)) return v;
    const uint32_t s = (v >> 29) & 3u, d = v & 0x1fffffffu;
    const uint32_t x = s == 0 ? r0 : s == 1 ? r1 : r2;
    return x > d ? x - d : 1u;
}

__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// copies one LDS table to an arena slot with the 64 lanes
__device__ __forceinline__ void put_table(uint8_t *slot, const void *lds, uint32_t bytes, uint32_t lane) {
    for (uint32_t i = 4 * lane; i < bytes; i += 256)
        *(__attribute__((address_space(1))) uint32_t *)(slot + i) = *(const uint32_t *)((const char *)lds + i);
}

// ---------------------------------------------------------------------------
// phase 1: frame and block headers, tables into arena slots
// ---------------------------------------------------------------------------
template <class Env>
__device__ __forceinline__ int32_t scan_block(Env &e, Shared &S, Mode &m, uint8_t *arena, BDesc &D, uint32_t bi, int32_t p,
                              int32_t n, uint32_t &litTotal, uint32_t &seqTotal, uint16_t (&slots)[4]) {
    Tables &t = S.t;
    if (n >= (int32_t)kBlockMax || n < 3) return kFallback;
    const int32_t end = p + n;
    const uint32_t h0 = e.in8(p);
    const uint32_t ltype = h0 & 3, sf = (h0 >> 2) & 3;
    uint32_t litSize, nst = 0, hl = 0, seg = 0, litOff = 0;
    int32_t lused, litSrc = 0, s1 = 0, ls[4] = {0, 0, 0, 0};
    if (ltype == 0 || ltype == 1) {
        uint32_t lh;
        if (sf == 0 || sf == 2) {
            lh = 1;
            litSize = h0 >> 3;
        } else if (sf == 1) {
            lh = 2;
            litSize = (h0 | (e.in8(p + 1) << 8)) >> 4;
        } else {
            lh = 3;
            litSize = (h0 | (e.in8(p + 1) << 8) | (e.in8(p + 2) << 16)) >> 4;
        }
        if (ltype == 0) {
            if (lh + litSize > (uint32_t)n) return kFallback;
            litSrc = p + lh;
            lused = lh + litSize;
        } else {
            if (sf == 3 && n < 4) return kFallback;
            if (litSize > kBlockMax) return kFallback;
            litSrc = e.in8(p + lh);
            lused = lh + 1;
        }
    } else {
        if (ltype == 3 && m.hufLog == 0) return kFallback;
        if (n < 5) return kFallback;
        const uint32_t lhc = e.in8(p) | (e.in8(p + 1) << 8) | (e.in8(p + 2) << 16) | ((uint32_t)e.in8(p + 3) << 24);
        uint32_t lh, litC;
        bool single = false;
        if (sf <= 1) {
            single = sf == 0;
            lh = 3;
            litSize = (lhc >> 4) & 0x3ff;
            litC = (lhc >> 14) & 0x3ff;
        } else if (sf == 2) {
            lh = 4;
            litSize = (lhc >> 4) & 0x3fff;
            litC = lhc >> 18;
        } else {
            lh = 5;
            litSize = (lhc >> 4) & 0x3ffff;
            litC = (lhc >> 22) + ((uint32_t)e.in8(p + 4) << 10);
        }
        if (litSize > kBlockMax) return kFallback;
        if (litC + lh > (uint32_t)n) return kFallback;
        int32_t q = p + lh, qn = litC;
        if (ltype == 2) {
            const int32_t hs = huf_table(e, t, q, qn, hl);
            if (hs < 0 || hs >= qn || hl > kHufLogTab) return kFallback;
            m.hufLog = hl;
            slots[0] = (uint16_t)bi;
            put_table(arena + (size_t)bi * kSlot, t.huf, 2u << hl, e.lane);
            q += hs;
            qn -= hs;
        }
        hl = m.hufLog;
        if (single) {
            nst = 1;
            s1 = q;
            ls[0] = qn;
            seg = litSize;
        } else {
            if (litSize == 0) return kFallback;
            if (qn < 10) return kFallback;
            ls[0] = e.in8(q) | (e.in8(q + 1) << 8);
            ls[1] = e.in8(q + 2) | (e.in8(q + 3) << 8);
            ls[2] = e.in8(q + 4) | (e.in8(q + 5) << 8);
            ls[3] = qn - (ls[0] + ls[1] + ls[2] + 6);
            if (ls[3] < 0) return kFallback;
            seg = (litSize + 3) / 4;
            if (3 * seg > litSize) return kFallback;
            nst = 4;
            s1 = q + 6;
        }
        litOff = litTotal;
        litTotal += (litSize + 15) & ~15u;
        if (litTotal > kLitCap) return kFallback;
        lused = lh + litC;
    }
    // sequences section
    int32_t s = p + lused;
    if (s >= end) return kFallback;
    uint32_t nbSeq = e.in8(s++);
    if (nbSeq == 0) {
        if (s != end) return kFallback;
    } else {
        if (nbSeq > 0x7f) {
            if (nbSeq == 0xff) {
                if (s + 2 > end) return kFallback;
                nbSeq = (e.in8(s) | (e.in8(s + 1) << 8)) + 0x7f00;
                s += 2;
            } else {
                if (s >= end) return kFallback;
                nbSeq = ((nbSeq - 0x80) << 8) + e.in8(s);
                s++;
            }
        }
        if (s + 1 > end) return kFallback;
        const uint32_t modes = e.in8(s++);
        int32_t u;
        if ((u = seq_table(e, t, m, KLL, modes >> 6, s, end)) < 0) return kFallback;
        if ((modes >> 6) != 3) {
            slots[1] = (uint16_t)bi;
            put_table(arena + (size_t)bi * kSlot + kSlotLL, t.ll, 4u << m.llLog, e.lane);
        }
        s += u;
        if ((u = seq_table(e, t, m, KOF, (modes >> 4) & 3, s, end)) < 0) return kFallback;
        if (((modes >> 4) & 3) != 3) {
            slots[3] = (uint16_t)bi;
            put_table(arena + (size_t)bi * kSlot + kSlotOF, t.of, 4u << m.ofLog, e.lane);
        }
        s += u;
        if ((u = seq_table(e, t, m, KML, (modes >> 2) & 3, s, end)) < 0) return kFallback;
        if (((modes >> 2) & 3) != 3) {
            slots[2] = (uint16_t)bi;
            put_table(arena + (size_t)bi * kSlot + kSlotML, t.ml, 4u << m.mlLog, e.lane);
        }
        s += u;
        if (end - s <= 0) return kFallback;
        m.seqEntropy = true;
    }
    if (e.lane == 0) {
        D.type = 2;
        D.ltype = (uint8_t)ltype;
        D.nstreams = (uint8_t)nst;
        D.hlog = (uint8_t)hl;
        D.llLog = (uint8_t)m.llLog;
        D.mlLog = (uint8_t)m.mlLog;
        D.ofLog = (uint8_t)m.ofLog;
        D.hufSlot = slots[0];
        D.llSlot = slots[1];
        D.mlSlot = slots[2];
        D.ofSlot = slots[3];
        D.litSize = litSize;
        D.litSrc = litSrc;
        D.litOff = litOff;
        D.s1 = s1;
        for (int k = 0; k < 4; k++) D.l[k] = ls[k];
        D.seg = seg;
        D.seqIn = s;
        D.seqLen = end - s;
        D.nbSeq = nbSeq;
        D.seqBase = seqTotal;
    }
    seqTotal += nbSeq;
    if (seqTotal > kSeqCap) return kFallback;
    return 0;
}

template <class Env>
__device__ __forceinline__ int32_t scan(Env &e, Shared &S, uint8_t *arena, uint32_t insize, Frame &F) {
    const int32_t n = (int32_t)insize;
    int32_t p = 0;
    if (n < 9) return kFallback;
    const uint32_t magic = e.in8(0) | (e.in8(1) << 8) | (e.in8(2) << 16) | ((uint32_t)e.in8(3) << 24);
    if (magic != 0xFD2FB528u) return kFallback;  // skippable or foreign frames: the serial decoder
    const uint32_t fhd = e.in8(p + 4);
    const uint32_t dictCode = fhd & 3, checksum = (fhd >> 2) & 1, single = (fhd >> 5) & 1, fcsId = fhd >> 6;
    const int32_t hsize = 5 + (single ? 0 : 1) + (dictCode == 3 ? 4 : dictCode) +
                          (fcsId == 0 ? (single ? 1 : 0) : fcsId == 1 ? 2 : fcsId == 2 ? 4 : 8);
    if (n - p < hsize + 3) return kFallback;
    if (fhd & 0x08) return kFallback;
    int32_t q = p + 5;
    if (!single) {
        const uint32_t wl = e.in8(q++);
        if ((wl >> 3) + 10 > 31) return kFallback;
    }
    uint32_t dict = 0;
    for (uint32_t k = 0, dn = dictCode == 3 ? 4 : dictCode; k < dn; k++) dict |= e.in8(q++) << (8 * k);
    if (dict) return kFallback;
    F.hasFcs = 1;
    F.fcs = 0;
    if (fcsId == 0) {
        if (single) F.fcs = e.in8(q++);
        else F.hasFcs = 0;
    } else {
        const uint32_t fb = fcsId == 1 ? 2 : fcsId == 2 ? 4 : 8;
        for (uint32_t k = 0; k < fb; k++) F.fcs |= (uint64_t)e.in8(q++) << (8 * k);
        if (fcsId == 1) F.fcs += 256;
    }
    Mode m;
    m.hufLog = 0;
    m.llLog = m.mlLog = m.ofLog = 0;
    m.seqEntropy = false;
    uint16_t slots[4] = {0, 0, 0, 0};
    uint32_t litTotal = 0, seqTotal = 0, nb = 0, nst = 0, nsq = 0;
    for (;;) {
        if (n - q < 3) return kFallback;
        const uint32_t bh = e.in8(q) | (e.in8(q + 1) << 8) | (e.in8(q + 2) << 16);
        q += 3;
        const uint32_t lastb = bh & 1, btype = (bh >> 1) & 3, bsize = bh >> 3;
        const int32_t csize = btype == 1 ? 1 : (int32_t)bsize;
        if (btype == 3) return kFallback;
        if (csize > n - q) return kFallback;
        if (nb == kMaxBlk) return kFallback;
        BDesc &D = S.d[nb];
        if (btype == 0 || btype == 1) {
            if (e.lane == 0) {
                D.type = (uint8_t)btype;
                D.in = q;
                D.size = bsize;
                D.nbSeq = 0;
                D.nstreams = 0;
            }
        } else {
            if (scan_block(e, S, m, arena, D, nb, q, csize, litTotal, seqTotal, slots) < 0) return kFallback;
            const uint32_t ns = uni(D.nstreams), nq = uni(D.nbSeq) ? 1u : 0u;
            for (uint32_t k = 0; k < ns; k++)
                if (e.lane == 0) S.smap[nst + k] = (uint8_t)(nb | k << 6);
            nst += ns;
            if (nq && e.lane == 0) S.qmap[nsq] = (uint8_t)nb;
            nsq += nq;
        }
        nb++;
        q += csize;
        if (lastb) break;
    }
    F.checksum = checksum;
    if (checksum) {
        if (n - q < 4) return kFallback;
        F.want = e.in8(q) | (e.in8(q + 1) << 8) | (e.in8(q + 2) << 16) | ((uint32_t)e.in8(q + 3) << 24);
        q += 4;
    }
    if (q != n) return kFallback;  // one frame only (concatenated frames: the serial decoder)
    F.nblk = nb;
    F.nstreams = nst;
    F.nseqblk = nsq;
    return 0;
}

// ---------------------------------------------------------------------------
// phase 2: one Huffman stream per lane (huf_stream of the serial decoder)
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool huf_lane(const uint8_t *src, int32_t insize, const uint16_t *tab, uint32_t hlog,
                                         int32_t p, int32_t len, uint8_t *out, uint32_t cnt) {
    LBwd b;
    if (!b.init(src, insize, p, len)) return false;
    const __attribute__((address_space(1))) uint16_t *h = (const __attribute__((address_space(1))) uint16_t *)tab;
    const uint32_t mask = (1u << hlog) - 1u;
    uint32_t k = 0;
    const bool al = ((uintptr_t)out & 3) == 0;
    for (; k + 4 <= cnt && b.ensure(4 * hlog); k += 4) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) {
            const uint32_t ent = h[(uint32_t)(b.cont >> ((uint32_t)(b.rem - (int32_t)hlog - b.cb * 8) & 63u)) & mask];
            b.rem -= (int32_t)(ent >> 8);
            w |= (ent & 255u) << (8 * i);
        }
        if (al) {
            *(__attribute__((address_space(1))) uint32_t *)(out + k) = w;
        } else {
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) *(gu8 *)(out + k + i) = (uint8_t)(w >> (8 * i));
        }
    }
    for (; k < cnt; k++) {
        const uint32_t ent = h[b.peek(hlog)];
        b.rem -= (int32_t)(ent >> 8);
        *(gu8 *)(out + k) = (uint8_t)ent;
    }
    return b.rem == 0;
}

// one block's sequence stream per lane: (ll, ml) and the offset (a value, or
// kSym | i << 29 | d = max(rep_i - d, 1) of the block's entry repeats).
// Returns false where the serial decoder would reject the block.
__device__ __forceinline__ bool seq_lane(const uint8_t *src, int32_t insize, const uint8_t *slotLL, const uint8_t *slotML,
                                         const uint8_t *slotOF, uint32_t llLog, uint32_t mlLog, uint32_t ofLog,
                                         int32_t p, int32_t len, uint32_t nbSeq, uint64_t *llml, uint32_t *offs,
                                         uint32_t fin[3]) {
    typedef __attribute__((address_space(1))) const uint32_t g32;
    LBwd b;
    if (!b.init(src, insize, p, len)) return false;
    uint32_t sl = b.read(llLog), so = b.read(ofLog), sm = b.read(mlLog);
    uint32_t r0 = kSym, r1 = kSym | (1u << 29), r2 = kSym | (2u << 29);
    bool ok = true;
    for (uint32_t k = 0; k < nbSeq; k++) {
        if (b.rem < 0) {
            ok = false;
            break;
        }
        const SeqDec dl = seq_dec<KLL>(((g32 *)slotLL)[sl]), dm = seq_dec<KML>(((g32 *)slotML)[sm]),
                     dof = seq_dec<KOF>(((g32 *)slotOF)[so]);
        const uint32_t ofc = dof.addBits;
        const uint32_t ll0 = dl.base == 0 && dl.addBits == 0 ? 1u : 0u;
        uint32_t off, ml, ll;
        const bool fast = b.ensure(ofc + dm.addBits + dl.addBits + dl.nbBits + dm.nbBits + dof.nbBits);
        auto rd = [&](uint32_t nb) -> uint32_t { return fast ? (nb ? b.take(nb) : 0u) : b.read(nb); };
        if (ofc > 1) {
            off = dof.base + rd(ofc) - 3;
            if (off & kSym) ok = false;  // never below the output position: rejected when executed
            r2 = r1;
            r1 = r0;
            r0 = off;
        } else if (ofc == 0) {
            if (!ll0) {
                off = r0;
            } else {
                off = r1;
                r1 = r0;
                r0 = off;
            }
        } else {
            const uint32_t idx = 1 + ll0 + rd(1);
            uint32_t tmp;
            if (idx == 3) {
                if (r0 & kSym) {
                    tmp = r0 + 1;  // d + 1
                    if ((tmp & 0x1fffffffu) == 0) ok = false;
                } else {
                    tmp = r0 - 1;
                    tmp += !tmp;
                }
            } else {
                tmp = idx == 2 ? r2 : r1;
            }
            if (idx != 1) r2 = r1;
            r1 = r0;
            r0 = tmp;
            off = tmp;
        }
        ml = dm.base + rd(dm.addBits);
        ll = dl.base + rd(dl.addBits);
        sl = dl.next + rd(dl.nbBits);
        sm = dm.next + rd(dm.nbBits);
        so = dof.next + rd(dof.nbBits);
        *(__attribute__((address_space(1))) uint64_t *)(llml + k) = (uint64_t)ll | ((uint64_t)ml << 32);
        *(__attribute__((address_space(1))) uint32_t *)(offs + k) = off;
        if (!ok) break;
    }
    if (b.rem > 0) ok = false;
    fin[0] = r0;
    fin[1] = r1;
    fin[2] = r2;
    return ok;
}

// ---------------------------------------------------------------------------
// phase 4 helpers: per-lane byte copies
// ---------------------------------------------------------------------------
// wave64 prefix sum with DPP (VALU latency, no LDS round trips): row_shr
// 1 / 2 / 4 / 8 scan each row of 16 lanes, row_bcast:15 and row_bcast:31 carry
// the row totals (GFX9 DPP)
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t lane, uint32_t &total) {
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    total = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    (void)lane;
    return x - v;
}

// number of lanes i with v_i <= x, for v non-decreasing over the 64 lanes
__device__ __forceinline__ uint32_t wave_count_le(uint32_t v, uint32_t x) {
    uint32_t c = 0;
#pragma unroll
    for (uint32_t step = 64; step >= 1; step >>= 1) {
        const uint32_t idx = c + step - 1;
        const uint32_t y = __shfl(v, (int)(idx & 63u), 64);
        if (idx < 64 && y <= x) c += step;
    }
    return c;
}

__device__ __forceinline__ void lane_copy(uint8_t *d, const uint8_t *s, uint32_t cnt) {
    uint32_t t = 0;
    for (; t + 4 <= cnt; t += 4) {
        const uint32_t a = *(gcu8 *)(s + t), b2 = *(gcu8 *)(s + t + 1), c = *(gcu8 *)(s + t + 2),
                       e = *(gcu8 *)(s + t + 3);
        *(gu8 *)(d + t) = (uint8_t)a;
        *(gu8 *)(d + t + 1) = (uint8_t)b2;
        *(gu8 *)(d + t + 2) = (uint8_t)c;
        *(gu8 *)(d + t + 3) = (uint8_t)e;
    }
    for (; t < cnt; t++) *(gu8 *)(d + t) = *(gcu8 *)(s + t);
}

__device__ __forceinline__ void lane_fill(uint8_t *d, uint32_t b, uint32_t cnt) {
    for (uint32_t t = 0; t < cnt; t++) *(gu8 *)(d + t) = (uint8_t)b;
}

// out[o + t] = out[o - off + t mod off], t < cnt (sources below o only)
__device__ __forceinline__ void lane_match(uint8_t *dst, uint32_t o, uint32_t off, uint32_t cnt) {
    if (off >= cnt) {
        lane_copy(dst + o, dst + o - off, cnt);
        return;
    }
    const uint8_t *m = dst + o - off;
    uint32_t r = 0;
    for (uint32_t t = 0; t < cnt; t++) {
        *(gu8 *)(dst + o + t) = *(gcu8 *)(m + r);
        r = r + 1 == off ? 0 : r + 1;
    }
}

// Execution state: output below F is in dst (and fenced), output in
// [max(V, W - kRing), W) is in the ring; W = output written so far.
struct Out {
    uint8_t *ring;
    uint8_t *dst;
    uint32_t a;  // dst mod 16
    uint32_t F, V, W;
    __device__ __forceinline__ uint32_t slot(uint32_t p) const { return (p + a) & kRingMask; }
    // ring -> dst for [F, end): head bytes, 16-byte units, tail bytes when `all`
    __device__ __forceinline__ void flush(uint32_t lane, bool all) {
        const uint32_t end = all ? W : ((W + a) & ~15u) - a;
        if (!all && (W + a) < 16u) return;
        if (end <= F) return;
        uint32_t h = ((F + a + 15u) & ~15u) - a;
        if (h > end) h = end;
        if (lane < h - F) *(gu8 *)(dst + F + lane) = ring[slot(F + lane)];
        const uint32_t e16 = ((end + a) & ~15u) - a;
        if (e16 > h) {
            for (uint32_t j = 16 * lane; j < e16 - h; j += 1024) {
                const uint4 v = *(const uint4 *)(ring + slot(h + j));
                jfsx::gst16(dst + h + j, v);
            }
            h = e16;
        }
        if (lane < end - h) *(gu8 *)(dst + h + lane) = ring[slot(h + lane)];
        F = end;
        wave_fence();
    }
    // a byte of earlier output (q < W): ring or dst
    __device__ __forceinline__ uint32_t rd(uint32_t q, uint32_t lim) const {
        return q >= lim ? (uint32_t)ring[slot(q)] : (uint32_t) * (gcu8 *)(dst + q);
    }
};

// ---------------------------------------------------------------------------
// the fast path: decoded size, or kFallback
// ---------------------------------------------------------------------------
template <class Env>
__device__ __forceinline__ int32_t decompress_par(Env &e, Shared &S, uint8_t *arena, uint32_t insize, uint32_t cap) {
    const uint32_t lane = e.lane;
    Frame F;
    if (scan(e, S, arena, insize, F) < 0) return kFallback;
    wave_fence();  // arena tables and LDS descriptors before the lanes read them
    e.stamp(0);    // (-DJFSX_ZSTD_STAMP builds: cycles per phase)
    const uint8_t *src = e.src;
    const int32_t n = (int32_t)insize;
    uint8_t *lit = arena + kLitOff;
    uint64_t *llml = (uint64_t *)(arena + kLLMLOff);
    uint32_t *offs = (uint32_t *)(arena + kOffOff);
    // ---- Huffman streams, one per lane ----
    bool bad = false, badq = false;
    for (uint32_t g0 = 0; g0 < F.nstreams; g0 += 64) {
        const uint32_t g = g0 + lane;
        if (g < F.nstreams) {
            const uint32_t bi = S.smap[g] & 63u, k = S.smap[g] >> 6;
            const BDesc &D = S.d[bi];
            int32_t sp = D.s1;
            for (uint32_t i = 0; i < k; i++) sp += D.l[i];
            const uint32_t cnt = D.nstreams == 1 ? D.litSize : k < 3 ? D.seg : D.litSize - 3 * D.seg;
            if (!huf_lane(src, n, (const uint16_t *)(arena + (size_t)D.hufSlot * kSlot), D.hlog, sp, D.l[k],
                          lit + D.litOff + k * D.seg, cnt))
                bad = true;
        }
    }
    e.stamp(1);
    // ---- sequence streams, one block per lane ----
    for (uint32_t g0 = 0; g0 < F.nseqblk; g0 += 64) {
        const uint32_t g = g0 + lane;
        if (g < F.nseqblk) {
            const uint32_t bi = S.qmap[g];
            BDesc &D = S.d[bi];
            uint32_t fin[3];
            if (!seq_lane(src, n, arena + (size_t)D.llSlot * kSlot + kSlotLL, arena + (size_t)D.mlSlot * kSlot + kSlotML,
                          arena + (size_t)D.ofSlot * kSlot + kSlotOF, D.llLog, D.mlLog, D.ofLog, D.seqIn, D.seqLen,
                          D.nbSeq, llml + D.seqBase, offs + D.seqBase, fin))
                badq = true;
            D.fin[0] = fin[0];
            D.fin[1] = fin[1];
            D.fin[2] = fin[2];
        }
    }
    if (__ballot(bad)) return kFbHuf;
    if (__ballot(badq)) return kFbSeq;
    wave_fence();  // literals and sequences before the execution reads them
    e.stamp(2);
    // ---- repeat offsets chained over the blocks ----
    {
        uint32_t r0 = 1, r1 = 4, r2 = 8;
        for (uint32_t bi = 0; bi < F.nblk; bi++) {
            BDesc &D = S.d[bi];
            if (uni(D.type) == 2 && uni(D.nbSeq)) {
                const uint32_t f0 = uni(D.fin[0]), f1 = uni(D.fin[1]), f2 = uni(D.fin[2]);
                if (lane == 0) {
                    D.rep[0] = r0;
                    D.rep[1] = r1;
                    D.rep[2] = r2;
                }
                const uint32_t n0 = resolve(f0, r0, r1, r2), n1 = resolve(f1, r0, r1, r2), n2 = resolve(f2, r0, r1, r2);
                r0 = n0;
                r1 = n1;
                r2 = n2;
            }
        }
    }
    e.stamp(2);
    // ---- execution in frame order ----
    // Windows of up to kWinMax output bytes go through the LDS ring (a wave's
    // LDS accesses are ordered, so lanes read what earlier lanes and rounds
    // wrote without fences; flushed in aligned 16-byte stores); larger windows,
    // raw and RLE blocks write dst directly after a full flush.
    Out O{S.ring, e.dst, (uint32_t)((uintptr_t)e.dst & 15), 0, 0, 0};
    uint8_t *dst = e.dst;
    for (uint32_t bi = 0; bi < F.nblk; bi++) {
        const BDesc &D = S.d[bi];
        const uint32_t type = uni(D.type);
        if (type != 2) {
            const uint32_t sz = uni(D.size), o = O.W;
            if (sz > cap - o) return kFbRaw;
            O.flush(lane, true);
            const int32_t in = (int32_t)uni((uint32_t)D.in);
            if (type == 0) {
                for (uint32_t j = lane; j < sz; j += 64) *(gu8 *)(dst + o + j) = *(gcu8 *)(src + in + (int32_t)j);
            } else {
                const uint32_t by = lin8(src, n, in);
                for (uint32_t j = lane; j < sz; j += 64) *(gu8 *)(dst + o + j) = (uint8_t)by;
            }
            wave_fence();
            O.W = O.F = O.V = o + sz;
            continue;
        }
        const uint32_t litSize = uni(D.litSize), ltype = uni(D.ltype), nbSeq = uni(D.nbSeq), sb = uni(D.seqBase);
        const uint32_t litSrc = uni((uint32_t)D.litSrc), litOff = uni(D.litOff);
        const uint32_t r0 = uni(D.rep[0]), r1 = uni(D.rep[1]), r2 = uni(D.rep[2]);
        const uint8_t *lsrc = ltype == 0 ? src + (int32_t)litSrc : lit + litOff;
        uint32_t lp = 0;
        // the next step's sequences are loaded while this one executes
        uint64_t nv = 0;
        uint32_t noff = 0;
        if (lane < nbSeq) {
            nv = *(__attribute__((address_space(1))) const uint64_t *)(llml + sb + lane);
            noff = *(__attribute__((address_space(1))) const uint32_t *)(offs + sb + lane);
        }
        for (uint32_t w = 0; w < nbSeq; w += 64) {
            const uint32_t k = w + lane, o = O.W;
            const bool valid = k < nbSeq;
            uint32_t ll = 0, ml = 0, off = 0;
            if (valid) {
                ll = (uint32_t)nv;
                ml = (uint32_t)(nv >> 32);
                off = resolve(noff, r0, r1, r2);
            }
            if (k + 64 < nbSeq) {
                nv = *(__attribute__((address_space(1))) const uint64_t *)(llml + sb + k + 64);
                noff = *(__attribute__((address_space(1))) const uint32_t *)(offs + sb + k + 64);
            }
            uint32_t tll, tall;
            const uint32_t xl = wave_excl_sum(ll, lane, tll);
            const uint32_t xo = wave_excl_sum(ll + ml, lane, tall);
            const uint64_t oj = (uint64_t)o + xo, lj = (uint64_t)lp + xl;
            const bool err = valid && ((uint64_t)ll + ml > (uint64_t)cap - oj || (uint64_t)ll > (uint64_t)litSize - lj ||
                                       (uint64_t)off > oj + ll);
            if (__ballot(err)) return kFbExec;
            bool done = !valid || ml == 0;
            const uint32_t mo = (uint32_t)oj + ll, ms = mo - off, need = ms + (off < ml ? off : ml);
            // the lanes this match waits for: those whose match part
            // [mo_i, oend_i) overlaps its source [ms, need) (sources of
            // overlapping copies come from the first period, [ms, mo))
            uint64_t dep = 0;
            if (tall > kWinBytes) {
                const uint32_t oend = (uint32_t)oj + ll + ml;  // non-decreasing (invalid lanes: the window end)
                const uint32_t ks = wave_count_le(oend, ms);     // lanes ending at or before ms
                const uint32_t ke1 = wave_count_le((uint32_t)oj, need - 1);  // lanes starting before need
                const uint32_t mks = __shfl(mo, (int)(ks & 63u), 64), mke = __shfl(mo, (int)((ke1 - 1) & 63u), 64);
                if (!done && need > o && ke1 > 0) {
                    const uint32_t s0 = need > mks ? ks : ks + 1, e0 = need > mke ? ke1 - 1 : ke1 - 2;
                    if ((int32_t)s0 <= (int32_t)e0 && e0 < 64)
                        dep = (e0 - s0 == 63 ? ~0ull : ((1ull << (e0 - s0 + 1)) - 1)) << s0;
                }
            }
            ZSTAT(0, lane == 0 ? 1 : 0);
            ZSTAT(3, valid ? ll + ml : 0);
            e.stamp(3);
            if (tall <= kWinBytes) {
                // byte-parallel window: lane L owns window bytes [16L, 16L + 16)
                if (o - O.F >= kWinMax) O.flush(lane, false);
                const uint32_t old = o + tall > kRing ? o + tall - kRing : 0u;
                const uint32_t lim = O.V > old ? O.V : old;
                S.seqtab[lane] = make_uint4((uint32_t)oj - o, mo - o, off, (uint32_t)lj - lp);
                if (lane == 0) S.seqtab[64] = make_uint4(tall, tall, 0, 0);
                // the step's literal bytes [lp, lp + tll): aligned dwords into LDS
                const bool stage = ltype != 1 && tll + 3 <= kLitStage;
                const uint32_t lsh = (uint32_t)((uintptr_t)(lsrc + lp) & 3);
                if (stage) {
                    const uintptr_t la = (uintptr_t)(lsrc + lp) - lsh;
                    const uint32_t nd = (lsh + tll + 3) >> 2;
                    for (uint32_t d = lane; d < nd; d += 64) S.litst[d] = *(gcu32 *)(la + 4 * d);
                }
                const uint8_t *lstage = (const uint8_t *)S.litst + lsh;
                const uint32_t r0 = 16 * lane;
                uint32_t j = wave_count_le((uint32_t)oj - o, r0);
                j = j ? j - 1 : 0;
                uint4 sq = S.seqtab[j];
                uint32_t nxt = S.seqtab[j + 1].x;
                uint32_t pend = 0;  // bytes of this lane still copying a window byte
                uint32_t val[16];
#pragma unroll
                for (uint32_t i = 0; i < 16; i++) {
                    const uint32_t r = r0 + i;
                    val[i] = 0;
                    if (r < tall) {
                        while (r >= nxt) {
                            j++;
                            sq = S.seqtab[j];
                            nxt = S.seqtab[j + 1].x;
                        }
                        if (r < sq.y) {  // literal byte
                            val[i] = ltype == 1 ? litSrc
                                     : stage    ? (uint32_t)lstage[sq.w + (r - sq.x)]
                                                : (uint32_t) * (gcu8 *)(lsrc + lp + sq.w + (r - sq.x));
                            S.ptr[r] = kDone;
                        } else {
                            const uint32_t q = o + r - sq.z;  // the byte it copies
                            if (q < o) {
                                val[i] = O.rd(q, lim);
                                S.ptr[r] = kDone;
                            } else {
                                S.ptr[r] = (uint16_t)(q - o);
                                pend |= 1u << i;
                            }
                        }
                    }
                }
#pragma unroll
                for (uint32_t i = 0; i < 16; i++)
                    if (r0 + i < tall && !(pend >> i & 1)) O.ring[O.slot(o + r0 + i)] = (uint8_t)val[i];
                // pointer jumping: a byte whose source is final takes its
                // value (ring written before the kDone mark), else follows
                // the source's pointer; chains halve every pass
                while (__ballot(pend != 0)) {
                    ZSTAT(1, lane == 0 ? 1 : 0);
#pragma unroll
                    for (uint32_t i = 0; i < 16; i++) {
                        if (pend >> i & 1) {
                            const uint32_t r = r0 + i, q = S.ptr[r], pq = S.ptr[q];
                            if (pq == kDone) {
                                O.ring[O.slot(o + r)] = O.ring[O.slot(o + q)];
                                S.ptr[r] = kDone;
                                pend &= ~(1u << i);
                            } else {
                                S.ptr[r] = (uint16_t)pq;
                            }
                        }
                    }
                }
                e.stamp(7);
            } else if (tall <= kWinMax) {
                // ring path: the window's slots must not hold unflushed output
                if (o - O.F >= kWinMax) O.flush(lane, false);
                // sources at or above lim are in the ring, below it in dst
                const uint32_t old = o + tall > kRing ? o + tall - kRing : 0u;
                const uint32_t lim = O.V > old ? O.V : old;
                if (valid) {
                    uint32_t t = 0;
                    if (ltype == 1) {
                        for (; t < ll; t++) O.ring[O.slot((uint32_t)oj + t)] = (uint8_t)litSrc;
                    } else {
                        const uint8_t *ls = lsrc + lj;
                        for (; t + 4 <= ll; t += 4) {
                            const uint32_t b0 = *(gcu8 *)(ls + t), b1 = *(gcu8 *)(ls + t + 1),
                                           b2 = *(gcu8 *)(ls + t + 2), b3 = *(gcu8 *)(ls + t + 3);
                            O.ring[O.slot((uint32_t)oj + t)] = (uint8_t)b0;
                            O.ring[O.slot((uint32_t)oj + t + 1)] = (uint8_t)b1;
                            O.ring[O.slot((uint32_t)oj + t + 2)] = (uint8_t)b2;
                            O.ring[O.slot((uint32_t)oj + t + 3)] = (uint8_t)b3;
                        }
                        for (; t < ll; t++) O.ring[O.slot((uint32_t)oj + t)] = *(gcu8 *)(ls + t);
                    }
                }
                // far matches (source wholly in dst, below lim): no
                // dependency inside the window, so their bytes are loaded
                // now, with the literals, as aligned dwords
                const bool farm = !done && ml <= 32 && off >= ml && ms + ml <= lim;
                uint32_t fw[8];
                if (farm) {
                    const uintptr_t a0 = (uintptr_t)(dst + ms), al = a0 & ~(uintptr_t)3, aend = a0 + ml;
                    const uint32_t sh = (uint32_t)(a0 & 3);
                    uint32_t dw[9];
#pragma unroll
                    for (uint32_t k = 0; k < 9; k++) dw[k] = al + 4 * k < aend ? *(gcu32 *)(al + 4 * k) : 0u;
#pragma unroll
                    for (uint32_t m = 0; m < 8; m++) fw[m] = __builtin_amdgcn_alignbyte(dw[m + 1], dw[m], sh);
                }
                e.stamp(6);
                for (;;) {
                    const uint64_t pend = __ballot(!done);
                    if (!pend) break;
                    ZSTAT(1, lane == 0 ? 1 : 0);
                    if (!done && (dep & pend) == 0) {
                        ZSTAT(2, farm ? 1 : 0);
                        if (farm) {
#pragma unroll
                            for (uint32_t t = 0; t < 32; t++)
                                if (t < ml) O.ring[O.slot(mo + t)] = (uint8_t)(fw[t >> 2] >> (8 * (t & 3)));
                        } else if (off >= 4) {
                            // 4 source bytes per round trip: ms + t + 3 < mo + t
                            for (uint32_t t = 0; t < ml; t += 4) {
                                const uint32_t b0 = O.rd(ms + t, lim), b1 = t + 1 < ml ? O.rd(ms + t + 1, lim) : 0u,
                                               b2 = t + 2 < ml ? O.rd(ms + t + 2, lim) : 0u,
                                               b3 = t + 3 < ml ? O.rd(ms + t + 3, lim) : 0u;
                                O.ring[O.slot(mo + t)] = (uint8_t)b0;
                                if (t + 1 < ml) O.ring[O.slot(mo + t + 1)] = (uint8_t)b1;
                                if (t + 2 < ml) O.ring[O.slot(mo + t + 2)] = (uint8_t)b2;
                                if (t + 3 < ml) O.ring[O.slot(mo + t + 3)] = (uint8_t)b3;
                            }
                        } else {
                            // ms + t reaches this lane's own bytes: written
                            // before they are read (LDS order)
                            for (uint32_t t = 0; t < ml; t++) O.ring[O.slot(mo + t)] = (uint8_t)O.rd(ms + t, lim);
                        }
                        done = true;
                    }
                }
                e.stamp(7);
            } else {
                // a window larger than half the ring: straight to dst
                O.flush(lane, true);
                if (valid && ll) {
                    if (ltype == 1) lane_fill(dst + oj, litSrc, ll);
                    else lane_copy(dst + oj, lsrc + lj, ll);
                }
                wave_fence();
                for (;;) {
                    const uint64_t pend = __ballot(!done);
                    if (!pend) break;
                    if (!done && (dep & pend) == 0) {
                        lane_match(dst, mo, off, ml);
                        done = true;
                    }
                    wave_fence();
                }
                O.F = O.V = o + tall;
            }
            O.W = o + tall;
            lp += tll;
        }
        const uint32_t last = litSize - lp, o = O.W;
        if (last > cap - o) return kFbLast;
        if (last <= kWinMax) {
            if (o - O.F >= kWinMax) O.flush(lane, false);
            for (uint32_t j = lane; j < last; j += 64)
                O.ring[O.slot(o + j)] = ltype == 1 ? (uint8_t)litSrc : *(gcu8 *)(lsrc + lp + j);
        } else {
            O.flush(lane, true);
            if (ltype == 1) {
                for (uint32_t j = lane; j < last; j += 64) *(gu8 *)(dst + o + j) = (uint8_t)litSrc;
            } else {
                for (uint32_t j = lane; j < last; j += 64) *(gu8 *)(dst + o + j) = *(gcu8 *)(lsrc + lp + j);
            }
            wave_fence();
            O.F = O.V = o + last;
        }
        O.W = o + last;
    }
    O.flush(lane, true);
    const uint32_t o = O.W;
    e.stamp(4);
    if (F.hasFcs && (uint64_t)o != F.fcs) return kFbFcs;
    if (F.checksum && (uint32_t)xxh64(e, 0, o) != F.want) return kFbSum;
    e.stamp(5);
    return (int32_t)o;
}

}  // namespace jzd2

// jfsx_zstd.h -- Zstandard frame decoder (RFC 8878), the load side of the
// compressed block path for volumes formatted with --compress zstd.
//
// Replaces, per block, ZStandard.Decompress = zstd.Decompress(dst, src)
// (pkg/compress/compress.go:93-100, github.com/DataDog/zstd v1.5.0, go.mod:10,
// over the zstd C library's ZSTD_decompress), called by cachedStore.load after
// the object is read (pkg/chunk/cached_store.go:680-745).  Decoding is defined
// by the format, so any conforming decoder yields the same bytes; the accept /
// reject rules follow the zstd library's one-shot ZSTD_decompress (checked in
// tests against the system libzstd 1.4.8).
//
// One code path for host and device.  On the device every lane of the wave
// runs the same (uniform) decoder over tables in LDS: ZD_ONE(stmt) makes a
// table or output write happen once (lane 0) and the Env's copy helpers spread
// literal / match copies over the lanes.  Frames may be concatenated and may
// include skippable frames, as ZSTD_decompress allows.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <type_traits>

#if defined(__HIPCC__)
#define ZD_HD __host__ __device__ __attribute__((always_inline))
#else
#define ZD_HD
#endif
#if defined(__HIP_DEVICE_COMPILE__)
#define ZD_ONE(x)                    \
    do {                             \
        if (__lane_id() == 0) { x; } \
    } while (0)
#else
#define ZD_ONE(x) \
    do {          \
        x;        \
    } while (0)
#endif

// Values the whole wave agrees on (table entries read back from LDS, input
// words): on the device, taken from lane 0 so the decoder's control state
// stays in SGPRs and its input reads stay scalar.
#if defined(__HIP_DEVICE_COMPILE__)
#define ZD_U32(x) ((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x)))
#else
#define ZD_U32(x) ((uint32_t)(x))
#endif

namespace jzd {

ZD_HD inline uint64_t zd_u64(uint64_t v) {
    return (uint64_t)ZD_U32(v) | ((uint64_t)ZD_U32(v >> 32) << 32);
}

enum : int { ZD_OK = 0, ZD_EFORMAT = -1, ZD_EDSTSIZE = -2 };

constexpr uint32_t kBlockMax = 128 * 1024;  // ZSTD_BLOCKSIZE_MAX
constexpr uint32_t kHufLogMax = 12;          // HUF_TABLELOG_MAX
constexpr uint32_t kHufLogTab = 11;          // larger tables (log 12) live in Env::huf_g()
constexpr uint32_t kMaxLL = 35, kMaxML = 52, kMaxOff = 31;
constexpr uint32_t kLLLog = 9, kMLLog = 9, kOffLog = 8;

// sequence FSE decoding entry (ZSTD_seqSymbol), packed into 32 bits so the
// tables take 5 KiB of LDS: next state base [8:0], state bits [12:9], extra
// bits [17:13], value base as m << e in [23:18] and [27:24] (ML: + 3; OF:
// 1 << extra bits, not stored)
struct SeqEnt {
    uint32_t v;
};
struct SeqDec {
    uint32_t base, next, nbBits, addBits;
};

// Per-frame decoding state that persists across blocks; in LDS on the device.
struct Tables {
    uint16_t huf[1u << kHufLogTab];  // Huffman X1: symbol | nbBits << 8 (log <= 11)
    SeqEnt ll[1u << kLLLog], ml[1u << kMLLog], of[1u << kOffLog];
    union {
        uint32_t fw[64];                // Huffman-weight FSE table: sym | nb << 8 | next << 16
        uint32_t rank[kHufLogMax + 2];  // then: Huffman weight counts, then rank starts
    };
    uint8_t w[256];                  // Huffman weights
    int16_t norm[256];
    uint16_t snext[256];
};

// Frame-to-frame state (registers): which tables the repeat modes reuse.
struct Mode {
    uint32_t hufLog;        // 0: no Huffman table yet (set_repeat is an error)
    uint32_t llLog, mlLog, ofLog;
    bool seqEntropy;        // a block with sequences seen (set_repeat allowed)
    uint32_t rep[3];
};

ZD_HD inline uint32_t highbit(uint32_t v) {  // v > 0
    return 31u - (uint32_t)__builtin_clz(v);
}

// ---------------------------------------------------------------------------
// Bit readers over input bytes (Env::in8 / in64: zeros outside [0, insize))
// ---------------------------------------------------------------------------
// (readers keep a copy of the Env, a few pointers: no address of the Env is
// taken, so on the device it stays in registers)
template <class Env>
struct Fwd {  // forward, LSB-first (FSE_readNCount)
    Env e;
    int32_t base;
    uint32_t pos;
    ZD_HD uint32_t peek(uint32_t k) const {  // k <= 32; bits past the region read as zeros by the caller's bound
        const uint64_t v = e.in64(base + (int32_t)(pos >> 3));
        return (uint32_t)(v >> (pos & 7)) & (uint32_t)((1ull << k) - 1);
    }
};

// backward (BIT_DStream): bits taken from the top of [base, base + n); rem =
// valid bits not yet consumed (negative once over-read; missing low bits read
// as zeros, as libzstd's shifted container gives them)
template <class Env>
struct Bwd {
    Env e;
    int32_t base;
    int32_t rem;
    uint64_t cont;  // stream bytes [cb, cb + 8)
    int32_t cb;
    ZD_HD void fill() {
        const int32_t top = (rem - 1) >> 3;  // byte of the next bit
        if (top >= 7) {
            cb = top - 7;
            cont = e.in64u(base + cb);  // inside the stream region
        } else {
            cb = 0;
            cont = zd_u64(e.in64(base));
        }
    }
    ZD_HD uint32_t peek(uint32_t k) {  // k <= 32
        const int32_t lo = rem - (int32_t)k;
        if (rem > cb * 8 + 64 || (lo < cb * 8 && cb > 0)) fill();
        const int32_t sh = lo - cb * 8;
        if (sh >= 0) return (uint32_t)((cont >> sh) & ((1ull << k) - 1));
        // over-read below byte 0 (cb == 0): the missing low bits are zero
        if (rem <= 0) return 0;
        return (uint32_t)((cont << (uint32_t)(-sh)) & ((1ull << k) - 1));
    }
    ZD_HD uint32_t read(uint32_t k) {
        if (k == 0) return 0;
        const uint32_t v = peek(k);
        rem -= k;
        return v;
    }
    // true when bits [rem - t, rem) all lie in the window (after at most one
    // refill): the caller may then take t bits with take(), no further checks
    ZD_HD bool ensure(uint32_t t) {
        if (rem - (int32_t)t >= cb * 8) return true;
        if (cb == 0) return false;
        fill();
        return rem - (int32_t)t >= cb * 8;
    }
    ZD_HD uint32_t take(uint32_t k) {  // k <= 31, inside an ensure()d budget
        rem -= (int32_t)k;
        return (uint32_t)(cont >> ((uint32_t)(rem - cb * 8) & 63u)) & ((1u << k) - 1u);
    }
};

// BIT_initDStream: error if n == 0 or the last byte (end marker) is 0.  Bytes
// of the stream region only: the region must lie inside the input.
template <class Env>
ZD_HD bool bwd_init(Bwd<Env> &b, const Env &e, int32_t base, int32_t n) {
    if (n <= 0) return false;
    const uint32_t last = ZD_U32(e.in8(base + n - 1));
    if (last == 0) return false;
    b.e = e;
    b.base = base;
    b.rem = 8 * (n - 1) + (int32_t)highbit(last);
    b.cb = 1 << 30;
    b.cont = 0;
    b.fill();
    return true;
}

// ---------------------------------------------------------------------------
// FSE normalized counts (FSE_readNCount).  Region [base, base + n).  Returns
// the bytes used, or -1.  maxsv in: largest allowed symbol; out: last symbol.
// ---------------------------------------------------------------------------
template <class Env>
ZD_HD int32_t read_ncount(const Env &e, int32_t base, int32_t n, int16_t *norm, uint32_t &maxsv, uint32_t &tlog) {
    // headers shorter than 4 bytes are read zero-padded to 4 (libzstd copies
    // them into a 4-byte buffer); bits past the region read as zeros
    const int32_t nb4 = n < 4 ? 4 : n;
    struct Lim {
        Env e;
        int32_t base, n;
        ZD_HD uint64_t in64(int32_t i) const {
            uint64_t v = 0;
            for (int k = 0; k < 8; k++) {
                const int32_t j = i + k;
                if (j >= base && j < base + n) v |= (uint64_t)e.in8(j) << (8 * k);
            }
            return v;
        }
    };
    Fwd<Lim> r{Lim{e, base, n}, base, 0};
    for (uint32_t i = 0; i <= maxsv; i++) ZD_ONE(norm[i] = 0);
    uint32_t nbits = r.peek(4) + 5;
    r.pos += 4;
    if (nbits > 15) return -1;
    tlog = nbits;
    int32_t remaining = (1 << nbits) + 1, threshold = 1 << nbits;
    nbits++;
    uint32_t ch = 0;
    bool prev0 = false;
    while (remaining > 1 && ch <= maxsv) {
        if (prev0) {
            uint32_t n0 = ch, rr;
            do {
                rr = r.peek(2);
                r.pos += 2;
                n0 += rr;
            } while (rr == 3);
            if (n0 > maxsv) return -1;
            ch = n0;
        }
        const int32_t mx = (2 * threshold - 1) - remaining;
        int32_t count;
        const uint32_t low = r.peek(nbits - 1);
        if ((int32_t)low < mx) {
            count = (int32_t)low;
            r.pos += nbits - 1;
        } else {
            count = (int32_t)r.peek(nbits);
            if (count >= threshold) count -= mx;
            r.pos += nbits;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        ZD_ONE(norm[ch] = (int16_t)count);
        ch++;
        prev0 = count == 0;
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
        if (r.pos > 8ull * (uint32_t)nb4 + 64) return -1;  // libzstd's clamped read fails at the end
    }
    if (remaining != 1) return -1;
    if (r.pos > 8ull * (uint32_t)nb4) return -1;
    const int32_t used = (int32_t)((r.pos + 7) >> 3);
    if (used > n) return -1;
    maxsv = ch - 1;
    return used;
}

// FSE spread of the symbols (FSE_buildDTable / ZSTD_buildFSETable): out[u]
// = symbol of state u (the table being built, converted in place after),
// t.snext[s] = first "next state" of symbol s.  Returns false when the
// spread does not close on position 0.
ZD_HD inline bool fse_spread(Tables &t, uint32_t *out, uint32_t maxsv, uint32_t tlog) {
    const uint32_t size = 1u << tlog;
    uint32_t high = size - 1;
    for (uint32_t s = 0; s <= maxsv; s++) {
        const int32_t ns = (int16_t)ZD_U32((uint16_t)t.norm[s]);
        if (ns == -1) {
            ZD_ONE(out[high] = s);
            high--;
            ZD_ONE(t.snext[s] = 1);
        } else {
            ZD_ONE(t.snext[s] = (uint16_t)ns);
        }
    }
    const uint32_t mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= maxsv; s++)
        for (int32_t i = 0, ns = (int16_t)ZD_U32((uint16_t)t.norm[s]); i < ns; i++) {
            ZD_ONE(out[pos] = s);
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    return pos == 0;
}

// a table entry as wave-uniform values (kind: 0 LL, 1 ML, 2 OF)
template <uint32_t KIND>
ZD_HD inline SeqDec ld_seq(const SeqEnt *p) {
    const uint32_t w = ZD_U32(p->v);
    SeqDec d;
    d.next = w & 511u;
    d.nbBits = (w >> 9) & 15u;
    d.addBits = (w >> 13) & 31u;
    d.base = KIND == 2 ? 1u << d.addBits : (((w >> 18) & 63u) << ((w >> 24) & 15u)) + (KIND == 1 ? 3u : 0u);
    return d;
}

// sequence table from counts (ZSTD_buildFSETable) into dt[1 << tlog]
ZD_HD inline uint32_t code_bits(uint32_t kind, uint32_t s);
ZD_HD inline SeqEnt seq_pack(uint32_t kind, uint32_t s, uint32_t nb, uint32_t next);
ZD_HD inline void build_seq(Tables &t, SeqEnt *dt, uint32_t maxsv, uint32_t tlog, uint32_t kind) {
    fse_spread(t, &dt->v, maxsv, tlog);
    const uint32_t size = 1u << tlog;
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t s = ZD_U32(dt[u].v);
        const uint32_t nx = ZD_U32(t.snext[s]);
        ZD_ONE(t.snext[s] = (uint16_t)(nx + 1));
        const uint32_t nb = tlog - highbit(nx);
        ZD_ONE(dt[u] = seq_pack(kind, s, nb, (nx << nb) - size));
    }
}

// ---------------------------------------------------------------------------
// Sequence code tables (RFC 8878 3.1.1.3.2.1.1) and predefined distributions
// ---------------------------------------------------------------------------
constexpr uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,   10,  11,  12,   13,   14,   15,    16,    18,
                                   20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
constexpr uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,   16,   17,   18,   19,    20,
                                  21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,   34,   35,   37,   39,    41,
                                  43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
constexpr uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// predefined distributions (RFC 8878 3.1.1.3.2.2)
constexpr int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// code -> extra bits (offset codes: c bits over a base of 1 << c, the offset
// value before the repeat rules)
ZD_HD inline uint32_t code_bits(uint32_t kind, uint32_t s);

enum Kind : uint32_t { KLL = 0, KML = 1, KOF = 2 };

ZD_HD inline SeqEnt seq_pack(uint32_t kind, uint32_t s, uint32_t nb, uint32_t next) {
    // LL and ML - 3 bases are m << e with m < 64 exactly (kLLBase, kMLBase)
    uint32_t m = kind == KLL ? kLLBase[s] : kind == KML ? kMLBase[s] - 3 : 0, e = 0;
    while (m >= 64) {
        m >>= 1;
        e++;
    }
    SeqEnt d;
    d.v = next | nb << 9 | code_bits(kind, s) << 13 | m << 18 | e << 24;
    return d;
}

ZD_HD inline void kind_params(uint32_t kind, uint32_t &maxsv, uint32_t &maxlog) {
    maxsv = kind == KLL ? kMaxLL : kind == KML ? kMaxML : kMaxOff;
    maxlog = kind == KLL ? kLLLog : kind == KML ? kMLLog : kOffLog;
}

ZD_HD inline uint32_t code_bits(uint32_t kind, uint32_t s) {
    return kind == KLL ? kLLBits[s] : kind == KML ? kMLBits[s] : s;
}

// ZSTD_buildSeqTable for one of LL / ML / OF; returns bytes used or -1
template <class Env>
ZD_HD int32_t seq_table(const Env &e, Tables &t, Mode &m, uint32_t kind, uint32_t type, int32_t p, int32_t end) {
    uint32_t maxsv, maxlog;
    kind_params(kind, maxsv, maxlog);
    SeqEnt *dt = kind == KLL ? t.ll : kind == KML ? t.ml : t.of;
    uint32_t &logr = kind == KLL ? m.llLog : kind == KML ? m.mlLog : m.ofLog;
    if (type == 0) {  // predefined
        const uint32_t n = kind == KLL ? 36 : kind == KML ? 53 : 29;
        for (uint32_t s = 0; s < n; s++)
            ZD_ONE(t.norm[s] = kind == KLL ? kLLDef[s] : kind == KML ? kMLDef[s] : kOFDef[s]);
        const uint32_t lg = kind == KOF ? 5 : 6;
        build_seq(t, dt, n - 1, lg, kind);
        logr = lg;
        return 0;
    }
    if (type == 1) {  // RLE: one symbol
        if (p >= end) return -1;
        const uint32_t s = e.in8(p);
        if (s > maxsv) return -1;
        ZD_ONE(dt[0] = seq_pack(kind, s, 0, 0));
        logr = 0;
        return 1;
    }
    if (type == 3) {  // repeat
        if (!m.seqEntropy) return -1;
        return 0;
    }
    uint32_t mx = maxsv, tlog;
    const int32_t hs = read_ncount(e, p, end - p, t.norm, mx, tlog);
    if (hs < 0 || tlog > maxlog) return -1;
    build_seq(t, dt, mx, tlog, kind);
    logr = tlog;
    return hs;
}

// ---------------------------------------------------------------------------
// Huffman weights and table (HUF_readStats + HUF_readDTableX1)
// ---------------------------------------------------------------------------
template <class Env>
ZD_HD int32_t huf_table(const Env &e, Tables &t, int32_t p, int32_t n, uint32_t &hlog) {
    if (n <= 0) return -1;
    uint32_t hb = e.in8(p), nw;
    int32_t isize;
    if (hb >= 128) {  // direct 4-bit weights
        nw = hb - 127;
        isize = (nw + 1) / 2;
        if (isize + 1 > n) return -1;
        if (nw >= 256) return -1;
        for (uint32_t k = 0; k < nw; k++) {
            const uint32_t by = e.in8(p + 1 + k / 2);
            ZD_ONE(t.w[k] = (uint8_t)((k & 1) ? (by & 15) : (by >> 4)));
        }
    } else {  // FSE-compressed weights (accuracy <= 6), two interleaved states
        isize = hb;
        if (isize + 1 > n) return -1;
        const int32_t q = p + 1;
        uint32_t mx = 255, tlog;
        const int32_t hs = read_ncount(e, q, isize, t.norm, mx, tlog);
        if (hs < 0 || tlog > 6) return -1;
        if (!fse_spread(t, t.fw, mx, tlog)) return -1;
        const uint32_t size = 1u << tlog;
        for (uint32_t u = 0; u < size; u++) {
            const uint32_t s = ZD_U32(t.fw[u]);
            const uint32_t nx = ZD_U32(t.snext[s]);
            ZD_ONE(t.snext[s] = (uint16_t)(nx + 1));
            const uint32_t nb = tlog - highbit(nx);
            ZD_ONE(t.fw[u] = s | (nb << 8) | (((nx << nb) - size) << 16));
        }
        Bwd<Env> b;
        if (!bwd_init(b, e, q + hs, isize - hs)) return -1;
        uint32_t s1 = (uint32_t)b.read(tlog), s2 = (uint32_t)b.read(tlog);
        uint32_t o = 0;
        const uint32_t omax = 255;  // FSE_decompress_wksp(.., hwSize - 1 = 255, ..)
        for (;;) {
            if (o > omax - 2) return -1;
            uint32_t f = ZD_U32(t.fw[s1]);
            ZD_ONE(t.w[o] = (uint8_t)(f & 255));
            o++;
            s1 = (f >> 16) + (uint32_t)b.read((f >> 8) & 255);
            if (b.rem < 0) {
                ZD_ONE(t.w[o] = (uint8_t)(ZD_U32(t.fw[s2]) & 255));
                o++;
                break;
            }
            if (o > omax - 2) return -1;
            f = ZD_U32(t.fw[s2]);
            ZD_ONE(t.w[o] = (uint8_t)(f & 255));
            o++;
            s2 = (f >> 16) + (uint32_t)b.read((f >> 8) & 255);
            if (b.rem < 0) {
                ZD_ONE(t.w[o] = (uint8_t)(ZD_U32(t.fw[s1]) & 255));
                o++;
                break;
            }
        }
        nw = o;
    }
    // weight statistics, implied last weight
    uint32_t *rank = t.rank;
    for (uint32_t k = 0; k <= kHufLogMax + 1; k++) ZD_ONE(rank[k] = 0);
    uint32_t total = 0;
    for (uint32_t k = 0; k < nw; k++) {
        const uint32_t wk = ZD_U32(t.w[k]);
        if (wk >= kHufLogMax) return -1;
        const uint32_t rk = ZD_U32(rank[wk]);
        ZD_ONE(rank[wk] = rk + 1);
        total += (1u << wk) >> 1;
    }
    if (total == 0) return -1;
    const uint32_t tl = highbit(total) + 1;
    if (tl > kHufLogMax) return -1;
    const uint32_t rest = (1u << tl) - total;
    if ((1u << highbit(rest)) != rest) return -1;
    const uint32_t lastw = highbit(rest) + 1;
    ZD_ONE(t.w[nw] = (uint8_t)lastw);
    {
        const uint32_t rk = ZD_U32(rank[lastw]);
        ZD_ONE(rank[lastw] = rk + 1);
    }
    const uint32_t r1 = ZD_U32(rank[1]);
    if (r1 < 2 || (r1 & 1)) return -1;
    const uint32_t nsym = nw + 1;
    // X1 table: symbols in order, each weight's range starting at rankStart[w]
    // (rank[] turned into the starts in place)
    uint32_t next = 0;
    for (uint32_t wv = 1; wv <= tl; wv++) {
        const uint32_t cur = next;
        next += ZD_U32(rank[wv]) << (wv - 1);
        ZD_ONE(rank[wv] = cur);
    }
    for (uint32_t s = 0; s < nsym; s++) {
        const uint32_t wv = ZD_U32(t.w[s]);
        if (!wv) continue;
        const uint32_t len = (1u << wv) >> 1;
        const uint16_t ent = (uint16_t)(s | ((tl + 1 - wv) << 8));
        const uint32_t st = ZD_U32(rank[wv]);
        e.huf_fill((tl <= kHufLogTab ? t.huf : e.huf_g()) + st, ent, len);
        ZD_ONE(rank[wv] = st + len);
    }
    if (tl > kHufLogTab) e.huf_sync();
    hlog = tl;
    return isize + 1;
}

// Huffman symbols [k, cnt) of one stream into the literal buffer at o + k,
// bit by bit (the tail of a stream, and over-reads past its start)
template <class Env, class H>
ZD_HD void huf_tail(const Env &e, const H &h, Bwd<Env> &b, uint32_t hlog, uint32_t o, uint32_t k, uint32_t cnt) {
    for (; k < cnt; k++) {
        const uint32_t ent = h(b.peek(hlog));
        b.rem -= ent >> 8;
        e.lit_put(o + k, ent & 255);
    }
}

// one symbol from an ensure()d window: returns it, consumes its bits
template <class Env, class H>
ZD_HD uint32_t huf_sym(const H &h, Bwd<Env> &b, uint32_t hlog) {
    const uint32_t ent =
        h((uint32_t)(b.cont >> ((uint32_t)(b.rem - (int32_t)hlog - b.cb * 8) & 63u)) & ((1u << hlog) - 1u));
    b.rem -= ent >> 8;
    return ent & 255;
}

// four symbols of one stream, packed little-endian (window ensure()d for 4 * hlog bits)
template <class Env, class H>
ZD_HD uint32_t huf_sym4(const H &h, Bwd<Env> &b, uint32_t hlog) {
    uint32_t w = huf_sym(h, b, hlog);
    w |= huf_sym(h, b, hlog) << 8;
    w |= huf_sym(h, b, hlog) << 16;
    return w | huf_sym(h, b, hlog) << 24;
}

// one Huffman stream [p, p + n) into the literal buffer [o, o + cnt)
template <class Env, class H>
ZD_HD bool huf_stream(const Env &e, const H &h, uint32_t hlog, int32_t p, int32_t n, uint32_t o, uint32_t cnt) {
    Bwd<Env> b;
    if (!bwd_init(b, e, p, n)) return false;
    uint32_t k = 0;
    for (; k + 4 <= cnt && b.ensure(4 * hlog); k += 4) {
        const uint32_t w = huf_sym4(h, b, hlog);
        e.lit_put4(o + k, w, o + k, w, o + k, w, o + k, w);
    }
    huf_tail(e, h, b, hlog, o, k, cnt);
    return b.rem == 0;
}

// the four streams of a 4-stream literal section, decoded interleaved (four
// independent table-lookup chains) into [0, seg), [seg, 2 seg), ...
template <class Env, class H>
ZD_HD bool huf_streams4(const Env &e, const H &h, uint32_t hlog, int32_t s1, int32_t l1, int32_t s2, int32_t l2,
                        int32_t s3, int32_t l3, int32_t s4, int32_t l4, uint32_t seg, uint32_t c4) {
    Bwd<Env> b0, b1, b2, b3;
    if (!bwd_init(b0, e, s1, l1) || !bwd_init(b1, e, s2, l2) || !bwd_init(b2, e, s3, l3) || !bwd_init(b3, e, s4, l4))
        return false;
    const uint32_t need = 4 * hlog;
    uint32_t k = 0;  // c4 <= seg
    for (; k + 4 <= c4 && b0.ensure(need) && b1.ensure(need) && b2.ensure(need) && b3.ensure(need); k += 4) {
        uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
        for (uint32_t i = 0; i < 4; i++) {
            w0 |= huf_sym(h, b0, hlog) << (8 * i);
            w1 |= huf_sym(h, b1, hlog) << (8 * i);
            w2 |= huf_sym(h, b2, hlog) << (8 * i);
            w3 |= huf_sym(h, b3, hlog) << (8 * i);
        }
        e.lit_put4(k, w0, seg + k, w1, 2 * seg + k, w2, 3 * seg + k, w3);
    }
    huf_tail(e, h, b0, hlog, 0, k, seg);
    huf_tail(e, h, b1, hlog, seg, k, seg);
    huf_tail(e, h, b2, hlog, 2 * seg, k, seg);
    huf_tail(e, h, b3, hlog, 3 * seg, k, c4);
    return b0.rem == 0 && b1.rem == 0 && b2.rem == 0 && b3.rem == 0;
}

// ---------------------------------------------------------------------------
// One compressed block (ZSTD_decompressBlock_internal).  Output at op (frame
// relative, the frame starting at Env output position fo); returns bytes
// written or an error (< 0).
// ---------------------------------------------------------------------------
template <class Env>
ZD_HD int32_t block(Env &e, Tables &t, Mode &m, int32_t p, int32_t n, uint32_t fo, uint32_t op, uint32_t cap) {
    if (n >= (int32_t)kBlockMax) return ZD_EFORMAT;
    if (n < 3) return ZD_EFORMAT;  // MIN_CBLOCK_SIZE
    const int32_t end = p + n;
    // ---- literals section ----
    e.stamp(4);
    const uint32_t h0 = e.in8(p);
    const uint32_t ltype = h0 & 3, sf = (h0 >> 2) & 3;
    uint32_t litSize;
    int32_t lused;
    bool litInInput = false;  // raw literals read straight from the input
    int32_t litSrc = 0;
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
            if (lh + litSize > (uint32_t)n) return ZD_EFORMAT;
            litInInput = true;
            litSrc = p + lh;
            lused = lh + litSize;
        } else {
            if (sf == 3 && n < 4) return ZD_EFORMAT;
            if (litSize > kBlockMax) return ZD_EFORMAT;
            const uint32_t bv = e.in8(p + lh);
            e.lit_fill(0, bv, litSize);
            lused = lh + 1;
        }
    } else {
        if (ltype == 3 && m.hufLog == 0) return ZD_EFORMAT;
        if (n < 5) return ZD_EFORMAT;
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
        if (litSize > kBlockMax) return ZD_EFORMAT;
        if (litC + lh > (uint32_t)n) return ZD_EFORMAT;
        int32_t q = p + lh, qn = litC;
        if (ltype == 2) {
            uint32_t hl;
            const int32_t hs = huf_table(e, t, q, qn, hl);
            if (hs < 0) return ZD_EFORMAT;
            if (hs >= qn) return ZD_EFORMAT;
            m.hufLog = hl;
            q += hs;
            qn -= hs;
        }
        // the Huffman table: LDS (log <= 11) or Env::huf_g() (log 12)
        auto hufL = [&](uint32_t i) -> uint32_t { return ZD_U32(t.huf[i]); };
        auto hufG = [&](uint32_t i) -> uint32_t { return e.huf_ld(i); };
        if (single) {
            if (!(m.hufLog <= kHufLogTab ? huf_stream(e, hufL, m.hufLog, q, qn, 0, litSize)
                                         : huf_stream(e, hufG, m.hufLog, q, qn, 0, litSize)))
                return ZD_EFORMAT;
        } else {
            if (litSize == 0) return ZD_EFORMAT;
            if (qn < 10) return ZD_EFORMAT;
            const int32_t l1 = e.in8(q) | (e.in8(q + 1) << 8), l2 = e.in8(q + 2) | (e.in8(q + 3) << 8),
                          l3 = e.in8(q + 4) | (e.in8(q + 5) << 8);
            const int32_t l4 = qn - (l1 + l2 + l3 + 6);
            if (l4 < 0) return ZD_EFORMAT;
            const uint32_t seg = (litSize + 3) / 4;
            if (3 * seg > litSize) {
                // libzstd decodes stream 4 into a negative range (nothing) and
                // the first streams into its spare buffer room
                return ZD_EFORMAT;
            }
            const int32_t s1 = q + 6, s2 = s1 + l1, s3 = s2 + l2, s4 = s3 + l3;
            if (!(m.hufLog <= kHufLogTab
                      ? huf_streams4(e, hufL, m.hufLog, s1, l1, s2, l2, s3, l3, s4, l4, seg, litSize - 3 * seg)
                      : huf_streams4(e, hufG, m.hufLog, s1, l1, s2, l2, s3, l3, s4, l4, seg, litSize - 3 * seg)))
                return ZD_EFORMAT;
        }
        lused = lh + litC;
    }
    e.lit_sync();
    e.stamp(0);  // literals
    // ---- sequences section ----
    int32_t s = p + lused;
    if (s >= end) return ZD_EFORMAT;  // MIN_SEQUENCES_SIZE
    uint32_t nbSeq = e.in8(s++);
    if (nbSeq == 0) {
        if (s != end) return ZD_EFORMAT;
    } else {
        if (nbSeq > 0x7f) {
            if (nbSeq == 0xff) {
                if (s + 2 > end) return ZD_EFORMAT;
                nbSeq = (e.in8(s) | (e.in8(s + 1) << 8)) + 0x7f00;
                s += 2;
            } else {
                if (s >= end) return ZD_EFORMAT;
                nbSeq = ((nbSeq - 0x80) << 8) + e.in8(s);
                s++;
            }
        }
        if (s + 1 > end) return ZD_EFORMAT;
        const uint32_t modes = e.in8(s++);
        int32_t u;
        if ((u = seq_table(e, t, m, KLL, modes >> 6, s, end)) < 0) return ZD_EFORMAT;
        s += u;
        if ((u = seq_table(e, t, m, KOF, (modes >> 4) & 3, s, end)) < 0) return ZD_EFORMAT;
        s += u;
        if ((u = seq_table(e, t, m, KML, (modes >> 2) & 3, s, end)) < 0) return ZD_EFORMAT;
        s += u;
    }
    // ---- execute ----
    e.stamp(1);  // sequence headers and tables
    uint32_t o = op, lp = 0;  // output, literal read position
    if (nbSeq) {
        m.seqEntropy = true;
        Bwd<Env> b;
        if (!bwd_init(b, e, s, end - s)) return ZD_EFORMAT;
        uint32_t sl = (uint32_t)b.read(m.llLog), so = (uint32_t)b.read(m.ofLog), sm = (uint32_t)b.read(m.mlLog);
        for (uint32_t k = 0; k < nbSeq; k++) {
            if (b.rem < 0) return ZD_EFORMAT;  // BIT_reloadDStream overflow before a sequence
            const SeqDec dl = ld_seq<KLL>(t.ll + sl), dm = ld_seq<KML>(t.ml + sm), dof = ld_seq<KOF>(t.of + so);
            e.stamp(5);  // table reads
            const uint32_t ofc = dof.addBits;  // the offset takes ofc bits (1 for ofc == 1)
            const uint32_t ll0 = dl.base == 0 && dl.addBits == 0 ? 1u : 0u;
            uint32_t off, ml, ll;
            // one window check per sequence when its bits are all in the
            // window (the common case); otherwise bit-by-bit reads
            auto decode = [&](auto fastc) {
                auto rd = [&](uint32_t nb) -> uint32_t {
                    uint32_t v;
                    if constexpr (decltype(fastc)::value)
                        v = b.take(nb);
                    else
                        v = b.read(nb);
                    return v;
                };
                if (ofc > 1) {
                    off = dof.base + rd(ofc) - 3;
                    m.rep[2] = m.rep[1];
                    m.rep[1] = m.rep[0];
                    m.rep[0] = (uint32_t)off;
                } else if (ofc == 0) {
                    if (!ll0) {
                        off = m.rep[0];
                    } else {
                        off = m.rep[1];
                        m.rep[1] = m.rep[0];
                        m.rep[0] = (uint32_t)off;
                    }
                } else {
                    const uint32_t idx = 1 + ll0 + rd(1);
                    uint32_t tmp = idx == 3 ? m.rep[0] - 1 : idx == 2 ? m.rep[2] : m.rep[1];
                    tmp += !tmp;
                    if (idx != 1) m.rep[2] = m.rep[1];
                    m.rep[1] = m.rep[0];
                    m.rep[0] = (uint32_t)tmp;
                    off = tmp;
                }
                ml = dm.base + rd(dm.addBits);
                ll = dl.base + rd(dl.addBits);
                // state updates (libzstd 1.4 updates after the last sequence too)
                sl = dl.next + rd(dl.nbBits);
                sm = dm.next + rd(dm.nbBits);
                so = dof.next + rd(dof.nbBits);
            };
            if (b.ensure(ofc + dm.addBits + dl.addBits + dl.nbBits + dm.nbBits + dof.nbBits))
                decode(std::true_type{});
            else
                decode(std::false_type{});
            e.stamp(2);  // sequence decode
            // ZSTD_execSequence
            if (ll + ml > cap - o) return ZD_EDSTSIZE;
            const uint32_t litAvail = litSize - lp;
            if (ll > litAvail) return ZD_EFORMAT;
            if (litInInput)
                e.out_from_in(fo + o, litSrc + (int32_t)lp, ll);
            else
                e.out_from_lit(fo + o, lp, ll);
            o += ll;
            lp += ll;
            if (off > o) return ZD_EFORMAT;
            e.out_match(fo + o, off, ml);
            o += ml;
            e.stamp(3);  // sequence execution
        }
        if (b.rem > 0) return ZD_EFORMAT;  // not all bits consumed
    }
    // last literals
    const uint32_t last = litSize - lp;
    if (last > cap - o) return ZD_EDSTSIZE;
    if (litInInput)
        e.out_from_in(fo + o, litSrc + (int32_t)lp, last);
    else
        e.out_from_lit(fo + o, lp, last);
    o += last;
    return (int32_t)(o - op);
}

// ---------------------------------------------------------------------------
// XXH64 (content checksum) of output [fo, fo + len)
// ---------------------------------------------------------------------------
constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
ZD_HD inline uint64_t rotl64(uint64_t x, uint32_t r) { return (x << r) | (x >> (64 - r)); }
ZD_HD inline uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * P2;
    acc = rotl64(acc, 31);
    return acc * P1;
}
ZD_HD inline uint64_t xmerge(uint64_t acc, uint64_t v) {
    v = xround(0, v);
    acc ^= v;
    return acc * P1 + P4;
}
template <class Env>
ZD_HD uint64_t xxh64(const Env &e, uint32_t fo, uint32_t len) {
    uint64_t h;
    uint32_t i = 0;
    if (len >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
        for (; i + 32 <= len; i += 32) {
            v1 = xround(v1, e.out64(fo + i));
            v2 = xround(v2, e.out64(fo + i + 8));
            v3 = xround(v3, e.out64(fo + i + 16));
            v4 = xround(v4, e.out64(fo + i + 24));
        }
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = P5;
    }
    h += len;
    for (; i + 8 <= len; i += 8) {
        h ^= xround(0, e.out64(fo + i));
        h = rotl64(h, 27) * P1 + P4;
    }
    // the tail reads only bytes below fo + len (the output may end at the
    // end of its allocation)
    if (i + 4 <= len) {
        h ^= (uint64_t)e.out32(fo + i) * P1;
        h = rotl64(h, 23) * P2 + P3;
        i += 4;
    }
    for (; i < len; i++) {
        h ^= (uint64_t)e.out8(fo + i) * P5;
        h = rotl64(h, 11) * P1;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

// ---------------------------------------------------------------------------
// ZSTD_decompress: all frames of the input into the output (capacity cap).
// Returns the decoded size, or ZD_EFORMAT / ZD_EDSTSIZE.
// ---------------------------------------------------------------------------
template <class Env>
ZD_HD int32_t decompress(Env &e, Tables &t, uint32_t insize, uint32_t cap) {
    int32_t p = 0;
    const int32_t n = (int32_t)insize;
    uint32_t out = 0;
    while (n - p >= 5) {
        const uint32_t magic = e.in8(p) | (e.in8(p + 1) << 8) | (e.in8(p + 2) << 16) | ((uint32_t)e.in8(p + 3) << 24);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
            if (n - p < 8) return ZD_EFORMAT;
            const uint64_t sz = e.in8(p + 4) | (e.in8(p + 5) << 8) | (e.in8(p + 6) << 16) | ((uint64_t)e.in8(p + 7) << 24);
            if (sz + 8 > (uint64_t)(n - p)) return ZD_EFORMAT;
            p += 8 + (int32_t)sz;
            continue;
        }
        if (magic != 0xFD2FB528u) return ZD_EFORMAT;
        if (n - p < 9) return ZD_EFORMAT;  // ZSTD_FRAMEHEADERSIZE_MIN + block header
        const uint32_t fhd = e.in8(p + 4);
        const uint32_t dictCode = fhd & 3, checksum = (fhd >> 2) & 1, single = (fhd >> 5) & 1, fcsId = fhd >> 6;
        const int32_t hsize = 5 + (single ? 0 : 1) + (dictCode == 3 ? 4 : dictCode) +
                              (fcsId == 0 ? (single ? 1 : 0) : fcsId == 1 ? 2 : fcsId == 2 ? 4 : 8);
        if (n - p < hsize + 3) return ZD_EFORMAT;
        if (fhd & 0x08) return ZD_EFORMAT;
        int32_t q = p + 5;
        if (!single) {
            const uint32_t wl = e.in8(q++);
            if ((wl >> 3) + 10 > 31) return ZD_EFORMAT;
        }
        uint32_t dict = 0;
        for (uint32_t k = 0, dn = dictCode == 3 ? 4 : dictCode; k < dn; k++) dict |= e.in8(q++) << (8 * k);
        if (dict) return ZD_EFORMAT;  // no dictionary loaded
        bool hasFcs = true;
        uint64_t fcs = 0;
        if (fcsId == 0) {
            if (single) fcs = e.in8(q++);
            else hasFcs = false;
        } else {
            const uint32_t fb = fcsId == 1 ? 2 : fcsId == 2 ? 4 : 8;
            for (uint32_t k = 0; k < fb; k++) fcs |= (uint64_t)e.in8(q++) << (8 * k);
            if (fcsId == 1) fcs += 256;
        }
        // frame
        Mode m;
        m.hufLog = 0;
        m.llLog = m.mlLog = m.ofLog = 0;
        m.seqEntropy = false;
        m.rep[0] = 1;
        m.rep[1] = 4;
        m.rep[2] = 8;
        const uint32_t fo = out;
        uint32_t op = 0;
        for (;;) {
            if (n - q < 3) return ZD_EFORMAT;
            const uint32_t bh = e.in8(q) | (e.in8(q + 1) << 8) | (e.in8(q + 2) << 16);
            q += 3;
            const uint32_t lastb = bh & 1, btype = (bh >> 1) & 3, bsize = bh >> 3;
            const int32_t csize = btype == 1 ? 1 : (int32_t)bsize;
            if (btype == 3) return ZD_EFORMAT;
            if (csize > n - q) return ZD_EFORMAT;
            int32_t got;
            if (btype == 0) {
                if (bsize > cap - out - op) return ZD_EDSTSIZE;
                e.out_from_in(fo + op, q, bsize);
                got = bsize;
            } else if (btype == 1) {
                if (bsize > cap - out - op) return ZD_EDSTSIZE;
                e.out_fill(fo + op, e.in8(q), bsize);
                got = bsize;
            } else {
                got = block(e, t, m, q, csize, fo, op, cap - out);
                if (got < 0) return got;
            }
            e.out_sync();
            op += (uint32_t)got;
            q += csize;
            if (lastb) break;
        }
        if (hasFcs && (uint64_t)op != fcs) return ZD_EFORMAT;
        if (checksum) {
            if (n - q < 4) return ZD_EFORMAT;
            const uint32_t want = e.in8(q) | (e.in8(q + 1) << 8) | (e.in8(q + 2) << 16) | ((uint32_t)e.in8(q + 3) << 24);
            if ((uint32_t)xxh64(e, fo, op) != want) return ZD_EFORMAT;
            q += 4;
        }
        out += op;
        p = q;
    }
    if (p != n) return ZD_EFORMAT;
    return (int32_t)out;
}

}  // namespace jzd

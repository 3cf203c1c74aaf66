// jfsx_zstdc.h -- Zstandard level-1 frame encoder, the upload side of the
// compressed block path for volumes formatted with --compress zstd.
//
// Replaces, per block, ZStandard.Compress = zstd.CompressLevel(dst, src, 1)
// (pkg/compress/compress.go:82-91, github.com/DataDog/zstd v1.5.0, go.mod:10,
// over the zstd C library's ZSTD_compress), called by cachedStore.upload before
// the object is put (pkg/chunk/cached_store.go:371-392, Compress at :387).
//
// Unlike decoding, compression is not defined by the format: the bytes are
// those of one library's parser and entropy heuristics.  This restates the
// zstd library's level-1 one-shot path as the system libzstd 1.4.8 writes it
// (tests compare whole frames byte for byte with ZSTD_compress(level 1); the
// 1.5.0 the reference vendors is not in the tree, so parity with it is
// unpinned -- DESIGN.md):
//   parameters   ZSTD_defaultCParameters[tableID][1] + ZSTD_adjustCParams_internal
//   frame        ZSTD_writeFrameHeader, ZSTD_compress_frameChunk (128 KiB blocks,
//                raw / RLE / compressed block choice, first-block rule)
//   parser       ZSTD_compressBlock_fast_generic (greedy, two positions per
//                step, repcode check at ip+2, hash of minMatch 4..7 bytes)
//   literals     ZSTD_compressLiterals + HUF_compress_internal (4 streams or
//                one, table reuse, weight header by FSE or 4-bit)
//   sequences    ZSTD_entropyCompressSequences_internal (ZSTD_selectEncodingType
//                for ZSTD_fast, FSE_normalizeCount, FSE_writeNCount,
//                FSE_buildCTable, ZSTD_encodeSequences)
//
// One source for host and device.  The host harness (tests/harness/
// zstdc_host.cpp) runs the scalar code below; the GPU kernel (jfsx_zstdc.hip)
// runs the same entropy stages and replaces the parser loop and the per-byte
// passes with wave-parallel versions that must produce the same sequences.
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define ZC_HD __host__ __device__ inline
#else
#define ZC_HD inline
#endif

namespace jzc {

constexpr uint32_t kBlockMax = 128 * 1024;   // ZSTD_BLOCKSIZE_MAX
constexpr uint32_t kMaxSeq = kBlockMax / 4;  // maxNbSeq: blockSize / 4 for minMatch >= 4
constexpr uint32_t kHashLogMax = 15;         // level 1, inputs <= 16 KiB
constexpr uint32_t kMaxLL = 35, kMaxML = 52, kMaxOff = 31, kDefaultMaxOff = 28;
constexpr uint32_t kLLLog = 9, kMLLog = 9, kOffLog = 8;
constexpr uint32_t kHufLogDefault = 11, kHufLogMax = 12;
constexpr uint32_t kLongNbSeq = 0x7F00;
constexpr uint32_t kRleMaxLength = 25;  // ZSTD_compressBlock_internal rleMaxLength

enum SetType : uint32_t { kSetBasic = 0, kSetRle = 1, kSetCompressed = 2, kSetRepeat = 3 };

// ---------------------------------------------------------------------------
// parameters (zstd_compress.c: ZSTD_defaultCParameters level-1 rows and
// ZSTD_adjustCParams_internal for a known source size, no dictionary)
// ---------------------------------------------------------------------------
struct Params {
    uint32_t wlog, hlog, mls;
};

ZC_HD uint32_t highbit32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

ZC_HD Params level1_params(uint64_t n) {
    Params p;
    if (n <= 16384) p = {14, 15, 5};
    else if (n <= 131072) p = {17, 13, 6};
    else if (n <= 262144) p = {18, 14, 6};
    else p = {19, 14, 7};
    if (n < ((uint64_t)1 << 30)) {
        const uint32_t srcLog = n < 64 ? 6u : highbit32((uint32_t)(n - 1)) + 1;
        if (p.wlog > srcLog) p.wlog = srcLog;
    }
    if (p.hlog > p.wlog + 1) p.hlog = p.wlog + 1;
    if (p.wlog < 10) p.wlog = 10;  // ZSTD_WINDOWLOG_ABSOLUTEMIN
    return p;
}

// ZSTD_compressBound
ZC_HD uint64_t compress_bound(uint64_t n) {
    return n + (n >> 8) + (n < kBlockMax ? (kBlockMax - n) >> 11 : 0);
}

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
ZC_HD uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
ZC_HD uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
ZC_HD void wr16(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}
ZC_HD void wr24(uint8_t *p, uint32_t v) {
    wr16(p, v);
    p[2] = (uint8_t)(v >> 16);
}
ZC_HD void wr32(uint8_t *p, uint32_t v) {
    wr16(p, v);
    wr16(p + 2, v >> 16);
}
ZC_HD void copy_bytes(uint8_t *d, const uint8_t *s, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) d[i] = s[i];
}

// ZSTD_hashPtr for minMatch 4..7 (zstd_compress_internal.h)
ZC_HD uint32_t hash_ptr(const uint8_t *p, uint32_t hlog, uint32_t mls) {
    if (mls == 5) return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> (64 - hlog));
    if (mls == 6) return (uint32_t)(((rd64(p) << 16) * 227718039650203ull) >> (64 - hlog));
    if (mls == 7) return (uint32_t)(((rd64(p) << 8) * 58295818150454627ull) >> (64 - hlog));
    return (rd32(p) * 2654435761u) >> (32 - hlog);
}

// ZSTD_count: equal bytes at a and b, a not past lim
ZC_HD uint32_t count_eq(const uint8_t *a, const uint8_t *b, const uint8_t *lim) {
    const uint8_t *s = a;
    while (a + 8 <= lim) {
        const uint64_t d = rd64(a) ^ rd64(b);
        if (d) return (uint32_t)(a - s) + ((uint32_t)__builtin_ctzll(d) >> 3);
        a += 8;
        b += 8;
    }
    while (a < lim && *a == *b) a++, b++;
    return (uint32_t)(a - s);
}

// ---------------------------------------------------------------------------
// sequence store (zstd_compress_internal.h seqStore_t, ZSTD_storeSeq)
// ---------------------------------------------------------------------------
struct SeqDef {
    uint32_t offset;  // offCode + 1: 1..3 repcodes, else distance + 3
    uint16_t ll;      // literal length (low 16 bits; see long_id)
    uint16_t ml;      // match length - MINMATCH(3) (low 16 bits)
};

struct SeqStore {
    SeqDef *seq;
    uint8_t *lit;
    uint8_t *llc, *mlc, *ofc;  // codes (ZSTD_seqToCodes)
    uint32_t nseq, nlit;
    uint32_t long_id, long_pos;  // 1: literal length > 0xFFFF, 2: match length
};

ZC_HD void store_seq(SeqStore &ss, const uint8_t *lits, uint32_t litLen, uint32_t offCode, uint32_t mlBase) {
    copy_bytes(ss.lit + ss.nlit, lits, litLen);
    ss.nlit += litLen;
    if (litLen > 0xFFFF) ss.long_id = 1, ss.long_pos = ss.nseq;
    if (mlBase > 0xFFFF) ss.long_id = 2, ss.long_pos = ss.nseq;
    SeqDef d;
    d.offset = offCode + 1;
    d.ll = (uint16_t)litLen;
    d.ml = (uint16_t)mlBase;
    ss.seq[ss.nseq++] = d;
}

// ---------------------------------------------------------------------------
// ZSTD_compressBlock_fast_generic over positions [istart, iend) of the object
// src (index of position p = p + 1: the window's base is src - 1, dictLimit
// 1).  rep[0..1] in/out.  Returns the trailing literal count.
// ---------------------------------------------------------------------------
ZC_HD int32_t prefix_start_index(int32_t endIndex, uint32_t wlog) {
    const uint32_t maxDist = 1u << wlog;
    return ((uint32_t)(endIndex - 1) > maxDist) ? endIndex - (int32_t)maxDist : 1;
}

ZC_HD uint32_t parse_fast(const uint8_t *src, int32_t istart, int32_t iend, uint32_t *htab, Params P, uint32_t rep[2],
                          SeqStore &ss) {
    const uint32_t hlog = P.hlog, mls = P.mls;
    const int32_t stepSize = 2;  // targetLength 0: 0 + !0 + 1
    const int32_t endIndex = iend + 1;
    const int32_t prefixStartIndex = prefix_start_index(endIndex, P.wlog);
    const int32_t prefixStart = prefixStartIndex - 1;  // as a position
    const int32_t ilimit = iend - 8;                   // HASH_READ_SIZE
    int32_t ip0 = istart, anchor = istart;
    uint32_t offset_1 = rep[0], offset_2 = rep[1], offsetSaved = 0;
    ip0 += (ip0 == prefixStart);
    int32_t ip1 = ip0 + 1;
    {
        const int32_t cur = ip0 + 1;
        const int32_t windowLow = prefix_start_index(cur, P.wlog);
        const uint32_t maxRep = (uint32_t)(cur - windowLow);
        if (offset_2 > maxRep) offsetSaved = offset_2, offset_2 = 0;
        if (offset_1 > maxRep) offsetSaved = offset_1, offset_1 = 0;
    }
    const uint8_t *const iendp = src + iend;
    while (ip1 < ilimit) {
        const int32_t ip2 = ip0 + 2;
        const uint32_t h0 = hash_ptr(src + ip0, hlog, mls), h1 = hash_ptr(src + ip1, hlog, mls);
        const uint32_t val0 = rd32(src + ip0), val1 = rd32(src + ip1);
        const int32_t current0 = ip0 + 1, current1 = ip1 + 1;
        const int32_t matchIndex0 = (int32_t)htab[h0], matchIndex1 = (int32_t)htab[h1];
        const int32_t repMatch = ip2 - (int32_t)offset_1;
        int32_t match0 = matchIndex0 - 1;
        uint32_t mLength, offcode;
        htab[h0] = (uint32_t)current0;
        htab[h1] = (uint32_t)current1;
        if ((offset_1 > 0) && rd32(src + repMatch) == rd32(src + ip2)) {
            mLength = (src[ip2 - 1] == src[repMatch - 1]) ? 1 : 0;
            ip0 = ip2 - (int32_t)mLength;
            match0 = repMatch - (int32_t)mLength;
            mLength += 4;
            offcode = 0;
        } else {
            if (matchIndex0 > prefixStartIndex && rd32(src + match0) == val0) {
                // found a regular match
            } else if (matchIndex1 > prefixStartIndex && rd32(src + matchIndex1 - 1) == val1) {
                ip0 = ip1;
                match0 = matchIndex1 - 1;
            } else {
                const int32_t step = ((ip0 - anchor) >> 7) + stepSize;  // kSearchStrength 8
                ip0 += step;
                ip1 += step;
                continue;
            }
            offset_2 = offset_1;
            offset_1 = (uint32_t)(ip0 - match0);
            offcode = offset_1 + 2;  // ZSTD_REP_MOVE
            mLength = 4;
            while (ip0 > anchor && match0 > prefixStart && src[ip0 - 1] == src[match0 - 1]) {
                ip0--;
                match0--;
                mLength++;
            }
        }
        mLength += count_eq(src + ip0 + mLength, src + match0 + mLength, iendp);
        store_seq(ss, src + anchor, (uint32_t)(ip0 - anchor), offcode, mLength - 3);
        ip0 += (int32_t)mLength;
        anchor = ip0;
        if (ip0 <= ilimit) {
            htab[hash_ptr(src + current0 + 1, hlog, mls)] = (uint32_t)(current0 + 2);
            htab[hash_ptr(src + ip0 - 2, hlog, mls)] = (uint32_t)(ip0 - 1);
            while (ip0 <= ilimit && offset_2 > 0 && rd32(src + ip0) == rd32(src + ip0 - (int32_t)offset_2)) {
                const uint32_t rLength = count_eq(src + ip0 + 4, src + ip0 + 4 - offset_2, iendp) + 4;
                const uint32_t t = offset_2;
                offset_2 = offset_1;
                offset_1 = t;
                htab[hash_ptr(src + ip0, hlog, mls)] = (uint32_t)(ip0 + 1);
                ip0 += (int32_t)rLength;
                store_seq(ss, src + anchor, 0, 0, rLength - 3);
                anchor = ip0;
            }
        }
        ip1 = ip0 + 1;
    }
    rep[0] = offset_1 ? offset_1 : offsetSaved;
    rep[1] = offset_2 ? offset_2 : offsetSaved;
    return (uint32_t)(iend - anchor);
}

// ---------------------------------------------------------------------------
// bit stream writer (bitstream.h BIT_CStream_t): little-endian, low bits first
// ---------------------------------------------------------------------------
struct BitC {
    uint64_t c;
    uint32_t pos;
    uint8_t *start, *ptr, *end;
};
ZC_HD bool bit_init(BitC &b, uint8_t *dst, uint64_t cap) {
    b.c = 0;
    b.pos = 0;
    b.start = b.ptr = dst;
    if (cap <= 8) return false;
    b.end = dst + cap - 8;
    return true;
}
ZC_HD void bit_add(BitC &b, uint64_t v, uint32_t nb) {
    if (!nb) return;
    b.c |= (v & ((nb >= 64) ? ~0ull : ((1ull << nb) - 1))) << b.pos;
    b.pos += nb;
}
ZC_HD void bit_flush(BitC &b) {
    const uint32_t nbytes = b.pos >> 3;
    for (uint32_t i = 0; i < nbytes; i++) b.ptr[i] = (uint8_t)(b.c >> (8 * i));
    b.ptr += nbytes;
    if (b.ptr > b.end) b.ptr = b.end;
    b.pos &= 7;
    b.c = nbytes == 8 ? 0 : b.c >> (8 * nbytes);
}
// add with a flush when the container could overflow (the library's flush
// points differ, the resulting stream does not)
ZC_HD void bit_put(BitC &b, uint64_t v, uint32_t nb) {
    if (b.pos + nb > 56) bit_flush(b);
    bit_add(b, v, nb);
}
ZC_HD uint64_t bit_close(BitC &b) {
    bit_put(b, 1, 1);
    bit_flush(b);
    if (b.pos) b.ptr[0] = (uint8_t)b.c;
    if (b.ptr >= b.end) return 0;
    return (uint64_t)(b.ptr - b.start) + (b.pos > 0);
}

// ---------------------------------------------------------------------------
// FSE (fse_compress.c, entropy_common.c)
// ---------------------------------------------------------------------------
struct FseCT {
    uint32_t tableLog;
    uint16_t state[1u << 9];
    int32_t dfs[64];   // deltaFindState
    uint32_t dnb[64];  // deltaNbBits
};

ZC_HD uint32_t fse_min_table_log(uint64_t n, uint32_t maxSym) {
    const uint32_t a = highbit32((uint32_t)n) + 1, b = highbit32(maxSym) + 2;
    return a < b ? a : b;
}

// FSE_optimalTableLog_internal
ZC_HD uint32_t fse_optimal_table_log(uint32_t maxLog, uint64_t n, uint32_t maxSym, uint32_t minus) {
    const uint32_t maxBitsSrc = highbit32((uint32_t)(n - 1)) - minus;
    uint32_t t = maxLog;
    const uint32_t minBits = fse_min_table_log(n, maxSym);
    if (maxBitsSrc < t) t = maxBitsSrc;
    if (minBits > t) t = minBits;
    if (t < 5) t = 5;
    if (t > 12) t = 12;
    return t;
}

// FSE_normalizeM2
ZC_HD int fse_normalize_m2(int16_t *norm, uint32_t tableLog, const uint32_t *count, uint64_t total, uint32_t maxSym,
                           int16_t lowProb) {
    const int16_t NOT_YET = -2;
    uint32_t distributed = 0;
    const uint32_t lowThreshold = (uint32_t)(total >> tableLog);
    uint32_t lowOne = (uint32_t)((total * 3) >> (tableLog + 1));
    for (uint32_t s = 0; s <= maxSym; s++) {
        if (count[s] == 0) {
            norm[s] = 0;
            continue;
        }
        if (count[s] <= lowThreshold) {
            norm[s] = lowProb;
            distributed++;
            total -= count[s];
            continue;
        }
        if (count[s] <= lowOne) {
            norm[s] = 1;
            distributed++;
            total -= count[s];
            continue;
        }
        norm[s] = NOT_YET;
    }
    uint32_t toDistribute = (1u << tableLog) - distributed;
    if (toDistribute == 0) return 0;
    if ((total / toDistribute) > lowOne) {
        lowOne = (uint32_t)((total * 3) / (toDistribute * 2));
        for (uint32_t s = 0; s <= maxSym; s++) {
            if (norm[s] == NOT_YET && count[s] <= lowOne) {
                norm[s] = 1;
                distributed++;
                total -= count[s];
            }
        }
        toDistribute = (1u << tableLog) - distributed;
    }
    if (distributed == maxSym + 1) {
        uint32_t maxV = 0, maxC = 0;
        for (uint32_t s = 0; s <= maxSym; s++)
            if (count[s] > maxC) maxV = s, maxC = count[s];
        norm[maxV] += (int16_t)toDistribute;
        return 0;
    }
    if (total == 0) {
        for (uint32_t s = 0; toDistribute > 0; s = (s + 1) % (maxSym + 1))
            if (norm[s] > 0) toDistribute--, norm[s]++;
        return 0;
    }
    {
        const uint64_t vStepLog = 62 - tableLog;
        const uint64_t mid = (1ull << (vStepLog - 1)) - 1;
        const uint64_t rStep = (((1ull << vStepLog) * toDistribute) + mid) / total;
        uint64_t tmpTotal = mid;
        for (uint32_t s = 0; s <= maxSym; s++) {
            if (norm[s] == NOT_YET) {
                const uint64_t end = tmpTotal + (count[s] * rStep);
                const uint32_t sStart = (uint32_t)(tmpTotal >> vStepLog), sEnd = (uint32_t)(end >> vStepLog);
                const uint32_t weight = sEnd - sStart;
                if (weight < 1) return -1;
                norm[s] = (int16_t)weight;
                tmpTotal = end;
            }
        }
    }
    return 0;
}

// FSE_normalizeCount (1.4.8: useLowProbCount selects -1 or 1 for rare symbols)
ZC_HD int fse_normalize(int16_t *norm, uint32_t tableLog, const uint32_t *count, uint64_t total, uint32_t maxSym,
                        bool useLowProb) {
    const uint32_t rtb[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
    const int16_t lowProb = useLowProb ? -1 : 1;
    const uint64_t scale = 62 - tableLog;
    const uint64_t step = (1ull << 62) / (uint32_t)total;
    const uint64_t vStep = 1ull << (scale - 20);
    int stillToDistribute = 1 << tableLog;
    uint32_t largest = 0;
    int16_t largestP = 0;
    const uint32_t lowThreshold = (uint32_t)(total >> tableLog);
    for (uint32_t s = 0; s <= maxSym; s++) {
        if (count[s] == total) return 0;  // rle: handled by the caller
        if (count[s] == 0) {
            norm[s] = 0;
            continue;
        }
        if (count[s] <= lowThreshold) {
            norm[s] = lowProb;
            stillToDistribute--;
        } else {
            int16_t proba = (int16_t)((count[s] * step) >> scale);
            if (proba < 8) {
                const uint64_t restToBeat = vStep * rtb[proba];
                proba += (count[s] * step) - ((uint64_t)proba << scale) > restToBeat;
            }
            if (proba > largestP) largestP = proba, largest = s;
            norm[s] = proba;
            stillToDistribute -= proba;
        }
    }
    if (-stillToDistribute >= (norm[largest] >> 1)) return fse_normalize_m2(norm, tableLog, count, total, maxSym, lowProb);
    norm[largest] += (int16_t)stillToDistribute;
    return 0;
}

// FSE_writeNCount_generic (buffer known to be large enough)
ZC_HD uint32_t fse_write_ncount(uint8_t *out, const int16_t *norm, uint32_t maxSym, uint32_t tableLog) {
    uint8_t *o = out;
    const int tableSize = 1 << tableLog;
    uint32_t bitStream = 0;
    int bitCount = 0;
    uint32_t symbol = 0;
    const uint32_t alphabetSize = maxSym + 1;
    bool previousIs0 = false;
    bitStream += (tableLog - 5) << bitCount;
    bitCount += 4;
    int remaining = tableSize + 1, threshold = tableSize, nbBits = (int)tableLog + 1;
    while (symbol < alphabetSize && remaining > 1) {
        if (previousIs0) {
            uint32_t start = symbol;
            while (symbol < alphabetSize && !norm[symbol]) symbol++;
            if (symbol == alphabetSize) break;
            while (symbol >= start + 24) {
                start += 24;
                bitStream += 0xFFFFu << bitCount;
                o[0] = (uint8_t)bitStream;
                o[1] = (uint8_t)(bitStream >> 8);
                o += 2;
                bitStream >>= 16;
            }
            while (symbol >= start + 3) {
                start += 3;
                bitStream += 3u << bitCount;
                bitCount += 2;
            }
            bitStream += (symbol - start) << bitCount;
            bitCount += 2;
            if (bitCount > 16) {
                o[0] = (uint8_t)bitStream;
                o[1] = (uint8_t)(bitStream >> 8);
                o += 2;
                bitStream >>= 16;
                bitCount -= 16;
            }
        }
        {
            int count = norm[symbol++];
            const int max = (2 * threshold - 1) - remaining;
            remaining -= count < 0 ? -count : count;
            count++;
            if (count >= threshold) count += max;
            bitStream += (uint32_t)count << bitCount;
            bitCount += nbBits;
            bitCount -= (count < max);
            previousIs0 = (count == 1);
            while (remaining < threshold) nbBits--, threshold >>= 1;
        }
        if (bitCount > 16) {
            o[0] = (uint8_t)bitStream;
            o[1] = (uint8_t)(bitStream >> 8);
            o += 2;
            bitStream >>= 16;
            bitCount -= 16;
        }
    }
    o[0] = (uint8_t)bitStream;
    o[1] = (uint8_t)(bitStream >> 8);
    o += (bitCount + 7) / 8;
    return (uint32_t)(o - out);
}

// FSE_buildCTable_wksp
ZC_HD void fse_build_ctable(FseCT &ct, const int16_t *norm, uint32_t maxSym, uint32_t tableLog, uint8_t *tableSymbol) {
    const uint32_t tableSize = 1u << tableLog, tableMask = tableSize - 1;
    const uint32_t step = (tableSize >> 1) + (tableSize >> 3) + 3;
    uint32_t cumul[64];
    uint32_t highThreshold = tableSize - 1;
    ct.tableLog = tableLog;
    cumul[0] = 0;
    for (uint32_t u = 1; u <= maxSym + 1; u++) {
        if (norm[u - 1] == -1) {
            cumul[u] = cumul[u - 1] + 1;
            tableSymbol[highThreshold--] = (uint8_t)(u - 1);
        } else {
            cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
        }
    }
    cumul[maxSym + 1] = tableSize + 1;
    {
        uint32_t position = 0;
        for (uint32_t s = 0; s <= maxSym; s++) {
            for (int k = 0; k < norm[s]; k++) {
                tableSymbol[position] = (uint8_t)s;
                position = (position + step) & tableMask;
                while (position > highThreshold) position = (position + step) & tableMask;
            }
        }
    }
    for (uint32_t u = 0; u < tableSize; u++) {
        const uint8_t s = tableSymbol[u];
        ct.state[cumul[s]++] = (uint16_t)(tableSize + u);
    }
    uint32_t total = 0;
    for (uint32_t s = 0; s <= maxSym; s++) {
        const int n = norm[s];
        if (n == 0) {
            ct.dnb[s] = ((tableLog + 1) << 16) - (1u << tableLog);
            ct.dfs[s] = 0;
        } else if (n == -1 || n == 1) {
            ct.dnb[s] = (tableLog << 16) - (1u << tableLog);
            ct.dfs[s] = (int32_t)total - 1;
            total++;
        } else {
            const uint32_t maxBitsOut = tableLog - highbit32((uint32_t)n - 1);
            const uint32_t minStatePlus = (uint32_t)n << maxBitsOut;
            ct.dnb[s] = (maxBitsOut << 16) - minStatePlus;
            ct.dfs[s] = (int32_t)total - n;
            total += (uint32_t)n;
        }
    }
}

// FSE_buildCTable_rle
ZC_HD void fse_build_ctable_rle(FseCT &ct, uint32_t sym) {
    ct.tableLog = 0;
    ct.state[0] = 0;
    ct.state[1] = 0;
    ct.dnb[sym] = 0;
    ct.dfs[sym] = 0;
}

struct FseState {
    uint32_t value;
};
ZC_HD void fse_init_state2(FseState &st, const FseCT &ct, uint32_t sym) {
    const uint32_t nbBitsOut = (ct.dnb[sym] + (1u << 15)) >> 16;
    uint32_t v = (nbBitsOut << 16) - ct.dnb[sym];
    st.value = ct.state[(int32_t)(v >> nbBitsOut) + ct.dfs[sym]];
}
ZC_HD void fse_encode(BitC &b, FseState &st, const FseCT &ct, uint32_t sym) {
    const uint32_t nbBitsOut = (st.value + ct.dnb[sym]) >> 16;
    bit_put(b, st.value, nbBitsOut);
    st.value = ct.state[(int32_t)(st.value >> nbBitsOut) + ct.dfs[sym]];
}
ZC_HD void fse_flush_state(BitC &b, const FseState &st, const FseCT &ct) { bit_put(b, st.value, ct.tableLog); }

// ---------------------------------------------------------------------------
// Huffman (huf_compress.c)
// ---------------------------------------------------------------------------
struct HufCT {
    uint16_t val[256];
    uint8_t nb[256];
};
enum HufRepeat : uint32_t { kHufNone = 0, kHufCheck = 1, kHufValid = 2 };

struct HufNode {
    uint32_t count;
    uint16_t parent;
    uint8_t byte, nbBits;
};
struct HufWork {
    HufNode node0[512];
    uint8_t fseSym[64];
    uint8_t weight[256];  // HUF_writeCTable's huffWeight
    FseCT fct;            // HUF_compressWeights' table
};

// HUF_setMaxHeight
ZC_HD uint32_t huf_set_max_height(HufNode *huffNode, uint32_t lastNonNull, uint32_t maxNbBits) {
    const uint32_t largestBits = huffNode[lastNonNull].nbBits;
    if (largestBits <= maxNbBits) return largestBits;
    int totalCost = 0;
    const uint32_t baseCost = 1u << (largestBits - maxNbBits);
    int n = (int)lastNonNull;
    while (huffNode[n].nbBits > maxNbBits) {
        totalCost += (int)(baseCost - (1u << (largestBits - huffNode[n].nbBits)));
        huffNode[n].nbBits = (uint8_t)maxNbBits;
        n--;
    }
    while (huffNode[n].nbBits == maxNbBits) n--;
    totalCost >>= (largestBits - maxNbBits);
    {
        const uint32_t noSymbol = 0xF0F0F0F0u;
        uint32_t rankLast[kHufLogMax + 2];
        for (uint32_t i = 0; i < kHufLogMax + 2; i++) rankLast[i] = noSymbol;
        {
            uint32_t currentNbBits = maxNbBits;
            for (int pos = n; pos >= 0; pos--) {
                if (huffNode[pos].nbBits >= currentNbBits) continue;
                currentNbBits = huffNode[pos].nbBits;
                rankLast[maxNbBits - currentNbBits] = (uint32_t)pos;
            }
        }
        while (totalCost > 0) {
            uint32_t nBitsToDecrease = highbit32((uint32_t)totalCost) + 1;
            for (; nBitsToDecrease > 1; nBitsToDecrease--) {
                const uint32_t highPos = rankLast[nBitsToDecrease], lowPos = rankLast[nBitsToDecrease - 1];
                if (highPos == noSymbol) continue;
                if (lowPos == noSymbol) break;
                {
                    const uint32_t highTotal = huffNode[highPos].count, lowTotal = 2 * huffNode[lowPos].count;
                    if (highTotal <= lowTotal) break;
                }
            }
            while (nBitsToDecrease <= kHufLogMax && rankLast[nBitsToDecrease] == noSymbol) nBitsToDecrease++;
            totalCost -= 1 << (nBitsToDecrease - 1);
            if (rankLast[nBitsToDecrease - 1] == noSymbol) rankLast[nBitsToDecrease - 1] = rankLast[nBitsToDecrease];
            huffNode[rankLast[nBitsToDecrease]].nbBits++;
            if (rankLast[nBitsToDecrease] == 0)
                rankLast[nBitsToDecrease] = noSymbol;
            else {
                rankLast[nBitsToDecrease]--;
                if (huffNode[rankLast[nBitsToDecrease]].nbBits != maxNbBits - nBitsToDecrease)
                    rankLast[nBitsToDecrease] = noSymbol;
            }
        }
        while (totalCost < 0) {
            if (rankLast[1] == noSymbol) {
                while (huffNode[n].nbBits == maxNbBits) n--;
                huffNode[n + 1].nbBits--;
                rankLast[1] = (uint32_t)(n + 1);
                totalCost++;
                continue;
            }
            huffNode[rankLast[1] + 1].nbBits--;
            rankLast[1]++;
            totalCost++;
        }
    }
    return maxNbBits;
}

// HUF_buildCTable_wksp: returns the table log actually used
ZC_HD uint32_t huf_build_ctable(HufCT &ct, const uint32_t *count, uint32_t maxSym, uint32_t maxNbBits, HufWork &w) {
    HufNode *const huffNode0 = w.node0;
    HufNode *const huffNode = huffNode0 + 1;
    const int STARTNODE = 256;
    for (int i = 0; i < 512; i++) huffNode0[i] = HufNode{0, 0, 0, 0};
    // HUF_sort: decreasing count, stable in symbol order
    {
        uint32_t base[34], cur[34];
        for (int i = 0; i < 34; i++) base[i] = 0;
        for (uint32_t n = 0; n <= maxSym; n++) base[highbit32(count[n] + 1)]++;
        for (int n = 32; n > 0; n--) base[n - 1] += base[n];
        for (int n = 0; n < 33; n++) cur[n] = base[n + 1];
        for (uint32_t n = 0; n <= maxSym; n++) {
            const uint32_t c = count[n];
            const uint32_t r = highbit32(c + 1) + 1;
            uint32_t pos = cur[r - 1]++;
            while (pos > base[r] && c > huffNode[pos - 1].count) {
                huffNode[pos] = huffNode[pos - 1];
                pos--;
            }
            huffNode[pos].count = c;
            huffNode[pos].byte = (uint8_t)n;
        }
    }
    // HUF_buildTree
    int nonNullRank = (int)maxSym;
    while (huffNode[nonNullRank].count == 0) nonNullRank--;
    int lowS = nonNullRank, nodeNb = STARTNODE;
    const int nodeRoot = nodeNb + lowS - 1;
    int lowN = nodeNb;
    huffNode[nodeNb].count = huffNode[lowS].count + huffNode[lowS - 1].count;
    huffNode[lowS].parent = huffNode[lowS - 1].parent = (uint16_t)nodeNb;
    nodeNb++;
    lowS -= 2;
    for (int n = nodeNb; n <= nodeRoot; n++) huffNode[n].count = 1u << 30;
    huffNode0[0].count = 1u << 31;
    while (nodeNb <= nodeRoot) {
        const int n1 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        const int n2 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        huffNode[nodeNb].count = huffNode[n1].count + huffNode[n2].count;
        huffNode[n1].parent = huffNode[n2].parent = (uint16_t)nodeNb;
        nodeNb++;
    }
    huffNode[nodeRoot].nbBits = 0;
    for (int n = nodeRoot - 1; n >= STARTNODE; n--) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
    for (int n = 0; n <= nonNullRank; n++) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
    maxNbBits = huf_set_max_height(huffNode, (uint32_t)nonNullRank, maxNbBits);
    // HUF_buildCTableFromTree
    {
        uint16_t nbPerRank[kHufLogMax + 1], valPerRank[kHufLogMax + 1];
        for (uint32_t i = 0; i <= kHufLogMax; i++) nbPerRank[i] = valPerRank[i] = 0;
        for (int n = 0; n <= nonNullRank; n++) nbPerRank[huffNode[n].nbBits]++;
        {
            uint16_t mn = 0;
            for (int n = (int)maxNbBits; n > 0; n--) {
                valPerRank[n] = mn;
                mn = (uint16_t)(mn + nbPerRank[n]);
                mn >>= 1;
            }
        }
        for (uint32_t n = 0; n <= maxSym; n++) ct.nb[huffNode[n].byte] = huffNode[n].nbBits;
        for (uint32_t n = 0; n <= maxSym; n++) ct.val[n] = valPerRank[ct.nb[n]]++;
        for (uint32_t n = maxSym + 1; n < 256; n++) ct.nb[n] = 0, ct.val[n] = 0;  // "zero unused symbols"
    }
    return maxNbBits;
}

// FSE_compress_usingCTable over a short symbol string (the Huffman weights)
ZC_HD uint64_t fse_compress_symbols(uint8_t *dst, uint64_t cap, const uint8_t *src, uint32_t n, const FseCT &ct) {
    if (n <= 2) return 0;
    BitC b;
    if (!bit_init(b, dst, cap)) return 0;
    FseState s1, s2;
    int32_t ip = (int32_t)n;
    if (n & 1) {
        fse_init_state2(s1, ct, src[--ip]);
        fse_init_state2(s2, ct, src[--ip]);
        fse_encode(b, s1, ct, src[--ip]);
    } else {
        fse_init_state2(s2, ct, src[--ip]);
        fse_init_state2(s1, ct, src[--ip]);
    }
    uint32_t rem = n - 2;
    if (rem & 2) {
        fse_encode(b, s2, ct, src[--ip]);
        fse_encode(b, s1, ct, src[--ip]);
    }
    while (ip > 0) {
        fse_encode(b, s2, ct, src[--ip]);
        fse_encode(b, s1, ct, src[--ip]);
        fse_encode(b, s2, ct, src[--ip]);
        fse_encode(b, s1, ct, src[--ip]);
    }
    fse_flush_state(b, s2, ct);
    fse_flush_state(b, s1, ct);
    return bit_close(b);
}

// HUF_compressWeights
ZC_HD uint64_t huf_compress_weights(uint8_t *dst, uint64_t cap, const uint8_t *w, uint32_t n, HufWork &wk) {
    if (n <= 1) return 0;
    uint32_t count[kHufLogMax + 1];
    for (uint32_t i = 0; i <= kHufLogMax; i++) count[i] = 0;
    for (uint32_t i = 0; i < n; i++) count[w[i]]++;
    uint32_t maxSym = kHufLogMax;
    while (!count[maxSym]) maxSym--;
    uint32_t maxCount = 0;
    for (uint32_t s = 0; s <= maxSym; s++)
        if (count[s] > maxCount) maxCount = count[s];
    if (maxCount == n) return 1;
    if (maxCount == 1) return 0;
    const uint32_t tableLog = fse_optimal_table_log(6, n, maxSym, 2);
    int16_t norm[kHufLogMax + 1];
    if (fse_normalize(norm, tableLog, count, n, maxSym, false)) return 0;
    const uint32_t hs = fse_write_ncount(dst, norm, maxSym, tableLog);
    fse_build_ctable(wk.fct, norm, maxSym, tableLog, wk.fseSym);
    const uint64_t cs = fse_compress_symbols(dst + hs, cap - hs, w, n, wk.fct);
    if (cs == 0) return 0;
    return hs + cs;
}

// HUF_writeCTable
ZC_HD uint64_t huf_write_ctable(uint8_t *op, uint64_t cap, const HufCT &ct, uint32_t maxSym, uint32_t huffLog,
                                HufWork &wk) {
    uint8_t bitsToWeight[kHufLogMax + 1];
    uint8_t *const huffWeight = wk.weight;
    bitsToWeight[0] = 0;
    for (uint32_t n = 1; n < huffLog + 1; n++) bitsToWeight[n] = (uint8_t)(huffLog + 1 - n);
    for (uint32_t n = 0; n < maxSym; n++) huffWeight[n] = bitsToWeight[ct.nb[n]];
    {
        const uint64_t hSize = huf_compress_weights(op + 1, cap - 1, huffWeight, maxSym, wk);
        if (hSize > 1 && hSize < maxSym / 2) {
            op[0] = (uint8_t)hSize;
            return hSize + 1;
        }
    }
    if (maxSym > 128) return 0;  // cannot happen for compressible literals
    op[0] = (uint8_t)(128 + (maxSym - 1));
    huffWeight[maxSym] = 0;
    for (uint32_t n = 0; n < maxSym; n += 2) op[(n / 2) + 1] = (uint8_t)((huffWeight[n] << 4) + huffWeight[n + 1]);
    return ((maxSym + 1) / 2) + 1;
}

// HUF_compress1X_usingCTable_internal: symbols encoded last to first
ZC_HD uint64_t huf_compress1x(uint8_t *dst, uint64_t cap, const uint8_t *src, uint32_t n, const HufCT &ct) {
    if (cap < 8) return 0;
    BitC b;
    if (!bit_init(b, dst, cap)) return 0;
    for (int32_t i = (int32_t)n - 1; i >= 0; i--) bit_put(b, ct.val[src[i]], ct.nb[src[i]]);
    return bit_close(b);
}

// HUF_compress4X_usingCTable_internal
ZC_HD uint64_t huf_compress4x(uint8_t *dst, uint64_t cap, const uint8_t *src, uint32_t n, const HufCT &ct) {
    const uint32_t seg = (n + 3) / 4;
    if (cap < 6 + 1 + 1 + 1 + 8) return 0;
    if (n < 12) return 0;
    uint8_t *op = dst + 6;
    const uint8_t *const oend = dst + cap;
    for (int k = 0; k < 4; k++) {
        const uint32_t len = k < 3 ? seg : n - 3 * seg;
        const uint64_t c = huf_compress1x(op, (uint64_t)(oend - op), src + k * seg, len, ct);
        if (c == 0) return 0;
        if (k < 3) wr16(dst + 2 * k, (uint32_t)c);
        op += c;
    }
    return (uint64_t)(op - dst);
}

// HUF_compressCTable_internal
ZC_HD uint64_t huf_compress_ctable(uint8_t *ostart, uint8_t *op, uint64_t cap, const uint8_t *src, uint32_t n,
                                   bool single, const HufCT &ct) {
    const uint8_t *const oend = ostart + cap;
    const uint64_t c = single ? huf_compress1x(op, (uint64_t)(oend - op), src, n, ct)
                              : huf_compress4x(op, (uint64_t)(oend - op), src, n, ct);
    if (c == 0) return 0;
    op += c;
    if ((uint64_t)(op - ostart) >= (uint64_t)n - 1) return 0;
    return (uint64_t)(op - ostart);
}

// literal statistics: count[256], *maxSym = largest present symbol; returns the largest count
ZC_HD uint32_t hist_bytes(uint32_t *count, uint32_t *maxSym, const uint8_t *src, uint32_t n) {
    for (int i = 0; i < 256; i++) count[i] = 0;
    for (uint32_t i = 0; i < n; i++) count[src[i]]++;
    uint32_t m = 255;
    while (m && !count[m]) m--;
    *maxSym = m;
    uint32_t largest = 0;
    for (uint32_t s = 0; s <= m; s++)
        if (count[s] > largest) largest = count[s];
    return largest;
}

struct HufState {
    HufCT ct;
    uint32_t repeat;  // HufRepeat
};

// HUF_compress_internal (four streams or one), with the repeat logic.
// count[] is the literal histogram; largest its maximum.
ZC_HD uint64_t huf_compress(uint8_t *dst, uint64_t cap, const uint8_t *src, uint32_t n, uint32_t maxSym, uint32_t largest,
                            const uint32_t *count, bool single, HufCT &oldTable, uint32_t *repeat, bool preferRepeat,
                            HufCT &newTable, HufWork &wk) {
    uint8_t *const ostart = dst;
    uint8_t *op = dst;
    if (!n || !cap) return 0;
    if (preferRepeat && *repeat == kHufValid) return huf_compress_ctable(ostart, op, cap, src, n, single, oldTable);
    if (largest == n) {
        *ostart = src[0];
        return 1;
    }
    if (largest <= (n >> 7) + 4) return 0;
    if (*repeat == kHufCheck) {
        bool bad = false;
        for (uint32_t s = 0; s <= maxSym; s++) bad |= (count[s] != 0) & (oldTable.nb[s] == 0);
        if (bad) *repeat = kHufNone;
    }
    if (preferRepeat && *repeat != kHufNone) return huf_compress_ctable(ostart, op, cap, src, n, single, oldTable);
    uint32_t huffLog = fse_optimal_table_log(kHufLogDefault, n, maxSym, 1);
    huffLog = huf_build_ctable(newTable, count, maxSym, huffLog, wk);
    {
        const uint64_t hSize = huf_write_ctable(op, cap, newTable, maxSym, huffLog, wk);
        if (hSize == 0) return 0;
        if (*repeat != kHufNone) {
            uint64_t oldBits = 0, newBits = 0;
            for (uint32_t s = 0; s <= maxSym; s++) {
                oldBits += (uint64_t)oldTable.nb[s] * count[s];
                newBits += (uint64_t)newTable.nb[s] * count[s];
            }
            if ((oldBits >> 3) <= hSize + (newBits >> 3) || hSize + 12 >= n)
                return huf_compress_ctable(ostart, op, cap, src, n, single, oldTable);
        }
        if (hSize + 12ul >= n) return 0;
        op += hSize;
        *repeat = kHufNone;
        oldTable = newTable;  // the new table replaces the old one
    }
    return huf_compress_ctable(ostart, op, cap, src, n, single, newTable);
}

// ZSTD_noCompressLiterals / ZSTD_compressRleLiteralsBlock
ZC_HD uint32_t lit_raw(uint8_t *dst, const uint8_t *src, uint32_t n) {
    const uint32_t fl = 1 + (n > 31) + (n > 4095);
    if (fl == 1) dst[0] = (uint8_t)(kSetBasic + (n << 3));
    else if (fl == 2) wr16(dst, kSetBasic + (1u << 2) + (n << 4));
    else wr24(dst, kSetBasic + (3u << 2) + (n << 4));
    copy_bytes(dst + fl, src, n);
    return fl + n;
}
ZC_HD uint32_t lit_rle(uint8_t *dst, uint8_t b, uint32_t n) {
    const uint32_t fl = 1 + (n > 31) + (n > 4095);
    if (fl == 1) dst[0] = (uint8_t)(kSetRle + (n << 3));
    else if (fl == 2) wr16(dst, kSetRle + (1u << 2) + (n << 4));
    else wr24(dst, kSetRle + (3u << 2) + (n << 4));
    dst[fl] = b;
    return fl + 1;
}

ZC_HD uint32_t min_gain(uint32_t n) { return (n >> 6) + 2; }  // ZSTD_minGain, strategy fast

// ZSTD_compressLiterals (strategy fast, literal compression enabled).
// prev is read, next written (next = prev unless a new table was used).
ZC_HD uint64_t compress_literals(const HufState &prev, HufState &next, uint8_t *dst, uint64_t cap, const uint8_t *src,
                                 uint32_t n, uint32_t *count, HufCT &scratch, HufWork &wk) {
    const uint32_t lhSize = 3 + (n >= 1024) + (n >= 16384);
    bool single = n < 256;
    uint32_t hType = kSetCompressed;
    next = prev;
    {
        const uint32_t minLitSize = prev.repeat == kHufValid ? 6 : 63;
        if (n <= minLitSize) return lit_raw(dst, src, n);
    }
    uint64_t cLitSize;
    {
        uint32_t repeat = prev.repeat;
        const bool preferRepeat = n <= 1024;
        if (repeat == kHufValid && lhSize == 3) single = true;
        uint32_t maxSym;
        const uint32_t largest = hist_bytes(count, &maxSym, src, n);
        cLitSize = huf_compress(dst + lhSize, cap - lhSize, src, n, maxSym, largest, count, single, next.ct, &repeat,
                                preferRepeat, scratch, wk);
        if (repeat != kHufNone) hType = kSetRepeat;
    }
    if (cLitSize == 0 || cLitSize >= n - min_gain(n)) {
        next = prev;
        return lit_raw(dst, src, n);
    }
    if (cLitSize == 1) {
        next = prev;
        return lit_rle(dst, src[0], n);
    }
    if (hType == kSetCompressed) next.repeat = kHufCheck;
    const uint32_t c = (uint32_t)cLitSize;
    switch (lhSize) {
    case 3:
        wr24(dst, hType + ((uint32_t)(!single) << 2) + (n << 4) + (c << 14));
        break;
    case 4:
        wr32(dst, hType + (2u << 2) + (n << 4) + (c << 18));
        break;
    default:
        wr32(dst, hType + (3u << 2) + (n << 4) + (c << 22));
        dst[4] = (uint8_t)(c >> 10);
        break;
    }
    return lhSize + cLitSize;
}

// ---------------------------------------------------------------------------
// sequences section (zstd_compress.c, zstd_compress_sequences.c)
// ---------------------------------------------------------------------------
constexpr uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// ZSTD_LLcode / ZSTD_MLcode
ZC_HD uint32_t ll_code(uint32_t ll) {
    if (ll > 63) return highbit32(ll) + 19;
    if (ll < 16) return ll;
    const uint8_t t[48] = {16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21, 22, 22, 22, 22, 22, 22, 22, 22,
                           23, 23, 23, 23, 23, 23, 23, 23, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24};
    return t[ll - 16];
}
ZC_HD uint32_t ml_code(uint32_t ml) {
    if (ml > 127) return highbit32(ml) + 36;
    if (ml < 32) return ml;
    if (ml < 40) return 32 + ((ml - 32) >> 1);
    if (ml < 48) return 36 + ((ml - 40) >> 2);
    if (ml < 64) return 38 + ((ml - 48) >> 3);
    if (ml < 96) return 40 + ((ml - 64) >> 4);
    return 42;
}

// ZSTD_seqToCodes
ZC_HD void seq_to_codes(SeqStore &ss) {
    for (uint32_t u = 0; u < ss.nseq; u++) {
        const SeqDef d = ss.seq[u];
        ss.llc[u] = (uint8_t)ll_code(d.ll);
        ss.ofc[u] = (uint8_t)highbit32(d.offset);
        ss.mlc[u] = (uint8_t)ml_code(d.ml);
    }
    if (ss.long_id == 1) ss.llc[ss.long_pos] = kMaxLL;
    if (ss.long_id == 2) ss.mlc[ss.long_pos] = kMaxML;
}

// HIST_countFast over code bytes: *maxSym = largest present, returns the largest count
ZC_HD uint32_t hist_codes(uint32_t *count, uint32_t *maxSym, const uint8_t *codes, uint32_t n, uint32_t maxSymIn) {
    for (uint32_t s = 0; s <= maxSymIn; s++) count[s] = 0;
    for (uint32_t i = 0; i < n; i++) count[codes[i]]++;
    uint32_t m = maxSymIn;
    while (m && !count[m]) m--;
    *maxSym = m;
    uint32_t largest = 0;
    for (uint32_t s = 0; s <= m; s++)
        if (count[s] > largest) largest = count[s];
    return largest;
}

// ZSTD_selectEncodingType for strategy fast (no table is ever "valid"
// without a dictionary, so set_repeat is not reachable here)
ZC_HD uint32_t select_type(uint32_t mostFrequent, uint32_t nbSeq, uint32_t defaultNormLog, bool defaultAllowed) {
    if (mostFrequent == nbSeq) return (defaultAllowed && nbSeq <= 2) ? kSetBasic : kSetRle;
    if (defaultAllowed) {
        const uint32_t dynamicMin = ((1u << defaultNormLog) * 9) >> 3;  // mult = 10 - strategy(1)
        if (nbSeq < dynamicMin || mostFrequent < (nbSeq >> (defaultNormLog - 1))) return kSetBasic;
    }
    return kSetCompressed;
}

struct SeqWork {
    uint32_t count[64];
    int16_t norm[64];
    uint8_t tableSymbol[1u << 9];
    FseCT ll, ml, of;
};

// ZSTD_buildCTable: writes the table description (NCount or RLE byte)
ZC_HD uint32_t build_ctable(uint8_t *op, FseCT &ct, uint32_t FSELog, uint32_t type, uint32_t *count, uint32_t max,
                            const uint8_t *codes, uint32_t nbSeq, const int16_t *defNorm, uint32_t defLog,
                            uint32_t defMax, SeqWork &w) {
    if (type == kSetRle) {
        fse_build_ctable_rle(ct, max);
        op[0] = codes[0];
        return 1;
    }
    if (type == kSetBasic) {
        fse_build_ctable(ct, defNorm, defMax, defLog, w.tableSymbol);
        return 0;
    }
    uint32_t nbSeq_1 = nbSeq;
    const uint32_t tableLog = fse_optimal_table_log(FSELog, nbSeq, max, 2);
    if (count[codes[nbSeq - 1]] > 1) {
        count[codes[nbSeq - 1]]--;
        nbSeq_1--;
    }
    fse_normalize(w.norm, tableLog, count, nbSeq_1, max, nbSeq_1 >= 2048);  // ZSTD_useLowProbCount
    const uint32_t ns = fse_write_ncount(op, w.norm, max, tableLog);
    fse_build_ctable(ct, w.norm, max, tableLog, w.tableSymbol);
    return ns;
}

// ZSTD_encodeSequences (windowLog <= 19 here: no long-offset split)
ZC_HD uint64_t encode_sequences(uint8_t *dst, uint64_t cap, const SeqStore &ss, const SeqWork &w) {
    BitC b;
    if (!bit_init(b, dst, cap)) return 0;
    const uint32_t n = ss.nseq;
    FseState sML, sOF, sLL;
    fse_init_state2(sML, w.ml, ss.mlc[n - 1]);
    fse_init_state2(sOF, w.of, ss.ofc[n - 1]);
    fse_init_state2(sLL, w.ll, ss.llc[n - 1]);
    bit_put(b, ss.seq[n - 1].ll, kLLBits[ss.llc[n - 1]]);
    bit_put(b, ss.seq[n - 1].ml, kMLBits[ss.mlc[n - 1]]);
    bit_put(b, ss.seq[n - 1].offset, ss.ofc[n - 1]);
    for (int32_t i = (int32_t)n - 2; i >= 0; i--) {
        const uint32_t llc = ss.llc[i], ofc = ss.ofc[i], mlc = ss.mlc[i];
        fse_encode(b, sOF, w.of, ofc);
        fse_encode(b, sML, w.ml, mlc);
        fse_encode(b, sLL, w.ll, llc);
        bit_put(b, ss.seq[i].ll, kLLBits[llc]);
        bit_put(b, ss.seq[i].ml, kMLBits[mlc]);
        bit_put(b, ss.seq[i].offset, ofc);
    }
    fse_flush_state(b, sML, w.ml);
    fse_flush_state(b, sOF, w.of);
    fse_flush_state(b, sLL, w.ll);
    return bit_close(b);
}

// ZSTD_entropyCompressSequences(_internal): the block body, or 0 when the
// block is not compressible (stored raw by the caller)
ZC_HD uint64_t compress_block_body(const HufState &prevHuf, HufState &nextHuf, SeqStore &ss, uint8_t *dst,
                                   uint64_t cap, uint32_t blockSize, uint32_t *litCount, HufCT &hufScratch,
                                   HufWork &hw, SeqWork &sw) {
    uint8_t *const ostart = dst;
    uint8_t *op = dst;
    op += compress_literals(prevHuf, nextHuf, op, cap, ss.lit, ss.nlit, litCount, hufScratch, hw);
    const uint32_t nbSeq = ss.nseq;
    if (nbSeq < 128) {
        *op++ = (uint8_t)nbSeq;
    } else if (nbSeq < kLongNbSeq) {
        op[0] = (uint8_t)((nbSeq >> 8) + 0x80);
        op[1] = (uint8_t)nbSeq;
        op += 2;
    } else {
        op[0] = 0xFF;
        wr16(op + 1, nbSeq - kLongNbSeq);
        op += 3;
    }
    if (nbSeq != 0) {
        uint8_t *seqHead = op++;
        uint8_t *lastNCount = nullptr;
        seq_to_codes(ss);
        uint32_t max, mf, t;
        // literal lengths
        mf = hist_codes(sw.count, &max, ss.llc, nbSeq, kMaxLL);
        const uint32_t LLtype = select_type(mf, nbSeq, 6, true);
        t = build_ctable(op, sw.ll, kLLLog, LLtype, sw.count, max, ss.llc, nbSeq, kLLDef, 6, kMaxLL, sw);
        if (LLtype == kSetCompressed) lastNCount = op;
        op += t;
        // offsets
        mf = hist_codes(sw.count, &max, ss.ofc, nbSeq, kMaxOff);
        const bool ofDefault = max <= kDefaultMaxOff;
        const uint32_t OFtype = select_type(mf, nbSeq, 5, ofDefault);
        t = build_ctable(op, sw.of, kOffLog, OFtype, sw.count, max, ss.ofc, nbSeq, kOFDef, 5, kDefaultMaxOff, sw);
        if (OFtype == kSetCompressed) lastNCount = op;
        op += t;
        // match lengths
        mf = hist_codes(sw.count, &max, ss.mlc, nbSeq, kMaxML);
        const uint32_t MLtype = select_type(mf, nbSeq, 6, true);
        t = build_ctable(op, sw.ml, kMLLog, MLtype, sw.count, max, ss.mlc, nbSeq, kMLDef, 6, kMaxML, sw);
        if (MLtype == kSetCompressed) lastNCount = op;
        op += t;
        *seqHead = (uint8_t)((LLtype << 6) + (OFtype << 4) + (MLtype << 2));
        if ((uint64_t)(op - ostart) + 16 >= cap) return 0;  // no room left: stored raw (dstSize_tooSmall)
        const uint64_t bs = encode_sequences(op, cap - (uint64_t)(op - ostart), ss, sw);
        if (bs == 0) return 0;
        op += bs;
        // zstd <= 1.3.4 decoders and a last NCount of < 4 bytes: stored raw
        if (lastNCount && (op - lastNCount) < 4) return 0;
    }
    const uint64_t cSize = (uint64_t)(op - ostart);
    if (cSize >= blockSize - min_gain(blockSize)) return 0;
    return cSize;
}

// ---------------------------------------------------------------------------
// frame (ZSTD_writeFrameHeader, ZSTD_compress_frameChunk)
// ---------------------------------------------------------------------------
ZC_HD uint32_t write_frame_header(uint8_t *op, uint64_t n, Params P) {
    const uint64_t windowSize = 1ull << P.wlog;
    const uint32_t single = windowSize >= n;
    const uint32_t fcsCode = (n >= 256) + (n >= 65536 + 256) + (n >= 0xFFFFFFFFull);
    wr32(op, 0xFD2FB528u);
    uint32_t pos = 4;
    op[pos++] = (uint8_t)((single << 5) + (fcsCode << 6));
    if (!single) op[pos++] = (uint8_t)((P.wlog - 10) << 3);
    switch (fcsCode) {
    case 0:
        if (single) op[pos++] = (uint8_t)n;
        break;
    case 1:
        wr16(op + pos, (uint32_t)(n - 256));
        pos += 2;
        break;
    case 2:
        wr32(op + pos, (uint32_t)n);
        pos += 4;
        break;
    default:
        wr32(op + pos, (uint32_t)n);
        wr32(op + pos + 4, (uint32_t)(n >> 32));
        pos += 8;
        break;
    }
    return pos;
}

ZC_HD bool is_rle(const uint8_t *p, uint32_t n) {
    for (uint32_t i = 1; i < n; i++)
        if (p[i] != p[0]) return false;
    return true;
}

// Everything one object's encoder keeps between blocks, plus scratch.  The
// literal stage's scratch and the sequence stage's share storage: a block's
// literals section is finished before its sequence tables are built (9.3 KiB
// instead of 14.8, so 16 one-wave workgroups fit a CU's LDS).
struct Work {
    HufState prev, next;
    union {
        struct {
            HufCT hufScratch;
            HufWork hw;
            uint32_t litCount[256];
        };
        SeqWork sw;
    };
};

// One compressed block body is built in a scratch buffer of kBodyCap bytes
// and copied to the frame only when it is kept, so the frame never grows past
// ZSTD_compressBound (the library's dstCapacity checks end in a raw block
// exactly when the body would not be kept here).
constexpr uint32_t kBodyCap = kBlockMax + 1024;

// The whole ZSTD_compress(level 1) of src[0, n) into dst (capacity >= bound).
// htab: (1 << kHashLogMax) words; seq / lit / codes: one block's worth;
// body: kBodyCap bytes.
ZC_HD uint64_t compress_frame(const uint8_t *src, uint64_t n, uint8_t *dst, uint32_t *htab, SeqDef *seqs, uint8_t *lits,
                              uint8_t *codes, uint8_t *body, Work &w) {
    const Params P = level1_params(n);
    uint8_t *op = dst;
    op += write_frame_header(op, n, P);
    if (n == 0) {
        wr24(op, 1);  // one empty raw last block
        return (uint64_t)(op + 3 - dst);
    }
    for (uint32_t i = 0; i < (1u << P.hlog); i++) htab[i] = 0;
    uint32_t rep[2] = {1, 4};  // repStartValue (the third, 8, is unused by this parser)
    w.prev.repeat = kHufNone;
    for (int i = 0; i < 256; i++) w.prev.ct.nb[i] = 0, w.prev.ct.val[i] = 0;
    const uint32_t blockMax = (1u << P.wlog) < kBlockMax ? (1u << P.wlog) : kBlockMax;
    bool first = true;
    for (uint64_t pos = 0; pos < n;) {
        const uint32_t bs = (uint32_t)((n - pos) < blockMax ? (n - pos) : blockMax);
        const uint32_t last = (pos + bs == n);
        const uint8_t *ip = src + pos;
        uint64_t cSize = 0;
        if (bs >= 7) {  // MIN_CBLOCK_SIZE + ZSTD_blockHeaderSize + 1
            SeqStore ss;
            ss.seq = seqs;
            ss.lit = lits;
            ss.llc = codes;
            ss.mlc = codes + kMaxSeq;
            ss.ofc = codes + 2 * kMaxSeq;
            ss.nseq = ss.nlit = 0;
            ss.long_id = ss.long_pos = 0;
            uint32_t nrep[2] = {rep[0], rep[1]};
            const uint32_t lastLL = parse_fast(src, (int32_t)pos, (int32_t)(pos + bs), htab, P, nrep, ss);
            copy_bytes(ss.lit + ss.nlit, src + pos + bs - lastLL, lastLL);
            ss.nlit += lastLL;
            cSize = compress_block_body(w.prev, w.next, ss, body, kBodyCap, bs, w.litCount, w.hufScratch, w.hw, w.sw);
            if (!first && cSize < kRleMaxLength && is_rle(ip, bs)) cSize = 1;
            if (cSize > 1) {
                // ZSTD_confirmRepcodesAndEntropyTables: the parse's repcodes
                // and tables become the next block's (the fast parser never
                // touches the third repcode)
                rep[0] = nrep[0];
                rep[1] = nrep[1];
                w.prev = w.next;
            }
        }
        if (cSize == 0) {
            wr24(op, last + (0u << 1) + (bs << 3));
            copy_bytes(op + 3, ip, bs);
            op += 3 + bs;
        } else if (cSize == 1) {
            wr24(op, last + (1u << 1) + (bs << 3));
            op[3] = ip[0];
            op += 4;
        } else {
            wr24(op, last + (2u << 1) + ((uint32_t)cSize << 3));
            copy_bytes(op + 3, body, (uint32_t)cSize);
            op += 3 + cSize;
        }
        pos += bs;
        first = false;
    }
    return (uint64_t)(op - dst);
}

}  // namespace jzc

/* jfs_lz4.c -- CPU restatement of the LZ4 block codec the reference's "lz4"
 * compressor calls (TEST INFRASTRUCTURE ONLY: loaded by tests/ and bench.py's
 * cpu_baseline leg through oracle/oracle.py, never by juicefs_amd/).
 *
 * Reference call sites: pkg/compress/compress.go:107-125 (LZ4.CompressBound ->
 * lz4.CompressBound, LZ4.Compress -> lz4.CompressDefault(src, dst),
 * LZ4.Decompress -> "decompress an empty input" on len(src)==0, else
 * lz4.DecompressSafe(src, dst)), used by cachedStore.upload
 * (pkg/chunk/cached_store.go:371-392: CompressBound-sized buffer, then
 * Compress) and cachedStore.load (:680-745: Decompress into the block page,
 * "read %s fully" when n < len(page)).
 *
 * The arithmetic lives in github.com/hungys/go-lz4 v0.0.0-20170805124057
 * (go.mod:34), a cgo wrapper over the LZ4 C library (LZ4_compress_default,
 * LZ4_decompress_safe, LZ4_compressBound); the vendored C sources are not in
 * /root/reference.  This file restates, from the published LZ4 block format
 * and the LZ4 1.9.x greedy "fast" compressor (acceleration 1, 16 KiB hash
 * table, 4-byte hash for inputs below 64 KiB + 11 bytes with a 2^13-entry
 * 16-bit table, 5-byte hash otherwise with a 2^12-entry 32-bit table, skip
 * trigger 6, MINMATCH 4, MFLIMIT 12, LASTLITERALS 5, max distance 65535):
 *   * orc_lz4_bound       = LZ4_compressBound(n)  = n + n/255 + 16
 *   * orc_lz4_compress    = LZ4_compress_default(src, dst, n, bound(n))
 *   * orc_lz4_decompress  = LZ4_decompress_safe(src, dst, n, cap)
 * It is pinned against the system liblz4 (1.9.3, dlopen'd by the tests).
 */
#include <stdint.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))

enum { MINMATCH = 4, MFLIMIT = 12, LASTLITERALS = 5, ML_BITS = 4, ML_MASK = 15, RUN_MASK = 15,
       SKIP_TRIGGER = 6, HASHLOG = 12, DIST_MAX = 65535, LIMIT64K = 65536 + MFLIMIT - 1 };

static inline uint32_t rd32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
static inline uint64_t rd64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

/* hash of the 4 (small inputs) or 5 (large inputs) bytes at p */
static inline uint32_t lz4_hash(const uint8_t *p, int small) {
    if (small) return (rd32(p) * 2654435761u) >> (32 - (HASHLOG + 1));
    return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> (64 - HASHLOG));
}

/* number of equal bytes at a and b, a's side capped at lim */
static inline uint32_t lz4_count(const uint8_t *a, const uint8_t *b, const uint8_t *lim) {
    const uint8_t *s = a;
    while (a < lim && *a == *b) a++, b++;
    return (uint32_t)(a - s);
}

EXPORT int orc_lz4_bound(int n) { return (n < 0 || n > 0x7E000000) ? 0 : n + n / 255 + 16; }

EXPORT int orc_lz4_compress(const uint8_t *src, int n, uint8_t *dst, int cap) {
    if (n < 0 || cap < orc_lz4_bound(n)) return 0;
    const int small = n < LIMIT64K;
    uint32_t table[1 << (HASHLOG + 1)];  /* 16 KiB: 8192 x u16 or 4096 x u32 */
    memset(table, 0, sizeof(table));
    uint16_t *t16 = (uint16_t *)table;
    uint32_t *t32 = table;
#define GET(h) (small ? (uint32_t)t16[h] : t32[h])
#define PUT(h, v) do { if (small) t16[h] = (uint16_t)(v); else t32[h] = (v); } while (0)
    const uint8_t *ip = src, *anchor = src;
    const uint8_t *const iend = src + n;
    const uint8_t *const mflimit1 = iend - MFLIMIT + 1;
    const uint8_t *const matchlimit = iend - LASTLITERALS;
    uint8_t *op = dst;
    const uint8_t *match;
    uint8_t *token;
    uint32_t fh;

    if (n < MFLIMIT + 1) goto last_literals;
    PUT(lz4_hash(ip, small), 0u);
    ip++;
    fh = lz4_hash(ip, small);
    for (;;) {
        /* find a match: attempts at ip, ip+step, ... with the step growing
         * by one every 64 misses */
        {
            const uint8_t *fip = ip;
            int step = 1, nb = 1 << SKIP_TRIGGER;
            for (;;) {
                const uint32_t h = fh;
                const uint32_t cur = (uint32_t)(fip - src);
                const uint32_t mi = GET(h);
                ip = fip;
                fip += step;
                step = nb++ >> SKIP_TRIGGER;
                if (fip > mflimit1) goto last_literals;
                match = src + mi;
                fh = lz4_hash(fip, small);
                PUT(h, cur);
                if (!small && mi + DIST_MAX < cur) continue;
                if (rd32(match) == rd32(ip)) break;
            }
        }
        /* catch up: extend backwards */
        while (ip > anchor && match > src && ip[-1] == match[-1]) ip--, match--;
        /* literals */
        {
            const uint32_t ll = (uint32_t)(ip - anchor);
            token = op++;
            if (ll >= RUN_MASK) {
                int len = (int)(ll - RUN_MASK);
                *token = RUN_MASK << ML_BITS;
                for (; len >= 255; len -= 255) *op++ = 255;
                *op++ = (uint8_t)len;
            } else {
                *token = (uint8_t)(ll << ML_BITS);
            }
            memcpy(op, anchor, ll);
            op += ll;
        }
    next_match:
        /* offset, match length */
        {
            const uint32_t off = (uint32_t)(ip - match);
            *op++ = (uint8_t)off;
            *op++ = (uint8_t)(off >> 8);
            uint32_t mc = lz4_count(ip + MINMATCH, match + MINMATCH, matchlimit);
            ip += mc + MINMATCH;
            if (mc >= ML_MASK) {
                *token += ML_MASK;
                mc -= ML_MASK;
                for (; mc >= 255; mc -= 255) *op++ = 255;
                *op++ = (uint8_t)mc;
            } else {
                *token += (uint8_t)mc;
            }
        }
        anchor = ip;
        if (ip >= mflimit1) break;
        /* fill the table at ip - 2, then try ip itself as a new match start */
        PUT(lz4_hash(ip - 2, small), (uint32_t)(ip - 2 - src));
        {
            const uint32_t h = lz4_hash(ip, small);
            const uint32_t cur = (uint32_t)(ip - src);
            const uint32_t mi = GET(h);
            match = src + mi;
            PUT(h, cur);
            if ((small || mi + DIST_MAX >= cur) && rd32(match) == rd32(ip)) {
                token = op++;
                *token = 0;
                goto next_match;
            }
        }
        fh = lz4_hash(++ip, small);
    }
last_literals:
    {
        size_t run = (size_t)(iend - anchor);
        if (run >= RUN_MASK) {
            size_t acc = run - RUN_MASK;
            *op++ = RUN_MASK << ML_BITS;
            for (; acc >= 255; acc -= 255) *op++ = 255;
            *op++ = (uint8_t)acc;
        } else {
            *op++ = (uint8_t)(run << ML_BITS);
        }
        memcpy(op, anchor, run);
        op += run;
    }
#undef GET
#undef PUT
    return (int)(op - dst);
}

/* LZ4_decompress_safe: the decoded size, or a negative value for a malformed
 * stream (reads past the input, writes past cap, an offset before the output
 * start, a match in the last 5 output bytes, or a last sequence that does not
 * end the input exactly).  The same accept/reject rules as the 1.9.x safe
 * decoder's general loop: a match may not end within LASTLITERALS of cap, a
 * literal run that reaches into the last MFLIMIT bytes of cap (or the last
 * 8 input bytes) must be the final sequence. */
EXPORT int orc_lz4_decompress(const uint8_t *src, int n, uint8_t *dst, int cap) {
    const uint8_t *ip = src, *const iend = src + n;
    uint8_t *op = dst, *const oend = dst + cap;
    if (cap == 0) return (n == 1 && *ip == 0) ? 0 : -1;
    if (n == 0) return -1;
    for (;;) {
        if (ip >= iend) return -1;
        const unsigned token = *ip++;
        size_t len = token >> ML_BITS;
        if (len == RUN_MASK) {
            unsigned s;
            do {
                if (ip >= iend - RUN_MASK) return -1;
                s = *ip++;
                len += s;
            } while (s == 255);
        }
        /* literals */
        uint8_t *cpy = op + len;
        if ((size_t)(oend - op) < len || (size_t)(iend - ip) < len) return -1;
        if (cpy > oend - MFLIMIT || ip + len > iend - (2 + 1 + LASTLITERALS)) {
            /* must be the last sequence */
            if (ip + len != iend || cpy > oend) return -1;
            memmove(op, ip, len);
            op += len;
            break;
        }
        memcpy(op, ip, len);
        ip += len;
        op = cpy;
        /* offset */
        const size_t off = (size_t)ip[0] | ((size_t)ip[1] << 8);
        ip += 2;
        if (off > (size_t)(op - dst)) return -1;
        const uint8_t *match = op - off;
        len = token & ML_MASK;
        if (len == ML_MASK) {
            unsigned s;
            do {
                if (ip > iend - LASTLITERALS) return -1;
                s = *ip++;
                len += s;
            } while (s == 255);
        }
        len += MINMATCH;
        if ((size_t)(oend - op) < len || op + len > oend - LASTLITERALS) return -1;
        for (size_t i = 0; i < len; i++) op[i] = match[i];  /* byte-wise: overlapping copies replicate */
        op += len;
    }
    return (int)(op - dst);
}

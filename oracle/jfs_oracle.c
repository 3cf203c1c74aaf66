/*
 * jfs_oracle.c -- CPU restatement of the JuiceFS per-block transform path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in juicefs_amd/ (the product) links,
 * loads or calls this file.  It is used by tests/ (as the parity checker),
 * by __graft_entry__.smoke() (as the checker) and by bench.py's
 * cpu_baseline leg (timed as the "port" of the reference's Go CPU path).
 *
 * What it restates (reference = /root/reference, JuiceFS 1.2.0):
 *   - dataEncryptor.Encrypt / Decrypt object format ......... pkg/object/encrypt.go:164-216
 *   - NewDataEncryptor algorithm dispatch ..................... pkg/object/encrypt.go:142-162
 *   - AES-256-GCM (Go crypto/aes + crypto/cipher.NewGCM,
 *     called at encrypt.go:150-156,192,215) per NIST SP 800-38D
 *     (96-bit IV, 128-bit tag, empty AAD)
 *   - ChaCha20-Poly1305 (golang.org/x/crypto v0.19.0
 *     chacha20poly1305.New, encrypt.go:158-159) per RFC 8439
 *   - CRC32C (Go hash/crc32, Castagnoli table) ............... pkg/chunk/disk_cache.go:1210
 *   - checksum(): one CRC32C per 32 KiB segment, big-endian .. pkg/chunk/disk_cache.go:1218-1231
 *                                                               pkg/utils/buffer.go:42-44,98-101
 *   - openCacheFile level detection ........................... pkg/chunk/disk_cache.go:1233-1253
 *   - cacheFile.ReadAt none/full/shrink/extend verify ......... pkg/chunk/disk_cache.go:1255-1329
 *
 * The arithmetic itself (AES, GHASH, ChaCha20, Poly1305, CRC32C) is not in
 * /root/reference: it lives in the Go standard library and in
 * golang.org/x/crypto v0.19.0 (go.mod:76).  It is restated here from the
 * published standards (FIPS-197, SP 800-38D, RFC 8439, RFC 3720 B.4) and
 * pinned by the published KATs plus OpenSSL-generated golden vectors
 * (tests/golden/, made by tests/golden/make_golden.py).
 *
 * Two implementations of AES-GCM and CRC32C are kept:
 *   portable  -- byte-oriented, bit-serial GHASH; the readable restatement.
 *   x86 fast  -- AES-NI + PCLMULQDQ + SSE4.2 crc32, the same instruction
 *                classes Go's amd64 assembly uses; used for the CPU baseline
 *                timing and cross-checked against the portable one in tests.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>
#include <dlfcn.h>
#include <immintrin.h>
#include <wmmintrin.h>
#include <nmmintrin.h>

#define ORC_EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------ */
/* synthetic data (shared definition with the GPU generator)           */
/* ------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
#define GOLDEN 0x9E3779B97F4A7C15ULL

/* word k of block b: mix64(seed + GOLDEN * ((b << 40) + k + 1)), little-endian bytes */
ORC_EXPORT void orc_gen_block(uint64_t seed, uint64_t b, uint8_t *out, uint64_t len) {
    uint64_t nw = len / 8, k;
    for (k = 0; k < nw; k++) {
        uint64_t w = mix64(seed + GOLDEN * ((b << 40) + k + 1));
        memcpy(out + 8 * k, &w, 8);
    }
    if (len % 8) {
        uint64_t w = mix64(seed + GOLDEN * ((b << 40) + nw + 1));
        memcpy(out + 8 * nw, &w, len % 8);
    }
}

/* per-block key (32 B) and nonce (12 B); the reference draws them from
 * crypto/rand (encrypt.go:165-168,177-180); the engine takes them as inputs. */
ORC_EXPORT void orc_gen_key(uint64_t seed, uint64_t b, uint8_t key[32], uint8_t nonce[12]) {
    int i;
    for (i = 0; i < 4; i++) {
        uint64_t w = mix64((seed ^ 0x4B4559ULL) + GOLDEN * ((b << 8) + i + 1));
        memcpy(key + 8 * i, &w, 8);
    }
    uint64_t w0 = mix64((seed ^ 0x4E4F4E4345ULL) + GOLDEN * ((b << 8) + 1));
    uint64_t w1 = mix64((seed ^ 0x4E4F4E4345ULL) + GOLDEN * ((b << 8) + 2));
    memcpy(nonce, &w0, 8);
    memcpy(nonce + 8, &w1, 4);
}

/* ------------------------------------------------------------------ */
/* CRC32C (Castagnoli, reflected poly 0x82F63B78, init/xorout ~0)      */
/* Go: crc32.MakeTable(crc32.Castagnoli), disk_cache.go:1210           */
/* ------------------------------------------------------------------ */
static uint32_t crc_tab[256];
static int crc_init_done;

static void crc_init(void) {
    if (crc_init_done) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        crc_tab[i] = c;
    }
    crc_init_done = 1;
}

/* crc32.Update(crc, castagnoli, p) -- portable, byte at a time */
ORC_EXPORT uint32_t orc_crc32c_update(uint32_t crc, const uint8_t *p, uint64_t n) {
    crc_init();
    crc = ~crc;
    for (uint64_t i = 0; i < n; i++) crc = crc_tab[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    return ~crc;
}

/* SSE4.2 variant (Go's amd64 castagnoliSSE42 class) */
__attribute__((target("sse4.2"))) ORC_EXPORT uint32_t orc_crc32c_update_hw(uint32_t crc, const uint8_t *p, uint64_t n) {
    uint64_t c = (uint32_t)~crc;
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        c = _mm_crc32_u64(c, w);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = (uint32_t)c;
    while (n--) c32 = _mm_crc32_u8(c32, *p++);
    return ~c32;
}

/* x^(8n) mod P in the reflected convention (bit 31 = x^0), for combining
 * CRC registers of adjacent spans: reg(A||B) = reg(A) * x^(8|B|) ^ reg0(B) */
static uint32_t crc_mulmod_r(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & 0x80000000u) p ^= b;
        a <<= 1;
        b = (b & 1) ? (b >> 1) ^ 0x82F63B78u : b >> 1;
    }
    return p;
}
static uint32_t crc_xpow8_r(uint64_t n) {
    uint32_t r = 0x80000000u, x = 0x00800000u; /* x^0, x^8 */
    for (; n; n >>= 1) {
        if (n & 1) r = crc_mulmod_r(x, r);
        x = crc_mulmod_r(x, x);
    }
    return r;
}

/* Three interleaved crc32 streams over thirds of the span, combined by GF(2)
 * shifts: the shape of Go's castagnoliSSE42Triple (hash/crc32, amd64), which
 * hides the crc32 instruction's latency.  Same value as orc_crc32c_update_hw. */
__attribute__((target("sse4.2"))) ORC_EXPORT uint32_t orc_crc32c_update_hw3(uint32_t crc, const uint8_t *p,
                                                                           uint64_t n) {
    static __thread uint64_t k_cached;
    static __thread uint32_t xk_cached;
    const uint64_t k = (n / 24) * 8; /* bytes per stream, a multiple of 8 */
    if (k < 256) return orc_crc32c_update_hw(crc, p, n);
    if (k != k_cached) {
        k_cached = k;
        xk_cached = crc_xpow8_r(k);
    }
    uint64_t a = (uint32_t)~crc, b = 0, c = 0;
    const uint8_t *pa = p, *pb = p + k, *pc = p + 2 * k;
    for (uint64_t i = 0; i < k; i += 8) {
        uint64_t wa, wb, wc;
        memcpy(&wa, pa + i, 8);
        memcpy(&wb, pb + i, 8);
        memcpy(&wc, pc + i, 8);
        a = _mm_crc32_u64(a, wa);
        b = _mm_crc32_u64(b, wb);
        c = _mm_crc32_u64(c, wc);
    }
    uint32_t r = crc_mulmod_r(xk_cached, crc_mulmod_r(xk_cached, (uint32_t)a) ^ (uint32_t)b) ^ (uint32_t)c;
    return orc_crc32c_update_hw(~r, p + 3 * k, n - 3 * k);
}

#define CS_BLOCK (32 << 10) /* csBlock, disk_cache.go:1207 */

static inline void put_be32(uint8_t *p, uint32_t v) {
    p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v;
}
static inline uint32_t get_be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* Go integer division truncates toward zero: ((length-1)/csBlock+1)*4, so
 * length 0 gives 4 bytes (disk_cache.go:1221, 1243). */
ORC_EXPORT int64_t orc_checksum_len(int64_t length) {
    return ((length - 1) / CS_BLOCK + 1) * 4;
}

/* checksum(data) -- disk_cache.go:1218-1231.  out must hold orc_checksum_len(n). */
ORC_EXPORT int64_t orc_checksum(const uint8_t *data, int64_t length, uint8_t *out, int hw) {
    int64_t ol = orc_checksum_len(length);
    memset(out, 0, (size_t)ol);
    int64_t off = 0;
    for (int64_t start = 0, end = 0; start < length; start = end) {
        end = start + CS_BLOCK;
        if (end > length) end = length;
        uint32_t sum = hw ? orc_crc32c_update_hw3(0, data + start, (uint64_t)(end - start))
                          : orc_crc32c_update(0, data + start, (uint64_t)(end - start));
        put_be32(out + off, sum);
        off += 4;
    }
    return ol;
}

/* checksum levels (disk_cache.go:1202-1205) */
enum { CS_NONE = 0, CS_FULL = 1, CS_SHRINK = 2, CS_EXTEND = 3 };

/* openCacheFile size rule (disk_cache.go:1233-1253): returns the effective
 * level, or -1 for "invalid file size". */
ORC_EXPORT int orc_open_cache_file(int64_t file_size, int64_t length, int level) {
    int64_t cl = orc_checksum_len(length);
    if (file_size - length == 0) return CS_NONE;
    if (file_size - length == cl) return level;
    return -1;
}

/* File.ReadAt on an in-memory file image: n bytes copied, eof flag if short */
static int64_t file_pread(const uint8_t *file, int64_t fsize, uint8_t *dst, int64_t size, int64_t off,
                          int *eof) {
    int64_t n = 0;
    *eof = 0;
    if (off < fsize) {
        n = fsize - off;
        if (n > size) n = size;
        memcpy(dst, file + off, (size_t)n);
    }
    if (n < size) *eof = 1;
    return n;
}

/*
 * cacheFile.ReadAt (disk_cache.go:1255-1329) on an in-memory image of the
 * cache file (data ‖ BE32 CRCs).  level is the effective level returned by
 * orc_open_cache_file.  Returns:
 *    0  ok (out filled, *n_out bytes)
 *    1  "data checksum %d != expect %d" (got/expect/bad_seg filled; *n_out as Go)
 *    2  short read (io.EOF)
 *   -1  bad arguments
 * bad_seg is the index (relative to the file's segment 0) of the first
 * failing segment.
 */
static int cache_readat(const uint8_t *file, int64_t fsize, int64_t length, int level, int64_t off, int64_t size,
                        uint8_t *out, int64_t *n_out, uint32_t *got, uint32_t *expect, int64_t *bad_seg, int hw);

ORC_EXPORT int orc_cache_readat(const uint8_t *file, int64_t fsize, int64_t length, int level,
                                int64_t off, int64_t size, uint8_t *out, int64_t *n_out,
                                uint32_t *got, uint32_t *expect, int64_t *bad_seg) {
    return cache_readat(file, fsize, length, level, off, size, out, n_out, got, expect, bad_seg, 0);
}

/* the same with the 3-stream SSE4.2 CRC (the CPU baseline's ReadAt) */
ORC_EXPORT int orc_cache_readat_hw(const uint8_t *file, int64_t fsize, int64_t length, int level,
                                   int64_t off, int64_t size, uint8_t *out, int64_t *n_out,
                                   uint32_t *got, uint32_t *expect, int64_t *bad_seg) {
    return cache_readat(file, fsize, length, level, off, size, out, n_out, got, expect, bad_seg, 1);
}

static int cache_readat(const uint8_t *file, int64_t fsize, int64_t length, int level, int64_t off, int64_t size,
                        uint8_t *out, int64_t *n_out, uint32_t *got, uint32_t *expect, int64_t *bad_seg, int hw) {
    int eof = 0;
    *n_out = 0;
    if (level == CS_NONE || (level == CS_FULL && (off != 0 || size != length))) {
        *n_out = file_pread(file, fsize, out, size, off, &eof);
        return eof ? 2 : 0;
    }
    uint8_t *rb = out;
    int64_t rbsize = size;
    int64_t roff = off;
    uint8_t *tmp = NULL;
    if (level == CS_EXTEND) {
        roff = off / CS_BLOCK * CS_BLOCK;
        int64_t rend = off + size;
        if (rend % CS_BLOCK != 0) {
            rend = (rend / CS_BLOCK + 1) * CS_BLOCK;
            if (rend > length) rend = length;
        }
        if (rend - roff != size) {
            rbsize = rend - roff;
            tmp = (uint8_t *)malloc(rbsize > 0 ? (size_t)rbsize : 1);
            rb = tmp;
        }
    }
    int64_t n = file_pread(file, fsize, rb, rbsize, roff, &eof);
    int rc = 0;
    if (eof) {
        rc = 2;
        goto done;
    }
    {
        int64_t ioff = roff / CS_BLOCK;
        int64_t cstart = 0, clen = rbsize;
        if (level == CS_SHRINK) {
            if (roff % CS_BLOCK != 0) {
                int64_t o = CS_BLOCK - roff % CS_BLOCK;
                if (clen <= o) goto done;
                cstart += o;
                clen -= o;
                ioff += 1;
            }
            int64_t end = roff + n;
            if (end != length && end % CS_BLOCK != 0) {
                if (clen <= end % CS_BLOCK) goto done;
                clen -= end % CS_BLOCK;
            }
        }
        int64_t nexp = (clen - 1) / CS_BLOCK + 1;
        uint8_t *ebuf = (uint8_t *)malloc((size_t)(nexp * 4));
        int eof2 = 0;
        file_pread(file, fsize, ebuf, nexp * 4, length + ioff * 4, &eof2);
        if (eof2) {
            free(ebuf);
            rc = 2;
            goto done;
        }
        int64_t k = 0;
        for (int64_t s = 0, e = 0; s < clen; s = e, k++) {
            e = s + CS_BLOCK;
            if (e > clen) e = clen;
            uint32_t sum = hw ? orc_crc32c_update_hw3(0, rb + cstart + s, (uint64_t)(e - s))
                              : orc_crc32c_update(0, rb + cstart + s, (uint64_t)(e - s));
            uint32_t ex = get_be32(ebuf + 4 * k);
            if (sum != ex) {
                *got = sum;
                *expect = ex;
                *bad_seg = ioff + k;
                rc = 1;
                break;
            }
        }
        free(ebuf);
    }
done:
    if (tmp) {
        /* extend: n = copy(b, rb[off-roff:]) on success, 0 on error */
        if (rc == 0) {
            int64_t avail = rbsize - (off - roff);
            int64_t c = avail < size ? avail : size;
            if (c > 0) memcpy(out, tmp + (off - roff), (size_t)c);
            *n_out = c;
        } else {
            *n_out = 0;
        }
        free(tmp);
    } else {
        *n_out = n;
    }
    return rc;
}

/* ------------------------------------------------------------------ */
/* AES-256 (FIPS-197), portable byte-oriented restatement               */
/* ------------------------------------------------------------------ */
static uint8_t sbox[256];
static int aes_init_done;

static uint8_t gf8_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0));
        b >>= 1;
    }
    return p;
}

static void aes_init(void) {
    if (aes_init_done) return;
    for (int x = 0; x < 256; x++) {
        /* inverse = x^254 in GF(2^8) mod x^8+x^4+x^3+x+1 (0 maps to 0) */
        uint8_t inv = 1, base = (uint8_t)x;
        int e = 254;
        while (e) {
            if (e & 1) inv = gf8_mul(inv, base);
            base = gf8_mul(base, base);
            e >>= 1;
        }
        if (x == 0) inv = 0;
        uint8_t s = inv;
        uint8_t r = s;
        for (int k = 1; k <= 4; k++) r ^= (uint8_t)((s << k) | (s >> (8 - k)));
        sbox[x] = r ^ 0x63;
    }
    aes_init_done = 1;
}

/* AES-256 key expansion: Nk=8, Nr=14, 60 words (240 bytes) */
ORC_EXPORT void orc_aes256_expand(const uint8_t key[32], uint8_t rk[240]) {
    aes_init();
    memcpy(rk, key, 32);
    uint8_t rcon = 1;
    for (int i = 8; i < 60; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            uint8_t t0 = t[0];
            t[0] = sbox[t[1]] ^ rcon;
            t[1] = sbox[t[2]];
            t[2] = sbox[t[3]];
            t[3] = sbox[t0];
            rcon = gf8_mul(rcon, 2);
        } else if (i % 8 == 4) {
            for (int k = 0; k < 4; k++) t[k] = sbox[t[k]];
        }
        for (int k = 0; k < 4; k++) rk[4 * i + k] = rk[4 * (i - 8) + k] ^ t[k];
    }
}

ORC_EXPORT void orc_aes256_encrypt_block(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    aes_init();
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= 14; r++) {
        uint8_t t[16];
        /* SubBytes + ShiftRows: byte (row i, col c) <- (row i, col c+i) */
        for (int c = 0; c < 4; c++)
            for (int i = 0; i < 4; i++) t[4 * c + i] = sbox[s[4 * ((c + i) & 3) + i]];
        if (r != 14) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3);
                s[4 * c + 3] = gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

ORC_EXPORT void orc_sbox(uint8_t out[256]) {
    aes_init();
    memcpy(out, sbox, 256);
}

/* ------------------------------------------------------------------ */
/* GCM (SP 800-38D), portable: bit-serial GF(2^128) multiply (Alg. 1)  */
/* ------------------------------------------------------------------ */
ORC_EXPORT void orc_gf128_mul(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) {
    uint8_t V[16], R[16];
    memcpy(V, Y, 16);
    memset(R, 0, 16);
    for (int i = 0; i < 128; i++) {
        if ((X[i >> 3] >> (7 - (i & 7))) & 1)
            for (int k = 0; k < 16; k++) R[k] ^= V[k];
        int lsb = V[15] & 1;
        for (int k = 15; k > 0; k--) V[k] = (uint8_t)((V[k] >> 1) | (V[k - 1] << 7));
        V[0] >>= 1;
        if (lsb) V[0] ^= 0xE1;
    }
    memcpy(Z, R, 16);
}

static void ghash_update(uint8_t Y[16], const uint8_t H[16], const uint8_t *p, uint64_t n) {
    while (n) {
        uint8_t blk[16] = {0};
        uint64_t c = n < 16 ? n : 16;
        memcpy(blk, p, c);
        for (int k = 0; k < 16; k++) Y[k] ^= blk[k];
        orc_gf128_mul(Y, H, Y);
        p += c;
        n -= c;
    }
}

static void gcm_core(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, uint64_t alen,
                     const uint8_t *in, uint64_t len, uint8_t *out, uint8_t tag[16], int decrypt) {
    uint8_t rk[240], H[16] = {0}, J0[16], EJ0[16], Y[16] = {0}, ctr[16], ks[16];
    orc_aes256_expand(key, rk);
    orc_aes256_encrypt_block(rk, H, H);
    memcpy(J0, nonce, 12);
    J0[12] = 0; J0[13] = 0; J0[14] = 0; J0[15] = 1;
    orc_aes256_encrypt_block(rk, J0, EJ0);
    ghash_update(Y, H, aad, alen);
    if (decrypt) ghash_update(Y, H, in, len);
    memcpy(ctr, J0, 16);
    uint32_t cnt = 1;
    for (uint64_t off = 0; off < len; off += 16) {
        cnt++; /* inc32: first data block uses counter 2 */
        put_be32(ctr + 12, cnt);
        orc_aes256_encrypt_block(rk, ctr, ks);
        uint64_t c = len - off < 16 ? len - off : 16;
        for (uint64_t k = 0; k < c; k++) out[off + k] = in[off + k] ^ ks[k];
    }
    if (!decrypt) ghash_update(Y, H, out, len);
    uint8_t L[16];
    uint64_t ab = alen * 8, cb = len * 8;
    for (int k = 0; k < 8; k++) {
        L[k] = (uint8_t)(ab >> (56 - 8 * k));
        L[8 + k] = (uint8_t)(cb >> (56 - 8 * k));
    }
    for (int k = 0; k < 16; k++) Y[k] ^= L[k];
    orc_gf128_mul(Y, H, Y);
    for (int k = 0; k < 16; k++) tag[k] = Y[k] ^ EJ0[k];
}

/* aead.Seal(dst, nonce, plaintext, nil) for cipher.NewGCM(aes.NewCipher(key)) */
ORC_EXPORT void orc_aes256gcm_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                                   uint64_t alen, const uint8_t *p, uint64_t len, uint8_t *c,
                                   uint8_t tag[16]) {
    gcm_core(key, nonce, aad, alen, p, len, c, tag, 0);
}

/* aead.Open: returns 0, or -1 on authentication failure (plaintext not released) */
ORC_EXPORT int orc_aes256gcm_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                                  uint64_t alen, const uint8_t *c, uint64_t len, const uint8_t tag[16],
                                  uint8_t *p) {
    uint8_t t[16];
    uint8_t *tmp = (uint8_t *)malloc(len ? (size_t)len : 1);
    gcm_core(key, nonce, aad, alen, c, len, tmp, t, 1);
    uint8_t d = 0;
    for (int k = 0; k < 16; k++) d |= t[k] ^ tag[k];
    if (d) {
        free(tmp);
        return -1;
    }
    memcpy(p, tmp, (size_t)len);
    free(tmp);
    return 0;
}

/* ------------------------------------------------------------------ */
/* AES-NI + PCLMULQDQ GCM (x86 fast path, same algorithm)              */
/* ------------------------------------------------------------------ */
#define ATTR_NI __attribute__((target("aes,pclmul,sse4.2,ssse3")))

ATTR_NI static inline __m128i bswap128(__m128i x) {
    const __m128i m = _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    return _mm_shuffle_epi8(x, m);
}

/* unreduced 256-bit carry-less product of byte-reflected operands */
ATTR_NI static inline void clmul256(__m128i a, __m128i b, __m128i *lo, __m128i *hi) {
    __m128i t3 = _mm_clmulepi64_si128(a, b, 0x00);
    __m128i t4 = _mm_clmulepi64_si128(a, b, 0x10);
    __m128i t5 = _mm_clmulepi64_si128(a, b, 0x01);
    __m128i t6 = _mm_clmulepi64_si128(a, b, 0x11);
    t4 = _mm_xor_si128(t4, t5);
    t5 = _mm_slli_si128(t4, 8);
    t4 = _mm_srli_si128(t4, 8);
    *lo = _mm_xor_si128(t3, t5);
    *hi = _mm_xor_si128(t6, t4);
}

/* shift the 256-bit product left by one and reduce mod x^128+x^7+x^2+x+1
 * (reflected domain), Intel CLMUL white paper, Algorithm 5 */
ATTR_NI static inline __m128i gf_reduce(__m128i t3, __m128i t6) {
    __m128i t7 = _mm_srli_epi32(t3, 31);
    __m128i t8 = _mm_srli_epi32(t6, 31);
    t3 = _mm_slli_epi32(t3, 1);
    t6 = _mm_slli_epi32(t6, 1);
    __m128i t9 = _mm_srli_si128(t7, 12);
    t8 = _mm_slli_si128(t8, 4);
    t7 = _mm_slli_si128(t7, 4);
    t3 = _mm_or_si128(t3, t7);
    t6 = _mm_or_si128(t6, t8);
    t6 = _mm_or_si128(t6, t9);
    t7 = _mm_slli_epi32(t3, 31);
    t8 = _mm_slli_epi32(t3, 30);
    t9 = _mm_slli_epi32(t3, 25);
    t7 = _mm_xor_si128(t7, t8);
    t7 = _mm_xor_si128(t7, t9);
    t8 = _mm_srli_si128(t7, 4);
    t7 = _mm_slli_si128(t7, 12);
    t3 = _mm_xor_si128(t3, t7);
    __m128i t2 = _mm_srli_epi32(t3, 1);
    __m128i t4 = _mm_srli_epi32(t3, 2);
    __m128i t5 = _mm_srli_epi32(t3, 7);
    t2 = _mm_xor_si128(t2, t4);
    t2 = _mm_xor_si128(t2, t5);
    t2 = _mm_xor_si128(t2, t8);
    t3 = _mm_xor_si128(t3, t2);
    return _mm_xor_si128(t6, t3);
}

ATTR_NI static inline __m128i gfmul_ni(__m128i a, __m128i b) {
    __m128i lo, hi;
    clmul256(a, b, &lo, &hi);
    return gf_reduce(lo, hi);
}

typedef struct {
    __m128i rk[15];
    __m128i hp[8]; /* reflected H^1..H^8 */
    __m128i ej0;
} gcm_ni_ctx;

ATTR_NI static inline __m128i aes_ni_enc(const __m128i *rk, __m128i x) {
    x = _mm_xor_si128(x, rk[0]);
    for (int r = 1; r < 14; r++) x = _mm_aesenc_si128(x, rk[r]);
    return _mm_aesenclast_si128(x, rk[14]);
}

ATTR_NI static void gcm_ni_init(gcm_ni_ctx *g, const uint8_t key[32], const uint8_t nonce[12]) {
    uint8_t rkb[240];
    orc_aes256_expand(key, rkb);
    for (int r = 0; r < 15; r++) g->rk[r] = _mm_loadu_si128((const __m128i *)(rkb + 16 * r));
    __m128i h = aes_ni_enc(g->rk, _mm_setzero_si128());
    g->hp[0] = bswap128(h);
    for (int i = 1; i < 8; i++) g->hp[i] = gfmul_ni(g->hp[i - 1], g->hp[0]);
    uint8_t j0[16];
    memcpy(j0, nonce, 12);
    j0[12] = 0; j0[13] = 0; j0[14] = 0; j0[15] = 1;
    g->ej0 = aes_ni_enc(g->rk, _mm_loadu_si128((const __m128i *)j0));
}

/* GHASH over n bytes, 8 blocks per aggregated reduction */
ATTR_NI static __m128i ghash_ni(const gcm_ni_ctx *g, __m128i y, const uint8_t *p, uint64_t n) {
    while (n >= 128) {
        __m128i lo = _mm_setzero_si128(), hi = _mm_setzero_si128();
        for (int i = 0; i < 8; i++) {
            __m128i x = bswap128(_mm_loadu_si128((const __m128i *)(p + 16 * i)));
            if (i == 0) x = _mm_xor_si128(x, y);
            __m128i l, h;
            clmul256(x, g->hp[7 - i], &l, &h);
            lo = _mm_xor_si128(lo, l);
            hi = _mm_xor_si128(hi, h);
        }
        y = gf_reduce(lo, hi);
        p += 128;
        n -= 128;
    }
    while (n) {
        uint8_t blk[16] = {0};
        uint64_t c = n < 16 ? n : 16;
        memcpy(blk, p, c);
        y = gfmul_ni(_mm_xor_si128(y, bswap128(_mm_loadu_si128((const __m128i *)blk))), g->hp[0]);
        p += c;
        n -= c;
    }
    return y;
}

ATTR_NI static void ctr_ni(const gcm_ni_ctx *g, const uint8_t nonce[12], const uint8_t *in, uint8_t *out,
                           uint64_t len) {
    uint32_t n0, n1, n2;
    memcpy(&n0, nonce, 4);
    memcpy(&n1, nonce + 4, 4);
    memcpy(&n2, nonce + 8, 4);
    uint32_t cnt = 2;
    uint64_t off = 0;
    while (len - off >= 128) {
        __m128i x[8];
        for (int i = 0; i < 8; i++) {
            x[i] = _mm_setr_epi32((int)n0, (int)n1, (int)n2, (int)__builtin_bswap32(cnt + i));
            x[i] = _mm_xor_si128(x[i], g->rk[0]);
        }
        for (int r = 1; r < 14; r++)
            for (int i = 0; i < 8; i++) x[i] = _mm_aesenc_si128(x[i], g->rk[r]);
        for (int i = 0; i < 8; i++) {
            x[i] = _mm_aesenclast_si128(x[i], g->rk[14]);
            __m128i d = _mm_loadu_si128((const __m128i *)(in + off + 16 * i));
            _mm_storeu_si128((__m128i *)(out + off + 16 * i), _mm_xor_si128(d, x[i]));
        }
        cnt += 8;
        off += 128;
    }
    while (off < len) {
        __m128i ks = aes_ni_enc(g->rk, _mm_setr_epi32((int)n0, (int)n1, (int)n2, (int)__builtin_bswap32(cnt)));
        uint8_t kb[16];
        _mm_storeu_si128((__m128i *)kb, ks);
        uint64_t c = len - off < 16 ? len - off : 16;
        for (uint64_t k = 0; k < c; k++) out[off + k] = in[off + k] ^ kb[k];
        cnt++;
        off += 16;
    }
}

ATTR_NI static void gcm_ni_tag(const gcm_ni_ctx *g, __m128i y, uint64_t alen, uint64_t len, uint8_t tag[16]) {
    uint8_t L[16];
    uint64_t ab = alen * 8, cb = len * 8;
    for (int k = 0; k < 8; k++) {
        L[k] = (uint8_t)(ab >> (56 - 8 * k));
        L[8 + k] = (uint8_t)(cb >> (56 - 8 * k));
    }
    y = gfmul_ni(_mm_xor_si128(y, bswap128(_mm_loadu_si128((const __m128i *)L))), g->hp[0]);
    _mm_storeu_si128((__m128i *)tag, _mm_xor_si128(bswap128(y), g->ej0));
}

ATTR_NI ORC_EXPORT void orc_aes256gcm_seal_ni(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *p,
                                             uint64_t len, uint8_t *c, uint8_t tag[16]) {
    gcm_ni_ctx g;
    gcm_ni_init(&g, key, nonce);
    ctr_ni(&g, nonce, p, c, len);
    __m128i y = ghash_ni(&g, _mm_setzero_si128(), c, len);
    gcm_ni_tag(&g, y, 0, len, tag);
}

ATTR_NI ORC_EXPORT int orc_aes256gcm_open_ni(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *c,
                                            uint64_t len, const uint8_t tag[16], uint8_t *p) {
    gcm_ni_ctx g;
    uint8_t t[16];
    gcm_ni_init(&g, key, nonce);
    __m128i y = ghash_ni(&g, _mm_setzero_si128(), c, len);
    gcm_ni_tag(&g, y, 0, len, t);
    uint8_t d = 0;
    for (int k = 0; k < 16; k++) d |= t[k] ^ tag[k];
    if (d) return -1;
    ctr_ni(&g, nonce, c, p, len);
    return 0;
}

/* ------------------------------------------------------------------ */
/* ChaCha20 + Poly1305 (RFC 8439)                                      */
/* ------------------------------------------------------------------ */
#define ROTL32(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QR(a, b, c, d)                 \
    a += b; d ^= a; d = ROTL32(d, 16); \
    c += d; b ^= c; b = ROTL32(b, 12); \
    a += b; d ^= a; d = ROTL32(d, 8);  \
    c += d; b ^= c; b = ROTL32(b, 7);

static inline uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32); }

ORC_EXPORT void orc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                                   uint8_t out[64]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865; s[1] = 0x3320646e; s[2] = 0x79622d32; s[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) s[4 + i] = le32(key + 4 * i);
    s[12] = counter;
    for (int i = 0; i < 3; i++) s[13 + i] = le32(nonce + 4 * i);
    memcpy(x, s, sizeof(s));
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) {
        uint32_t v = x[i] + s[i];
        out[4 * i] = (uint8_t)v; out[4 * i + 1] = (uint8_t)(v >> 8);
        out[4 * i + 2] = (uint8_t)(v >> 16); out[4 * i + 3] = (uint8_t)(v >> 24);
    }
}

/* Poly1305 with 44/44/42-bit limbs and 128-bit products */
typedef unsigned __int128 u128;
typedef struct {
    uint64_t r0, r1, r2, s1, s2, h0, h1, h2, pad0, pad1;
} poly_st;

static void poly_init(poly_st *st, const uint8_t key[32]) {
    uint64_t t0 = le64(key), t1 = le64(key + 8);
    st->r0 = t0 & 0xffc0fffffffULL;
    st->r1 = ((t0 >> 44) | (t1 << 20)) & 0xfffffc0ffffULL;
    st->r2 = (t1 >> 24) & 0x00ffffffc0fULL;
    st->s1 = st->r1 * (5 << 2);
    st->s2 = st->r2 * (5 << 2);
    st->h0 = st->h1 = st->h2 = 0;
    st->pad0 = le64(key + 16);
    st->pad1 = le64(key + 24);
}

static void poly_blocks(poly_st *st, const uint8_t *m, uint64_t n, uint64_t hibit) {
    const uint64_t M44 = 0xfffffffffffULL, M42 = 0x3ffffffffffULL;
    uint64_t r0 = st->r0, r1 = st->r1, r2 = st->r2, s1 = st->s1, s2 = st->s2;
    uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2;
    while (n >= 16) {
        uint64_t t0 = le64(m), t1 = le64(m + 8);
        h0 += t0 & M44;
        h1 += ((t0 >> 44) | (t1 << 20)) & M44;
        h2 += ((t1 >> 24) & M42) | hibit;
        u128 d0 = (u128)h0 * r0 + (u128)h1 * s2 + (u128)h2 * s1;
        u128 d1 = (u128)h0 * r1 + (u128)h1 * r0 + (u128)h2 * s2;
        u128 d2 = (u128)h0 * r2 + (u128)h1 * r1 + (u128)h2 * r0;
        uint64_t c = (uint64_t)(d0 >> 44); h0 = (uint64_t)d0 & M44;
        d1 += c; c = (uint64_t)(d1 >> 44); h1 = (uint64_t)d1 & M44;
        d2 += c; c = (uint64_t)(d2 >> 42); h2 = (uint64_t)d2 & M42;
        h0 += c * 5; c = h0 >> 44; h0 &= M44;
        h1 += c;
        m += 16;
        n -= 16;
    }
    st->h0 = h0; st->h1 = h1; st->h2 = h2;
}

static void poly_finish(poly_st *st, uint8_t tag[16]) {
    const uint64_t M44 = 0xfffffffffffULL, M42 = 0x3ffffffffffULL;
    uint64_t h0 = st->h0, h1 = st->h1, h2 = st->h2, c;
    c = h1 >> 44; h1 &= M44;
    h2 += c; c = h2 >> 42; h2 &= M42;
    h0 += c * 5; c = h0 >> 44; h0 &= M44;
    h1 += c; c = h1 >> 44; h1 &= M44;
    h2 += c; c = h2 >> 42; h2 &= M42;
    h0 += c * 5; c = h0 >> 44; h0 &= M44;
    h1 += c;
    /* g = h + -p */
    uint64_t g0 = h0 + 5; c = g0 >> 44; g0 &= M44;
    uint64_t g1 = h1 + c; c = g1 >> 44; g1 &= M44;
    uint64_t g2 = h2 + c - (1ULL << 42);
    c = (g2 >> 63) - 1; /* all ones if h >= p */
    g0 &= c; g1 &= c; g2 &= c;
    c = ~c;
    h0 = (h0 & c) | g0; h1 = (h1 & c) | g1; h2 = (h2 & c) | g2;
    /* h = (h + pad) mod 2^128 */
    uint64_t t0 = st->pad0, t1 = st->pad1;
    h0 += t0 & M44; c = h0 >> 44; h0 &= M44;
    h1 += (((t0 >> 44) | (t1 << 20)) & M44) + c; c = h1 >> 44; h1 &= M44;
    h2 += ((t1 >> 24) & M42) + c; h2 &= M42;
    uint64_t o0 = h0 | (h1 << 44), o1 = (h1 >> 20) | (h2 << 24);
    memcpy(tag, &o0, 8);
    memcpy(tag + 8, &o1, 8);
}

ORC_EXPORT void orc_poly1305(const uint8_t key[32], const uint8_t *m, uint64_t n, uint8_t tag[16]) {
    poly_st st;
    poly_init(&st, key);
    poly_blocks(&st, m, n & ~15ULL, 1ULL << 40);
    if (n & 15) {
        uint8_t blk[16] = {0};
        memcpy(blk, m + (n & ~15ULL), n & 15);
        blk[n & 15] = 1;
        poly_blocks(&st, blk, 16, 0);
    }
    poly_finish(&st, tag);
}

static void chacha_xor(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *in, uint8_t *out,
                       uint64_t len) {
    uint32_t ctr = 1;
    uint8_t ks[64];
    for (uint64_t off = 0; off < len; off += 64, ctr++) {
        orc_chacha20_block(key, ctr, nonce, ks);
        uint64_t c = len - off < 64 ? len - off : 64;
        for (uint64_t k = 0; k < c; k++) out[off + k] = in[off + k] ^ ks[k];
    }
}

static void cp_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, uint64_t alen,
                   const uint8_t *c, uint64_t len, uint8_t tag[16]) {
    uint8_t blk0[64];
    orc_chacha20_block(key, 0, nonce, blk0);
    poly_st st;
    poly_init(&st, blk0);
    uint8_t pad[16] = {0};
    poly_blocks(&st, aad, alen & ~15ULL, 1ULL << 40);
    if (alen & 15) {
        memset(pad, 0, 16);
        memcpy(pad, aad + (alen & ~15ULL), alen & 15);
        poly_blocks(&st, pad, 16, 1ULL << 40);
    }
    poly_blocks(&st, c, len & ~15ULL, 1ULL << 40);
    if (len & 15) {
        memset(pad, 0, 16);
        memcpy(pad, c + (len & ~15ULL), len & 15);
        poly_blocks(&st, pad, 16, 1ULL << 40);
    }
    uint8_t lens[16];
    memcpy(lens, &alen, 8);
    memcpy(lens + 8, &len, 8);
    poly_blocks(&st, lens, 16, 1ULL << 40);
    poly_finish(&st, tag);
}

ORC_EXPORT void orc_chacha20poly1305_seal(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                                          uint64_t alen, const uint8_t *p, uint64_t len, uint8_t *c,
                                          uint8_t tag[16]) {
    chacha_xor(key, nonce, p, c, len);
    cp_tag(key, nonce, aad, alen, c, len, tag);
}

ORC_EXPORT int orc_chacha20poly1305_open(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad,
                                         uint64_t alen, const uint8_t *c, uint64_t len, const uint8_t tag[16],
                                         uint8_t *p) {
    uint8_t t[16];
    cp_tag(key, nonce, aad, alen, c, len, t);
    uint8_t d = 0;
    for (int k = 0; k < 16; k++) d |= t[k] ^ tag[k];
    if (d) return -1;
    chacha_xor(key, nonce, c, p, len);
    return 0;
}

/* ------------------------------------------------------------------ */
/* dataEncryptor object format (encrypt.go:164-216)                    */
/* ------------------------------------------------------------------ */
enum { ALGO_AES256GCM = 0, ALGO_CHACHA20P1305 = 1 };

/* Encrypt with an already-wrapped key: header BE16(klen) | nlen | wrapped | nonce,
 * then Seal in place after the header (encrypt.go:182-193).  Returns object size. */
ORC_EXPORT int64_t orc_data_encrypt(int algo, const uint8_t key[32], const uint8_t nonce[12],
                                    const uint8_t *wrapped, int wlen, const uint8_t *p, uint64_t len,
                                    uint8_t *out) {
    out[0] = (uint8_t)(wlen >> 8);
    out[1] = (uint8_t)(wlen & 0xff);
    out[2] = 12;
    memcpy(out + 3, wrapped, (size_t)wlen);
    memcpy(out + 3 + wlen, nonce, 12);
    uint8_t *c = out + 3 + wlen + 12;
    if (algo == ALGO_AES256GCM)
        orc_aes256gcm_seal(key, nonce, NULL, 0, p, len, c, c + len);
    else
        orc_chacha20poly1305_seal(key, nonce, NULL, 0, p, len, c, c + len);
    return 3 + wlen + 12 + (int64_t)len + 16;
}

/* Decrypt: parse header (encrypt.go:197-205); caller supplies the unwrapped key.
 * Returns plaintext length, -1 "misformed ciphertext", -2 AEAD open failure. */
ORC_EXPORT int64_t orc_data_decrypt(int algo, const uint8_t key[32], const uint8_t *obj, int64_t olen,
                                    uint8_t *out) {
    int klen = ((int)obj[0] << 8) + obj[1];
    int nlen = obj[2];
    if (3 + klen + nlen >= olen) return -1;
    if (nlen != 12) return -2; /* aead.Open panics on a bad nonce size; recovered as an error upstream */
    const uint8_t *nonce = obj + 3 + klen;
    const uint8_t *c = nonce + nlen;
    int64_t clen = olen - 3 - klen - nlen;
    if (clen < 16) return -2;
    int64_t len = clen - 16;
    int rc = algo == ALGO_AES256GCM ? orc_aes256gcm_open(key, nonce, NULL, 0, c, (uint64_t)len, c + len, out)
                                    : orc_chacha20poly1305_open(key, nonce, NULL, 0, c, (uint64_t)len, c + len, out);
    return rc ? -2 : len;
}

/* ------------------------------------------------------------------ */
/* CPU baseline: seal + checksum(full) of synthetic blocks, N threads  */
/* (the per-block work of cached_store.go upload: checksum() on the    */
/*  plaintext, then dataEncryptor.Encrypt's aead.Seal)                 */
/* ------------------------------------------------------------------ */
typedef struct {
    int algo;
    uint64_t seed, blen;
    uint64_t b0, b1;
    uint8_t *pbuf, *cbuf, *crc;
    uint32_t digest;
} bench_job;

static void *bench_worker(void *arg) {
    bench_job *j = (bench_job *)arg;
    uint32_t dg = 0;
    for (uint64_t b = j->b0; b < j->b1; b++) {
        uint8_t key[32], nonce[12], tag[16];
        orc_gen_key(j->seed, b, key, nonce);
        uint8_t *p = j->pbuf + (b - j->b0) * j->blen;
        orc_checksum(p, (int64_t)j->blen, j->crc, 1);
        if (j->algo == ALGO_AES256GCM)
            orc_aes256gcm_seal_ni(key, nonce, p, j->blen, j->cbuf, tag);
        else
            orc_chacha20poly1305_seal(key, nonce, NULL, 0, p, j->blen, j->cbuf, tag);
        dg ^= le32(tag) ^ le32(j->crc);
    }
    j->digest = dg;
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* Generates nblocks synthetic blocks (untimed), then times seal+checksum
 * over them with nthreads threads.  Returns wall seconds. */
ORC_EXPORT double orc_bench_seal_crc(int algo, int nthreads, uint64_t nblocks, uint64_t blen, uint64_t seed,
                                     uint32_t *digest) {
    if (nthreads < 1) nthreads = 1;
    bench_job *jobs = (bench_job *)calloc((size_t)nthreads, sizeof(bench_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t per = (nblocks + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        jobs[t].algo = algo;
        jobs[t].seed = seed;
        jobs[t].blen = blen;
        jobs[t].b0 = (uint64_t)t * per < nblocks ? (uint64_t)t * per : nblocks;
        jobs[t].b1 = jobs[t].b0 + per < nblocks ? jobs[t].b0 + per : nblocks;
        uint64_t nb = jobs[t].b1 - jobs[t].b0;
        jobs[t].pbuf = (uint8_t *)malloc(nb ? nb * blen : 1);
        jobs[t].cbuf = (uint8_t *)malloc(blen + 16);
        jobs[t].crc = (uint8_t *)malloc((size_t)orc_checksum_len((int64_t)blen));
        for (uint64_t b = jobs[t].b0; b < jobs[t].b1; b++)
            orc_gen_block(seed, b, jobs[t].pbuf + (b - jobs[t].b0) * blen, blen);
    }
    double t0 = now_s();
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
    uint32_t dg = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        dg ^= jobs[t].digest;
    }
    double el = now_s() - t0;
    for (int t = 0; t < nthreads; t++) {
        free(jobs[t].pbuf);
        free(jobs[t].cbuf);
        free(jobs[t].crc);
    }
    free(jobs);
    free(th);
    if (digest) *digest = dg;
    return el;
}

/* ------------------------------------------------------------------ */
/* CPU baseline through OpenSSL EVP (libcrypto.so.3, dlopen'ed): the   */
/* strongest AEAD the host has (AES-NI/VAES + (V)PCLMULQDQ stitched    */
/* GCM, SIMD ChaCha20-Poly1305), plus the 3-stream SSE4.2 checksum().  */
/* BASELINE.md §4 names this as the preferred CPU path.  Returns wall  */
/* seconds, or -1 when libcrypto is not loadable.                      */
/* ------------------------------------------------------------------ */
typedef void *(*evp_ctx_new_t)(void);
typedef void (*evp_ctx_free_t)(void *);
typedef const void *(*evp_cipher_t)(void);
typedef int (*evp_init_t)(void *, const void *, void *, const uint8_t *, const uint8_t *);
typedef int (*evp_update_t)(void *, uint8_t *, int *, const uint8_t *, int);
typedef int (*evp_final_t)(void *, uint8_t *, int *);
typedef int (*evp_ctrl_t)(void *, int, int, void *);

static struct {
    int ok;
    evp_ctx_new_t ctx_new;
    evp_ctx_free_t ctx_free;
    evp_cipher_t gcm, chacha;
    evp_init_t init;
    evp_update_t update;
    evp_final_t final;
    evp_ctrl_t ctrl;
} evp;

static int evp_load(void) {
    if (evp.ok) return evp.ok > 0;
    void *h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        evp.ok = -1;
        return 0;
    }
    evp.ctx_new = (evp_ctx_new_t)dlsym(h, "EVP_CIPHER_CTX_new");
    evp.ctx_free = (evp_ctx_free_t)dlsym(h, "EVP_CIPHER_CTX_free");
    evp.gcm = (evp_cipher_t)dlsym(h, "EVP_aes_256_gcm");
    evp.chacha = (evp_cipher_t)dlsym(h, "EVP_chacha20_poly1305");
    evp.init = (evp_init_t)dlsym(h, "EVP_EncryptInit_ex");
    evp.update = (evp_update_t)dlsym(h, "EVP_EncryptUpdate");
    evp.final = (evp_final_t)dlsym(h, "EVP_EncryptFinal_ex");
    evp.ctrl = (evp_ctrl_t)dlsym(h, "EVP_CIPHER_CTX_ctrl");
    evp.ok = (evp.ctx_new && evp.ctx_free && evp.gcm && evp.chacha && evp.init && evp.update && evp.final &&
              evp.ctrl) ? 1 : -1;
    return evp.ok > 0;
}

/* one Seal through EVP: 0 ok */
static int evp_seal(void *ctx, int algo, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *p,
                    uint64_t len, uint8_t *c, uint8_t tag[16]) {
    if (evp.init(ctx, algo == ALGO_AES256GCM ? evp.gcm() : evp.chacha(), NULL, key, nonce) != 1) return -1;
    uint64_t off = 0;
    while (off < len) {
        int chunk = len - off > (1u << 30) ? (1 << 30) : (int)(len - off), out = 0;
        if (evp.update(ctx, c + off, &out, p + off, chunk) != 1) return -1;
        off += (uint64_t)chunk;
    }
    int fin = 0;
    if (evp.final(ctx, c + len, &fin) != 1) return -1;
    return evp.ctrl(ctx, 0x10 /* EVP_CTRL_AEAD_GET_TAG */, 16, tag) == 1 ? 0 : -1;
}

/* exported for the tests: the EVP Seal must equal the oracle's */
ORC_EXPORT int orc_evp_seal(int algo, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *p,
                            uint64_t len, uint8_t *c, uint8_t tag[16]) {
    if (!evp_load()) return -1;
    void *ctx = evp.ctx_new();
    int rc = evp_seal(ctx, algo, key, nonce, p, len, c, tag);
    evp.ctx_free(ctx);
    return rc;
}

typedef struct {
    bench_job j;
    int rc;
} evp_job;

static void *evp_worker(void *arg) {
    evp_job *e = (evp_job *)arg;
    bench_job *j = &e->j;
    void *ctx = evp.ctx_new();
    uint32_t dg = 0;
    e->rc = 0;
    for (uint64_t b = j->b0; b < j->b1; b++) {
        uint8_t key[32], nonce[12], tag[16];
        orc_gen_key(j->seed, b, key, nonce);
        uint8_t *p = j->pbuf + (b - j->b0) * j->blen;
        orc_checksum(p, (int64_t)j->blen, j->crc, 1);
        if (evp_seal(ctx, j->algo, key, nonce, p, j->blen, j->cbuf, tag)) e->rc = -1;
        dg ^= le32(tag) ^ le32(j->crc);
    }
    evp.ctx_free(ctx);
    j->digest = dg;
    return NULL;
}

/* as orc_bench_seal_crc, with the AEAD from OpenSSL EVP; same digest */
ORC_EXPORT double orc_bench_seal_crc_evp(int algo, int nthreads, uint64_t nblocks, uint64_t blen, uint64_t seed,
                                         uint32_t *digest) {
    if (!evp_load()) return -1.0;
    if (nthreads < 1) nthreads = 1;
    evp_job *jobs = (evp_job *)calloc((size_t)nthreads, sizeof(evp_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t per = (nblocks + nthreads - 1) / nthreads;
    for (int t = 0; t < nthreads; t++) {
        bench_job *j = &jobs[t].j;
        j->algo = algo;
        j->seed = seed;
        j->blen = blen;
        j->b0 = (uint64_t)t * per < nblocks ? (uint64_t)t * per : nblocks;
        j->b1 = j->b0 + per < nblocks ? j->b0 + per : nblocks;
        uint64_t nb = j->b1 - j->b0;
        j->pbuf = (uint8_t *)malloc(nb ? nb * blen : 1);
        j->cbuf = (uint8_t *)malloc(blen + 16);
        j->crc = (uint8_t *)malloc((size_t)orc_checksum_len((int64_t)blen));
        for (uint64_t b = j->b0; b < j->b1; b++) orc_gen_block(seed, b, j->pbuf + (b - j->b0) * blen, blen);
    }
    double t0 = now_s();
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, evp_worker, &jobs[t]);
    uint32_t dg = 0;
    int rc = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        dg ^= jobs[t].j.digest;
        rc |= jobs[t].rc;
    }
    double el = now_s() - t0;
    for (int t = 0; t < nthreads; t++) {
        free(jobs[t].j.pbuf);
        free(jobs[t].j.cbuf);
        free(jobs[t].j.crc);
    }
    free(jobs);
    free(th);
    if (digest) *digest = dg;
    return rc ? -1.0 : el;
}

/* ------------------------------------------------------------------ */
/* CPU baselines for every BASELINE config (bench.py cpu_baseline):    */
/*   mode 0  seal: checksum(p) + EVP Seal         (configs[1], [2], [4]) */
/*   mode 1  open: EVP Open (tag checked) + checksum(p) compared with   */
/*           the stored CRCs, as cacheFile.ReadAt's verify does         */
/*           (encrypt.go:196-216 + disk_cache.go:1315-1327; configs[3])  */
/*   mode 2  CRC verify only (cache hit, disk_cache.go:1255-1329)        */
/*   mode 3  dataEncryptor.Encrypt + checksum(p): the object header (a   */
/*           256-B wrapped key, the nonce) built in the output buffer,   */
/*           EVP Seal into it at offset 271 (encrypt.go:182-193),        */
/*           checksum() of the plaintext for the staged cache file       */
/*   mode 4  dataEncryptor.Decrypt + checksum(p): header parsed, EVP     */
/*           Open from offset 271 (encrypt.go:196-215), checksum() of    */
/*           the plaintext for the cache file (cached_store.go:745)      */
/* Block b has lens[b] bytes (lens NULL: blen each; configs[4] ragged).  */
/* Inputs (and, for open, the sealed images) are made before the clock */
/* starts.  Returns wall seconds, -1 without libcrypto (modes 0/1), -2  */
/* if any block failed to open or verify.                               */
/* ------------------------------------------------------------------ */
typedef int (*evp_dinit_t)(void *, const void *, void *, const uint8_t *, const uint8_t *);
typedef int (*evp_dupdate_t)(void *, uint8_t *, int *, const uint8_t *, int);
typedef int (*evp_dfinal_t)(void *, uint8_t *, int *);
static evp_dinit_t evp_dinit;
static evp_dupdate_t evp_dupdate;
static evp_dfinal_t evp_dfinal;

static int evp_load_open(void) {
    if (!evp_load()) return 0;
    if (!evp_dinit) {
        void *h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
        if (!h) return 0;
        evp_dinit = (evp_dinit_t)dlsym(h, "EVP_DecryptInit_ex");
        evp_dupdate = (evp_dupdate_t)dlsym(h, "EVP_DecryptUpdate");
        evp_dfinal = (evp_dfinal_t)dlsym(h, "EVP_DecryptFinal_ex");
    }
    return evp_dinit && evp_dupdate && evp_dfinal;
}

/* one Open through EVP: 0 ok, -1 tag mismatch or error */
static int evp_open(void *ctx, int algo, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *c,
                    uint64_t len, const uint8_t tag[16], uint8_t *p) {
    if (evp_dinit(ctx, algo == ALGO_AES256GCM ? evp.gcm() : evp.chacha(), NULL, key, nonce) != 1) return -1;
    uint64_t off = 0;
    while (off < len) {
        int chunk = len - off > (1u << 30) ? (1 << 30) : (int)(len - off), out = 0;
        if (evp_dupdate(ctx, p + off, &out, c + off, chunk) != 1) return -1;
        off += (uint64_t)chunk;
    }
    if (evp.ctrl(ctx, 0x11 /* EVP_CTRL_AEAD_SET_TAG */, 16, (void *)tag) != 1) return -1;
    int fin = 0;
    return evp_dfinal(ctx, p + len, &fin) == 1 ? 0 : -1;
}

typedef struct {
    int algo, mode;
    uint64_t seed, b0, b1, maxlen;
    const uint64_t *lens;
    uint8_t *in, *work, *tags, *crcs;  /* per block: maxlen bytes of input, 16-B tag, CRC array */
    uint64_t crcstride;
    uint32_t digest;
    int bad;
} base_job;

static uint64_t base_len(const base_job *j, uint64_t b) { return j->lens ? j->lens[b] : j->maxlen; }
/* bytes per block of the input array: the object (header, C, tag) for mode 4 */
static uint64_t base_stride(const base_job *j) { return j->maxlen + (j->mode == 4 ? 287 : 0); }

static void *base_worker(void *arg) {
    base_job *j = (base_job *)arg;
    void *ctx = j->mode == 2 ? NULL : evp.ctx_new();
    uint8_t *mycrc = (uint8_t *)malloc((size_t)j->crcstride);
    uint32_t dg = 0;
    for (uint64_t b = j->b0; b < j->b1; b++) {
        const uint64_t n = base_len(j, b), k = b - j->b0;
        uint8_t key[32], nonce[12], tag[16];
        orc_gen_key(j->seed, b, key, nonce);
        uint8_t *in = j->in + k * base_stride(j);
        if (j->mode == 0) {
            orc_checksum(in, (int64_t)n, mycrc, 1);
            if (evp_seal(ctx, j->algo, key, nonce, in, n, j->work, tag)) j->bad = 1;
            dg ^= le32(tag) ^ le32(mycrc);
        } else if (j->mode == 1) {
            if (evp_open(ctx, j->algo, key, nonce, in, n, j->tags + 16 * k, j->work)) j->bad = 1;
            const int64_t cl = orc_checksum(j->work, (int64_t)n, mycrc, 1);
            if (memcmp(mycrc, j->crcs + k * j->crcstride, (size_t)cl)) j->bad = 1;
            dg ^= le32(mycrc);
        } else if (j->mode == 2) {
            const int64_t cl = orc_checksum(in, (int64_t)n, mycrc, 1);
            if (memcmp(mycrc, j->crcs + k * j->crcstride, (size_t)cl)) j->bad = 1;
            dg ^= le32(mycrc);
        } else if (j->mode == 3) {
            uint8_t *o = j->work;
            o[0] = 1;  /* BE16(256) */
            o[1] = 0;
            o[2] = 12;
            memcpy(o + 3, j->tags, 256);  /* the wrapped key (any 256 bytes) */
            memcpy(o + 259, nonce, 12);
            if (evp_seal(ctx, j->algo, key, nonce, in, n, o + 271, o + 271 + n)) j->bad = 1;
            orc_checksum(in, (int64_t)n, mycrc, 1);
            dg ^= le32(o + 271 + n) ^ le32(mycrc);
        } else {
            const uint8_t *o = in;
            const uint64_t kl = ((uint64_t)o[0] << 8) | o[1], hl = 3 + kl + o[2];
            if (evp_open(ctx, j->algo, key, o + 3 + kl, o + hl, n, o + hl + n, j->work)) j->bad = 1;
            const int64_t cl = orc_checksum(j->work, (int64_t)n, mycrc, 1);
            if (memcmp(mycrc, j->crcs + k * j->crcstride, (size_t)cl)) j->bad = 1;
            dg ^= le32(mycrc);
        }
    }
    if (ctx) evp.ctx_free(ctx);
    free(mycrc);
    j->digest = dg;
    return NULL;
}

ORC_EXPORT double orc_bench_baseline(int algo, int mode, int nthreads, uint64_t nblocks, const uint64_t *lens,
                                     uint64_t blen, uint64_t seed, uint32_t *digest) {
    if (mode < 0 || mode > 4) return -3.0;
    if (mode != 2 && !evp_load_open()) return -1.0;
    if (nthreads < 1) nthreads = 1;
    uint64_t maxlen = blen;
    if (lens)
        for (uint64_t b = 0; b < nblocks; b++) maxlen = lens[b] > maxlen ? lens[b] : maxlen;
    const uint64_t crcstride = (uint64_t)orc_checksum_len((int64_t)maxlen);
    base_job *jobs = (base_job *)calloc((size_t)nthreads, sizeof(base_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    const uint64_t per = (nblocks + nthreads - 1) / nthreads;
    void *sctx = mode == 1 || mode == 4 ? evp.ctx_new() : NULL;
    for (int t = 0; t < nthreads; t++) {
        base_job *j = &jobs[t];
        j->algo = algo;
        j->mode = mode;
        j->seed = seed;
        j->lens = lens;
        j->maxlen = maxlen;
        j->crcstride = crcstride;
        j->b0 = (uint64_t)t * per < nblocks ? (uint64_t)t * per : nblocks;
        j->b1 = j->b0 + per < nblocks ? j->b0 + per : nblocks;
        const uint64_t nb = j->b1 - j->b0, stride = base_stride(j);
        j->in = (uint8_t *)malloc(nb ? nb * stride : 1);
        j->work = (uint8_t *)malloc(maxlen + 16 + 271);
        j->tags = (uint8_t *)malloc(nb ? 16 * nb + 256 : 256);
        j->crcs = (uint8_t *)malloc(nb ? nb * crcstride : 1);
        for (int i = 0; i < 256; i++) j->tags[i] = (uint8_t)(i * 37 + 11);
        for (uint64_t b = j->b0; b < j->b1; b++) {
            const uint64_t n = base_len(j, b), k = b - j->b0;
            uint8_t *in = j->in + k * stride;
            orc_gen_block(seed, b, in, n);
            orc_checksum(in, (int64_t)n, j->crcs + k * crcstride, 1);  /* the cache file's stored CRCs */
            if (mode == 1) {  /* stored object: seal it, keep ciphertext and tag */
                uint8_t key[32], nonce[12];
                orc_gen_key(seed, b, key, nonce);
                if (evp_seal(sctx, algo, key, nonce, in, n, j->work, j->tags + 16 * k)) j->bad = 1;
                memcpy(in, j->work, (size_t)n);
            } else if (mode == 4) {  /* the encrypted object: header, C, tag */
                uint8_t key[32], nonce[12];
                orc_gen_key(seed, b, key, nonce);
                if (evp_seal(sctx, algo, key, nonce, in, n, j->work + 271, j->work + 271 + n)) j->bad = 1;
                j->work[0] = 1;
                j->work[1] = 0;
                j->work[2] = 12;
                memset(j->work + 3, 0x5A, 256);
                memcpy(j->work + 259, nonce, 12);
                memcpy(in, j->work, (size_t)(n + 287));
            }
        }
    }
    if (sctx) evp.ctx_free(sctx);
    double t0 = now_s();
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, base_worker, &jobs[t]);
    uint32_t dg = 0;
    int bad = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        dg ^= jobs[t].digest;
        bad |= jobs[t].bad;
    }
    double el = now_s() - t0;
    for (int t = 0; t < nthreads; t++) {
        free(jobs[t].in);
        free(jobs[t].work);
        free(jobs[t].tags);
        free(jobs[t].crcs);
    }
    free(jobs);
    free(th);
    if (digest) *digest = dg;
    return bad ? -2.0 : el;
}

/* ------------------------------------------------------------------ */
/* CPU baseline of cacheFile.ReadAt at a checksum level (configs[4],   */
/* bench.py --mode agg --agg-op readat): nblocks cache-file images     */
/* (block b: lens[b] synthetic bytes, then checksum(), made before the */
/* clock starts); read r takes blk[r]'s image at (off[r], size[r]).    */
/* nthreads threads split the reads and run them reps times, through   */
/* cache_readat with the 3-stream SSE4.2 CRC.  Returns wall seconds,   */
/* -2 if any read failed.  *bytes: the bytes the reads returned.       */
/* ------------------------------------------------------------------ */
typedef struct {
    const uint8_t *const *imgs;
    const uint64_t *lens, *off, *size;
    const uint32_t *blk;
    uint64_t r0, r1, reps, maxsize;
    int level, bad;
    uint64_t bytes;
} readat_job;

static void *readat_worker(void *arg) {
    readat_job *j = (readat_job *)arg;
    uint8_t *out = (uint8_t *)malloc(j->maxsize ? j->maxsize : 1);
    for (uint64_t rep = 0; rep < j->reps; rep++)
        for (uint64_t r = j->r0; r < j->r1; r++) {
            const uint64_t b = j->blk[r], len = j->lens[b];
            int64_t n = 0, bad_seg = -1;
            uint32_t got = 0, ex = 0;
            const int rc = cache_readat(j->imgs[b], (int64_t)(len + orc_checksum_len((int64_t)len)), (int64_t)len,
                                        j->level, (int64_t)j->off[r], (int64_t)j->size[r], out, &n, &got, &ex,
                                        &bad_seg, 1);
            if (rc) j->bad = 1;
            j->bytes += (uint64_t)n;
        }
    free(out);
    return NULL;
}

ORC_EXPORT double orc_bench_readat(int nthreads, int level, uint64_t nblocks, const uint64_t *lens, uint64_t seed,
                                   uint64_t nreads, const uint32_t *blk, const uint64_t *off, const uint64_t *size,
                                   uint64_t reps, uint64_t *bytes) {
    if (nthreads < 1) nthreads = 1;
    uint8_t **imgs = (uint8_t **)calloc((size_t)(nblocks ? nblocks : 1), sizeof(uint8_t *));
    for (uint64_t b = 0; b < nblocks; b++) {
        const uint64_t n = lens[b];
        imgs[b] = (uint8_t *)malloc((size_t)(n + orc_checksum_len((int64_t)n)));
        orc_gen_block(seed, b, imgs[b], n);
        orc_checksum(imgs[b], (int64_t)n, imgs[b] + n, 1);
    }
    uint64_t maxsize = 0;
    for (uint64_t r = 0; r < nreads; r++) maxsize = size[r] > maxsize ? size[r] : maxsize;
    readat_job *jobs = (readat_job *)calloc((size_t)nthreads, sizeof(readat_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    const uint64_t per = (nreads + nthreads - 1) / nthreads;
    double t0 = now_s();
    for (int t = 0; t < nthreads; t++) {
        readat_job *j = &jobs[t];
        j->imgs = (const uint8_t *const *)imgs;
        j->lens = lens;
        j->off = off;
        j->size = size;
        j->blk = blk;
        j->level = level;
        j->reps = reps;
        j->maxsize = maxsize;
        j->r0 = (uint64_t)t * per < nreads ? (uint64_t)t * per : nreads;
        j->r1 = j->r0 + per < nreads ? j->r0 + per : nreads;
        pthread_create(&th[t], NULL, readat_worker, j);
    }
    int bad = 0;
    uint64_t tot = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        bad |= jobs[t].bad;
        tot += jobs[t].bytes;
    }
    double el = now_s() - t0;
    for (uint64_t b = 0; b < nblocks; b++) free(imgs[b]);
    free(imgs);
    free(jobs);
    free(th);
    if (bytes) *bytes = tot;
    return bad ? -2.0 : el;
}

/* ------------------------------------------------------------------ */
/* Expected results of a whole bench batch (bench.py's full check):    */
/* for block b = block0 + i, len = lens[i] (or blen), the Seal tag and */
/* the checksum() array of the synthetic block, by the oracle's own    */
/* AEAD (AES-NI/PCLMUL GCM port, portable ChaCha20-Poly1305) and the   */
/* SSE4.2 CRC, nthreads threads.  tags: 16 B per block; crcs: crcstride */
/* bytes per block (checksum() bytes, BE).  Returns wall seconds.      */
/* ------------------------------------------------------------------ */
typedef struct {
    int algo;
    uint64_t seed, block0, i0, i1, blen, crcstride;
    const uint64_t *lens;
    uint8_t *tags, *crcs;
} expect_job;

static void *expect_worker(void *arg) {
    expect_job *j = (expect_job *)arg;
    uint64_t maxlen = j->blen;
    uint8_t *p = (uint8_t *)malloc(maxlen + 16), *c = (uint8_t *)malloc(maxlen + 16);
    for (uint64_t i = j->i0; i < j->i1; i++) {
        const uint64_t n = j->lens ? j->lens[i] : j->blen, b = j->block0 + i;
        uint8_t key[32], nonce[12];
        orc_gen_key(j->seed, b, key, nonce);
        orc_gen_block(j->seed, b, p, n);
        orc_checksum(p, (int64_t)n, j->crcs + i * j->crcstride, 1);
        if (j->algo == ALGO_AES256GCM)
            orc_aes256gcm_seal_ni(key, nonce, p, n, c, j->tags + 16 * i);
        else
            orc_chacha20poly1305_seal(key, nonce, NULL, 0, p, n, c, j->tags + 16 * i);
    }
    free(p);
    free(c);
    return NULL;
}

ORC_EXPORT double orc_expect_batch(int algo, int nthreads, uint64_t nblocks, const uint64_t *lens, uint64_t blen,
                                   uint64_t seed, uint64_t block0, uint8_t *tags, uint8_t *crcs, uint64_t crcstride) {
    if (nthreads < 1) nthreads = 1;
    uint64_t maxlen = blen;
    if (lens)
        for (uint64_t i = 0; i < nblocks; i++) maxlen = lens[i] > maxlen ? lens[i] : maxlen;
    if ((uint64_t)orc_checksum_len((int64_t)maxlen) > crcstride) return -3.0;
    expect_job *jobs = (expect_job *)calloc((size_t)nthreads, sizeof(expect_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    const uint64_t per = (nblocks + nthreads - 1) / nthreads;
    double t0 = now_s();
    for (int t = 0; t < nthreads; t++) {
        expect_job *j = &jobs[t];
        j->algo = algo;
        j->seed = seed;
        j->block0 = block0;
        j->blen = maxlen;
        j->lens = lens;
        j->crcstride = crcstride;
        j->tags = tags;
        j->crcs = crcs;
        j->i0 = (uint64_t)t * per < nblocks ? (uint64_t)t * per : nblocks;
        j->i1 = j->i0 + per < nblocks ? j->i0 + per : nblocks;
        pthread_create(&th[t], NULL, expect_worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    double el = now_s() - t0;
    free(jobs);
    free(th);
    return el;
}

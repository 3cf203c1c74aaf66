/* The cgo shim's call sequence, made from C through
 * the C-ABI exactly as the Go side makes it, checked against the CPU oracle.
 *
 *   §2 gpuEncryptor.Encrypt  -> jfsx_agg_data_encrypt over the multi-device
 *                               aggregator, from many threads, on malloc'd
 *                               (pageable, Go-heap-like) buffers (and the
 *                               one-call jfsx_data_encrypt, obj_crc NULL / set);
 *                               jfsx_agg_data_encrypt_ex / _decrypt_ex with the
 *                               plaintext checksum() out of the same call
 *      gpuEncryptor.Decrypt  -> jfsx_parse_header, [key unwrap], jfsx_agg_data_decrypt
 *                               (and jfsx_data_decrypt)
 *   §3 upload goroutines     -> jfsx_agg_seal / jfsx_agg_open on descriptors in
 *                               C memory whose src/dst/crc point into the pinned
 *                               pool (jfsx_alloc_pinned), from many threads;
 *                               the same over jfsx_mctx (every GPU)
 *   §4 checksum()            -> jfsx_checksum
 *      cacheFile.ReadAt      -> jfsx_checksum of rb, compared with the stored
 *                               CRCs; and jfsx_cache_verify for the level logic
 *   §5 LZ4.Compress/Decompress (cachedStore.upload / load) -> jfsx_agg_lz4_*
 *                               from many threads, zblk descriptors in C memory
 *      jfsxLZ4 / jfsxZstd run() with its empty-slice guards and stock
 *                               fallbacks, through the reference's own
 *                               testCompress (compress_test.go:25-76)
 *
 * Built in-tree by tests/harness/Makefile (from __graft_entry__.build());
 * run by tests/test_shim_sequence.py on the GPU box.  Exit 0 = all equal. */
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/jfsx.h"
#include "../../oracle/jfs_oracle.c"
#include "../../oracle/jfs_lz4.c"

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf(stderr, "shim check failed: %s (line %d)\n", #c, __LINE__); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

enum { SEED = 77, NTHREADS = 8, PER_THREAD = 3 };
static const uint64_t kLens[NTHREADS * PER_THREAD] = {
    0, 1, 17, 4096, 32767, 32768, 32769, 100003, 1 << 20, (4 << 20) - 3, 4 << 20, 65536 + 5,
    777, 5, 300000, 2 << 20, 3 << 20, 16, 1000000, 12345, 98309, 131072, 4095, 262144 + 9};

/* --- §2: one object per call ------------------------------------------ */
static void encrypt_decrypt(jfsx_ctx *ctx, int algo) {
    uint8_t wrapped[256];
    for (int k = 0; k < 256; k++) wrapped[k] = (uint8_t)(k * 7 + algo);
    for (int i = 0; i < 6; i++) {
        const uint64_t n = kLens[i * 4 + 1];
        uint8_t key[32], nonce[12];
        orc_gen_key(SEED, 1000 + i, key, nonce);
        uint8_t *p = malloc(n + 1), *obj = malloc(n + 287), *ref = malloc(n + 287), *back = malloc(n + 287);
        orc_gen_block(SEED, 1000 + i, p, n);
        uint64_t olen = 0;
        uint32_t ocrc = 0;
        CHECK(jfsx_data_encrypt(ctx, algo, key, nonce, wrapped, 256, p, n, obj, n + 287, &olen, NULL) == 0);
        CHECK(olen == n + 287);
        CHECK(orc_data_encrypt(algo, key, nonce, wrapped, 256, p, n, ref) == (int64_t)olen);
        CHECK(memcmp(obj, ref, olen) == 0);
        /* S3/OSS/COS: the object checksum in the same pass (checksum.go:31-53) */
        CHECK(jfsx_data_encrypt(ctx, algo, key, nonce, wrapped, 256, p, n, obj, n + 287, &olen, &ocrc) == 0);
        CHECK(ocrc == orc_crc32c_update(0, obj, olen));
        /* Decrypt: header, (key unwrap by the Go side), open */
        int klen = 0, nlen = 0;
        CHECK(jfsx_parse_header(obj, olen, &klen, &nlen) == 0 && klen == 256 && nlen == 12);
        uint64_t pl = 0;
        CHECK(jfsx_data_decrypt(ctx, algo, key, obj, olen, back, olen, &pl, NULL, NULL) == 0);
        CHECK(pl == n && memcmp(back, p, n) == 0);
        uint32_t got = 0;
        CHECK(jfsx_data_decrypt(ctx, algo, key, obj, olen, back, olen, &pl, &ocrc, &got) == 0 && got == ocrc);
        obj[olen - 1] ^= 1; /* tag */
        CHECK(jfsx_data_decrypt(ctx, algo, key, obj, olen, back, olen, &pl, NULL, NULL) == JFSX_ETAG);
        CHECK(jfsx_parse_header(obj, 271, &klen, &nlen) == JFSX_EMISFORMED);
        free(p), free(obj), free(ref), free(back);
    }
}

/* --- §2 as the shim runs it: per-object Encrypt / Decrypt from many
 * goroutines (max-uploads, cmd/flags.go:124-128) through the aggregator ---- */
typedef struct {
    jfsx_agg *agg;
    int algo, t, bad;
} obj_arg;

static void *obj_worker(void *vp) {
    obj_arg *a = (obj_arg *)vp;
    uint8_t wrapped[256];
    for (int k = 0; k < 256; k++) wrapped[k] = (uint8_t)(k * 5 + a->t);
    for (int j = 0; j < PER_THREAD; j++) {
        const int i = a->t * PER_THREAD + j;
        const uint64_t n = kLens[i];
        uint8_t key[32], nonce[12];
        orc_gen_key(SEED, 3000 + i, key, nonce);
        /* Go-heap shapes: the plaintext is io.ReadAll's slice, the object a
         * fresh make([]byte) (encrypt.go:183, :258) -- pageable malloc memory,
         * staged by the engine's bounce pool */
        uint8_t *p = malloc(n + 1), *obj = malloc(n + 287), *ref = malloc(n + 287), *back = malloc(n + 287);
        const int64_t cl = orc_checksum_len((int64_t)n);
        uint8_t *seg = malloc((size_t)cl), *seg2 = malloc((size_t)cl), *want = malloc((size_t)cl);
        orc_gen_block(SEED, 3000 + i, p, n);
        orc_checksum(p, (int64_t)n, want, 1);
        uint64_t olen = 0, pl = 0;
        uint32_t ocrc = 0, got = 0;
        if (jfsx_agg_data_encrypt(a->agg, a->algo, key, nonce, wrapped, 256, p, n, obj, n + 287, &olen, &ocrc) ||
            olen != n + 287 || orc_data_encrypt(a->algo, key, nonce, wrapped, 256, p, n, ref) != (int64_t)olen ||
            memcmp(obj, ref, olen) != 0 || ocrc != orc_crc32c_update(0, obj, olen))
            a->bad++;
        else if (jfsx_agg_data_decrypt(a->agg, a->algo, key, obj, olen, back, olen, &pl, &ocrc, &got) || pl != n ||
                 got != ocrc || memcmp(back, p, n) != 0)
            a->bad++;
        /* wSlice.upload -> bcache.stage + store.upload: checksum() of the
         * plaintext and the sealed object (and its object CRC) from one call;
         * store.load -> bcache.cache: the plaintext and its checksum() */
        memset(obj, 0, n + 287);
        ocrc = 0;
        if (jfsx_agg_data_encrypt_ex(a->agg, a->algo, key, nonce, wrapped, 256, p, n, obj, n + 287, &olen, &ocrc,
                                     seg) ||
            memcmp(obj, ref, olen) != 0 || ocrc != orc_crc32c_update(0, obj, olen) || memcmp(seg, want, (size_t)cl))
            a->bad++;
        else if (jfsx_agg_data_decrypt_ex(a->agg, a->algo, key, obj, olen, back, olen, &pl, &ocrc, &got, seg2) ||
                 pl != n || memcmp(back, p, n) != 0 || memcmp(seg2, want, (size_t)cl))
            a->bad++;
        else if (jfsx_agg_data_encrypt_ex(a->agg, a->algo, key, nonce, wrapped, 256, p, n, obj, n + 287, &olen, NULL,
                                          seg) || memcmp(obj, ref, olen) != 0 || memcmp(seg, want, (size_t)cl))
            a->bad++;
        free(p), free(obj), free(ref), free(back), free(seg), free(seg2), free(want);
    }
    return NULL;
}

static void agg_encrypt_decrypt(jfsx_mctx *m, int algo) {
    jfsx_agg *agg = NULL;
    CHECK(jfsx_agg_new_mctx(m, 0, 16u << 20, 500, &agg) == 0);
    pthread_t th[NTHREADS];
    obj_arg a[NTHREADS];
    for (int t = 0; t < NTHREADS; t++) {
        a[t] = (obj_arg){agg, algo, t, 0};
        CHECK(pthread_create(&th[t], NULL, obj_worker, &a[t]) == 0);
    }
    for (int t = 0; t < NTHREADS; t++) {
        CHECK(pthread_join(th[t], NULL) == 0);
        CHECK(a[t].bad == 0);
    }
    uint64_t calls = 0, batches = 0, blocks = 0;
    CHECK(jfsx_agg_stats(agg, &calls, &batches, &blocks) == 0 && calls == 5 * NTHREADS * PER_THREAD);
    CHECK(jfsx_agg_free(agg) == 0);
}

/* --- §3: per-block calls through the aggregator, descriptors in C memory -- */
typedef struct {
    jfsx_agg *agg;
    int algo, t;
    uint8_t *pool; /* pinned: plaintext | ciphertext | crc, per block */
    int bad;
} worker_arg;

static uint64_t slot_bytes(void) { return (4 << 20) + 4096; }

static void *worker(void *vp) {
    worker_arg *a = (worker_arg *)vp;
    for (int j = 0; j < PER_THREAD; j++) {
        const int i = a->t * PER_THREAD + j;
        const uint64_t n = kLens[i];
        uint8_t *p = a->pool + (uint64_t)i * 3 * slot_bytes(), *c = p + slot_bytes(), *crc = c + slot_bytes();
        jfsx_blk *b = (jfsx_blk *)calloc(1, sizeof(jfsx_blk)); /* C memory: cgo may pass it */
        orc_gen_key(SEED, (uint64_t)i, b->key, b->nonce);
        b->src = p;
        b->dst = c;
        b->len = n;
        b->crc = crc;
        if (jfsx_agg_seal(a->agg, a->algo, b, JFSX_CRC_GEN, JFSX_MEM_HOST) || b->status != JFSX_OK) a->bad++;
        uint8_t tag[16];
        memcpy(tag, b->tag, 16);
        /* read back: open + verify of the sealed block into the plaintext slot */
        memset(b, 0, sizeof(*b));
        orc_gen_key(SEED, (uint64_t)i, b->key, b->nonce);
        memcpy(b->tag, tag, 16);
        b->src = c;
        b->dst = p;
        b->len = n;
        b->crc = crc;
        if (jfsx_agg_open(a->agg, a->algo, b, JFSX_CRC_VERIFY, JFSX_MEM_HOST) || b->status != JFSX_OK) a->bad++;
        free(b);
    }
    return NULL;
}

static void aggregated(jfsx_ctx *ctx, jfsx_mctx *m, int algo) {
    void *pool = NULL;
    const uint64_t total = (uint64_t)NTHREADS * PER_THREAD * 3 * slot_bytes();
    CHECK(jfsx_alloc_pinned(ctx, total, &pool) == 0);
    uint8_t *pl = (uint8_t *)pool;
    for (int i = 0; i < NTHREADS * PER_THREAD; i++)
        orc_gen_block(SEED, (uint64_t)i, pl + (uint64_t)i * 3 * slot_bytes(), kLens[i]);
    jfsx_agg *agg = NULL;
    CHECK((m ? jfsx_agg_new_mctx(m, 0, 0, 500, &agg) : jfsx_agg_new(ctx, 0, 0, 500, &agg)) == 0);
    pthread_t th[NTHREADS];
    worker_arg wa[NTHREADS];
    for (int t = 0; t < NTHREADS; t++) {
        wa[t] = (worker_arg){agg, algo, t, pl, 0};
        CHECK(pthread_create(&th[t], NULL, worker, &wa[t]) == 0);
    }
    for (int t = 0; t < NTHREADS; t++) {
        pthread_join(th[t], NULL);
        CHECK(wa[t].bad == 0);
    }
    uint64_t calls = 0, batches = 0, blocks = 0;
    CHECK(jfsx_agg_stats(agg, &calls, &batches, &blocks) == 0);
    CHECK(calls == 2 * NTHREADS * PER_THREAD && blocks == calls && batches >= 2);
    CHECK(jfsx_agg_free(agg) == 0);
    /* after the round trip each plaintext slot holds its block again, and
     * the ciphertext / CRCs are the oracle's */
    for (int i = 0; i < NTHREADS * PER_THREAD; i++) {
        const uint64_t n = kLens[i];
        uint8_t *p = pl + (uint64_t)i * 3 * slot_bytes(), *c = p + slot_bytes(), *crc = c + slot_bytes();
        uint8_t *want = malloc(n + 1), *wc = malloc(n + 1), *wcrc = malloc(4 * (n / 32768 + 2));
        uint8_t key[32], nonce[12], tag[16];
        orc_gen_key(SEED, (uint64_t)i, key, nonce);
        orc_gen_block(SEED, (uint64_t)i, want, n);
        CHECK(memcmp(p, want, n) == 0);
        if (algo == JFSX_AES256GCM)
            orc_aes256gcm_seal_ni(key, nonce, want, n, wc, tag);
        else
            orc_chacha20poly1305_seal(key, nonce, NULL, 0, want, n, wc, tag);
        CHECK(memcmp(c, wc, n) == 0);
        const int64_t cl = orc_checksum(want, (int64_t)n, wcrc, 1);
        CHECK(memcmp(crc, wcrc, (size_t)cl) == 0);
        free(want), free(wc), free(wcrc);
    }
    CHECK(jfsx_free_pinned(ctx, pool) == 0);
}

/* --- §4: checksum() and the ReadAt verify ------------------------------ */
static void cache_checksums(jfsx_ctx *ctx) {
    for (int i = 0; i < 10; i++) {
        const uint64_t n = kLens[i + 3];
        const int64_t cl = orc_checksum_len((int64_t)n);
        uint8_t *file = malloc(n + (uint64_t)cl), *ref = malloc((size_t)cl), *gpu = malloc((size_t)cl);
        orc_gen_block(SEED, 500 + (uint64_t)i, file, n);
        CHECK(jfsx_checksum(ctx, file, n, gpu) == 0);
        orc_checksum(file, (int64_t)n, ref, 0);
        CHECK(memcmp(gpu, ref, (size_t)cl) == 0);
        memcpy(file + n, gpu, (size_t)cl); /* flushPage: data || checksum(data) */
        /* ReadAt full-block verify: checksum(rb) against the stored CRCs */
        if (n) {
            file[n / 2] ^= 0x20;
            CHECK(jfsx_checksum(ctx, file, n, gpu) == 0);
            const int64_t seg = (int64_t)(n / 2) / 32768;
            CHECK(memcmp(gpu, file + n, (size_t)cl) != 0 && memcmp(gpu + 4 * seg, file + n + 4 * seg, 4) != 0);
            file[n / 2] ^= 0x20;
        }
        /* level logic: jfsx_cache_verify == orc_cache_readat on a few ranges */
        for (int level = 0; level < 4; level++) {
            const uint64_t offs[3] = {0, n / 3, n > 100 ? n - 100 : 0};
            for (int r = 0; r < 3; r++) {
                const uint64_t off = offs[r], size = r == 0 ? n : (n - off) / 2 + 1;
                uint8_t *o1 = malloc(size + 1), *o2 = malloc(size + 1);
                uint64_t n1 = 0;
                int64_t n2 = 0, b1 = -1, b2 = -1;
                uint32_t g1 = 0, e1 = 0, g2 = 0, e2 = 0;
                const int rc1 = jfsx_cache_verify(ctx, file, n + (uint64_t)cl, n, level, off, size, o1, &n1, &g1, &e1, &b1);
                const int rc2 = orc_cache_readat(file, (int64_t)n + cl, (int64_t)n, level, (int64_t)off, (int64_t)size, o2,
                                                 &n2, &g2, &e2, &b2);
                CHECK(rc1 == (rc2 == 0 ? 0 : rc2 == 1 ? JFSX_ECRC : JFSX_EOF));
                CHECK(n1 == (uint64_t)n2 && memcmp(o1, o2, n1) == 0);
                free(o1), free(o2);
            }
        }
        free(file), free(ref), free(gpu);
    }
}

/* §5: one Compress then one Decompress per block and thread, as the upload
 * and load goroutines make them; text-like and incompressible blocks */
typedef struct {
    jfsx_agg *agg;
    uint8_t *src, *cmp, *back;
    uint64_t n, cap;
    int bad;
} lz4_arg;

static void *lz4_worker(void *vp) {
    lz4_arg *a = (lz4_arg *)vp;
    jfsx_zblk *z = (jfsx_zblk *)calloc(1, sizeof(jfsx_zblk));
    z->src = a->src, z->src_len = a->n, z->dst = a->cmp, z->dst_cap = a->cap;
    if (jfsx_agg_lz4_compress(a->agg, z, JFSX_MEM_HOST) || z->status) a->bad = 1;
    const uint64_t cl = z->out_len;
    z->src = a->cmp, z->src_len = cl, z->dst = a->back, z->dst_cap = a->n;
    if (jfsx_agg_lz4_decompress(a->agg, z, JFSX_MEM_HOST) || z->status || z->out_len != a->n) a->bad = 1;
    a->cap = cl;  /* compressed length, for the oracle check */
    free(z);
    return NULL;
}

static void lz4_stage(jfsx_ctx *ctx) {
    enum { T = 12 };
    jfsx_agg *agg = NULL;
    CHECK(jfsx_agg_new(ctx, 0, 0, 1000, &agg) == 0);
    lz4_arg a[T];
    pthread_t th[T];
    for (int t = 0; t < T; t++) {
        const uint64_t n = 20000 + 77777 * (uint64_t)t;
        memset(&a[t], 0, sizeof(a[t]));
        a[t].agg = agg, a[t].n = n, a[t].cap = jfsx_lz4_bound(n);
        a[t].src = (uint8_t *)malloc(n), a[t].cmp = (uint8_t *)malloc(a[t].cap), a[t].back = (uint8_t *)malloc(n);
        if (t % 3 == 2) {
            orc_gen_block(SEED, 500 + t, a[t].src, n);
        } else {
            /* words of a small vocabulary from an LCG */
            uint32_t x = 12345u + t;
            for (uint64_t i = 0; i < n; i++) {
                x = x * 1103515245u + 12345u;
                a[t].src[i] = (x >> 16) % 11 == 0 ? ' ' : (uint8_t)('a' + ((x >> 20) % (t % 3 ? 6 : 26)));
            }
        }
        CHECK(pthread_create(&th[t], NULL, lz4_worker, &a[t]) == 0);
    }
    for (int t = 0; t < T; t++) {
        CHECK(pthread_join(th[t], NULL) == 0);
        CHECK(a[t].bad == 0);
        uint8_t *ref = (uint8_t *)malloc(orc_lz4_bound((int)a[t].n));
        const int rl = orc_lz4_compress(a[t].src, (int)a[t].n, ref, orc_lz4_bound((int)a[t].n));
        CHECK((uint64_t)rl == a[t].cap && memcmp(ref, a[t].cmp, (size_t)rl) == 0);
        CHECK(memcmp(a[t].back, a[t].src, a[t].n) == 0);
        free(ref), free(a[t].src), free(a[t].cmp), free(a[t].back);
    }
    uint64_t calls, batches, blocks;
    CHECK(jfsx_agg_stats(agg, &calls, &batches, &blocks) == 0 && calls == 2 * T && batches < calls);
    CHECK(jfsx_agg_free(agg) == 0);
}

/* §5 jfsxEngine.run, as the Go shim makes it: descriptor and both buffers in
 * C memory (malloc(len + 1): never malloc(0)), the source copied in only when
 * non-empty, the output copied out only when status is OK and out_len > 0.
 * Returns 1 and sets *n / *st, or 0 when the engine failed as a whole. */
enum { OP_LZ4C, OP_LZ4D, OP_ZSTDC, OP_ZSTDD };
static int shim_run(jfsx_agg *agg, int op, uint8_t *dst, size_t dlen, const uint8_t *src, size_t slen, int *n,
                    int *st) {
    jfsx_zblk *z = (jfsx_zblk *)calloc(1, sizeof(jfsx_zblk));
    void *in = malloc(slen + 1), *out = malloc(dlen + 1);
    if (slen > 0) memcpy(in, src, slen);
    z->src = in, z->src_len = slen, z->dst = out, z->dst_cap = dlen;
    int rc = op == OP_LZ4C ? jfsx_agg_lz4_compress(agg, z, JFSX_MEM_HOST)
             : op == OP_LZ4D ? jfsx_agg_lz4_decompress(agg, z, JFSX_MEM_HOST)
             : op == OP_ZSTDC ? jfsx_agg_zstd_compress(agg, z, JFSX_MEM_HOST)
                              : jfsx_agg_zstd_decompress(agg, z, JFSX_MEM_HOST);
    int ok = rc == 0;
    if (ok) {
        *n = (int)z->out_len;
        *st = z->status;
        if (z->status == JFSX_OK && z->out_len > 0) memcpy(dst, out, z->out_len);
    }
    free(in), free(out), free(z);
    return ok;
}

/* the stock cgo codecs the shim falls back to: go-lz4 (the oracle's LZ4
 * restatement, pinned to liblz4) and DataDog/zstd (the system libzstd) */
static size_t (*zs_compress)(void *, size_t, const void *, size_t, int);
static size_t (*zs_decompress)(void *, size_t, const void *, size_t);
static size_t (*zs_bound)(size_t);
static unsigned (*zs_iserr)(size_t);
static void load_zstd(void) {
    void *h = dlopen("libzstd.so.1", RTLD_NOW);
    CHECK(h);
    zs_compress = (size_t(*)(void *, size_t, const void *, size_t, int))dlsym(h, "ZSTD_compress");
    zs_decompress = (size_t(*)(void *, size_t, const void *, size_t))dlsym(h, "ZSTD_decompress");
    zs_bound = (size_t(*)(size_t))dlsym(h, "ZSTD_compressBound");
    zs_iserr = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
    CHECK(zs_compress && zs_decompress && zs_bound && zs_iserr);
}
/* Compressor results: 0 ok (n set), -1 error */
static int stock(int op, uint8_t *dst, size_t dlen, const uint8_t *src, size_t slen, int *n) {
    if (op == OP_LZ4C) {
        int r = orc_lz4_compress(src, (int)slen, dst, (int)dlen);
        return r > 0 ? (*n = r, 0) : -1;
    }
    if (op == OP_LZ4D) {
        int r = orc_lz4_decompress(src, (int)slen, dst, (int)dlen);
        return r >= 0 ? (*n = r, 0) : -1;
    }
    if (op == OP_ZSTDC) {  /* CompressLevel: a new buffer below the bound -> "buffer too short" */
        if (dlen < zs_bound(slen)) return -1;
        size_t r = zs_compress(dst, dlen, src, slen, 1);
        return zs_iserr(r) ? -1 : (*n = (int)r, 0);
    }
    if (slen == 0) return -1; /* ErrEmptySlice */
    size_t r = zs_decompress(dst, dlen, src, slen); /* too small: a larger buffer, "buffer too short" */
    return zs_iserr(r) ? -1 : (*n = (int)r, 0);
}
/* jfsxLZ4 / jfsxZstd Compress and Decompress */
static int shim_codec(jfsx_agg *agg, int op, uint8_t *dst, size_t dlen, const uint8_t *src, size_t slen, int *n) {
    int st = 0;
    if (op == OP_LZ4C && dlen < jfsx_lz4_bound(slen)) return stock(op, dst, dlen, src, slen, n);
    if (op == OP_ZSTDC && dlen < jfsx_zstd_bound(slen)) return stock(op, dst, dlen, src, slen, n);
    if (op == OP_LZ4D && slen == 0) return -1; /* "decompress an empty input" */
    if (op == OP_ZSTDD && slen == 0) return stock(op, dst, dlen, src, slen, n);
    if (shim_run(agg, op, dst, dlen, src, slen, n, &st) && st == JFSX_OK) return 0;
    return stock(op, dst, dlen, src, slen, n);
}

/* compress_test.go:25-76, testCompress(t, c), for c = lz4 and zstd */
static void compress_contract(jfsx_agg *agg, int comp, int decomp, const char *name) {
    for (int pass = 0; pass < 2; pass++) {
        const uint8_t *src = pass == 0 ? (const uint8_t *)name : NULL;
        const size_t slen = pass == 0 ? strlen(name) : 0; /* testIt(src), testIt(nil) */
        uint8_t one[1];
        int n = 0, m = 0;
        if (slen > 1) CHECK(shim_codec(agg, comp, one, 1, src, slen, &n) != 0); /* short buffer error */
        const size_t bound = comp == OP_LZ4C ? jfsx_lz4_bound(slen) : jfsx_zstd_bound(slen);
        uint8_t *dst = (uint8_t *)malloc(bound + 1);
        CHECK(shim_codec(agg, comp, dst, bound, src, slen, &n) == 0);
        /* the engine's bytes are the stock codec's */
        uint8_t *ref = (uint8_t *)malloc(bound + 1);
        int rn = 0;
        CHECK(stock(comp, ref, bound, src, slen, &rn) == 0 && rn == n && memcmp(ref, dst, (size_t)n) == 0);
        if (slen > 1) CHECK(shim_codec(agg, decomp, one, 1, dst, (size_t)n, &m) != 0);
        uint8_t *src2 = (uint8_t *)malloc(slen + 1);
        CHECK(shim_codec(agg, decomp, src2, slen, dst, (size_t)n, &m) == 0);
        CHECK((size_t)m == slen && (slen == 0 || memcmp(src2, src, slen) == 0));
        free(dst), free(ref), free(src2);
    }
    /* CompressBound(0) > 0 for both: an empty input does not decompress */
    uint8_t buf[100];
    int m = 0;
    CHECK(shim_codec(agg, decomp, buf, sizeof(buf), (const uint8_t *)"", 0, &m) != 0);
}

int main(void) {
    CHECK(jfsx_abi_version() == JFSX_ABI_VERSION);
    int nd = 0;
    CHECK(jfsx_device_count(&nd) == 0 && nd > 0);
    jfsx_ctx *ctx = NULL;
    CHECK(jfsx_ctx_open(0, 0, &ctx) == 0);
    jfsx_mctx *m = NULL;
    CHECK(jfsx_mctx_open(0, 0, &m) == 0 && jfsx_mctx_ndev(m) == nd);
    for (int algo = 0; algo < 2; algo++) {
        encrypt_decrypt(ctx, algo);
        agg_encrypt_decrypt(m, algo);
        aggregated(ctx, NULL, algo);
        aggregated(ctx, m, algo);
    }
    cache_checksums(ctx);
    lz4_stage(ctx);
    {
        jfsx_agg *agg = NULL;
        load_zstd();
        CHECK(jfsx_agg_new_mctx(m, 0, 0, 200, &agg) == 0);
        compress_contract(agg, OP_LZ4C, OP_LZ4D, "LZ4");
        compress_contract(agg, OP_ZSTDC, OP_ZSTDD, "Zstd");
        CHECK(jfsx_agg_free(agg) == 0);
    }
    CHECK(jfsx_mctx_close(m) == 0);
    CHECK(jfsx_ctx_close(ctx) == 0);
    printf("shim sequence ok (%d device%s)\n", nd, nd == 1 ? "" : "s");
    return 0;
}

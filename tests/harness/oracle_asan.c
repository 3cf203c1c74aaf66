/* Sanitizer driver for the CPU oracle (oracle/jfs_oracle.c, test
 * infrastructure): built with -fsanitize=address,undefined by
 * tests/test_sanitizers.py and run standalone.  Exercises every exported
 * entry point on ragged sizes, including the cacheFile.ReadAt restatement on
 * random (level, off, size, corruption) cases, and checks the redundant
 * implementations against each other.  Exit 0 = consistent and clean. */
#include "../../oracle/jfs_oracle.c"

#include <stdio.h>

static uint64_t rng_s = 0x1234567;
static uint64_t rnd(void) {
    rng_s = rng_s * 6364136223846793005ULL + 1442695040888963407ULL;
    return rng_s >> 17;
}

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                                    \
        }                                                                \
    } while (0)

static int aead_cases(void) {
    static const uint64_t lens[] = {0, 1, 15, 16, 17, 63, 64, 65, 255, 1000, 4095, 32767, 32768, 32769, 100003};
    for (size_t i = 0; i < sizeof(lens) / sizeof(lens[0]); i++) {
        const uint64_t n = lens[i];
        uint8_t key[32], nonce[12], t1[16], t2[16], t3[16];
        orc_gen_key(3, i, key, nonce);
        uint8_t *p = malloc(n + 1), *c1 = malloc(n + 1), *c2 = malloc(n + 1), *c3 = malloc(n + 1), *q = malloc(n + 1);
        orc_gen_block(3, i, p, n);
        orc_aes256gcm_seal(key, nonce, NULL, 0, p, n, c1, t1);
        orc_aes256gcm_seal_ni(key, nonce, p, n, c2, t2);
        CHECK(!memcmp(c1, c2, n) && !memcmp(t1, t2, 16));
        CHECK(orc_aes256gcm_open(key, nonce, NULL, 0, c1, n, t1, q) == 0 && !memcmp(q, p, n));
        CHECK(orc_aes256gcm_open_ni(key, nonce, c1, n, t1, q) == 0 && !memcmp(q, p, n));
        t1[0] ^= 1;
        CHECK(orc_aes256gcm_open(key, nonce, NULL, 0, c1, n, t1, q) == -1);
        orc_chacha20poly1305_seal(key, nonce, NULL, 0, p, n, c3, t3);
        CHECK(orc_chacha20poly1305_open(key, nonce, NULL, 0, c3, n, t3, q) == 0 && !memcmp(q, p, n));
        if (evp_load()) {
            uint8_t te[16];
            CHECK(orc_evp_seal(0, key, nonce, p, n, c2, te) == 0 && !memcmp(c2, c1, n) && !memcmp(te, t2, 16));
            CHECK(orc_evp_seal(1, key, nonce, p, n, c2, te) == 0 && !memcmp(c2, c3, n) && !memcmp(te, t3, 16));
        }
        /* object format round trip (encrypt.go:164-216) */
        uint8_t wrapped[256];
        for (int k = 0; k < 256; k++) wrapped[k] = (uint8_t)k;
        uint8_t *obj = malloc(3 + 256 + 12 + n + 16), *back = malloc(3 + 256 + 12 + n + 16);
        for (int algo = 0; algo < 2; algo++) {
            int64_t ol = orc_data_encrypt(algo, key, nonce, wrapped, 256, p, n, obj);
            CHECK(ol == (int64_t)(3 + 256 + 12 + n + 16));
            CHECK(orc_data_decrypt(algo, key, obj, ol, back) == (int64_t)n && !memcmp(back, p, n));
            CHECK(orc_data_decrypt(algo, key, obj, 271, back) == -1);
        }
        /* CRC variants agree; checksum() layout */
        CHECK(orc_crc32c_update(7, p, n) == orc_crc32c_update_hw(7, p, n));
        CHECK(orc_crc32c_update(7, p, n) == orc_crc32c_update_hw3(7, p, n));
        uint8_t *cs1 = malloc((size_t)orc_checksum_len((int64_t)n)), *cs2 = malloc((size_t)orc_checksum_len((int64_t)n));
        CHECK(orc_checksum(p, (int64_t)n, cs1, 0) == orc_checksum_len((int64_t)n));
        orc_checksum(p, (int64_t)n, cs2, 1);
        CHECK(!memcmp(cs1, cs2, (size_t)orc_checksum_len((int64_t)n)));
        free(cs1), free(cs2), free(obj), free(back);
        free(p), free(c1), free(c2), free(c3), free(q);
    }
    return 0;
}

static int readat_cases(void) {
    static const int64_t lens[] = {1, 1000, 32768, 32769, 100000, 5 * 32768, (1 << 20) + 5};
    for (int it = 0; it < 3000; it++) {
        const int64_t len = lens[it % 7];
        const int64_t cl = orc_checksum_len(len);
        uint8_t *img = malloc((size_t)(len + cl));
        orc_gen_block(9, (uint64_t)it, img, (uint64_t)len);
        orc_checksum(img, len, img + len, 1);
        const int kind = (int)(rnd() % 4);
        if (kind == 1) img[rnd() % (uint64_t)len] ^= 1;
        if (kind == 2) img[len + (int64_t)(rnd() % (uint64_t)cl)] ^= 4;
        const int64_t fsize = kind == 3 ? len : len + cl;
        const int level = orc_open_cache_file(fsize, len, (int)(rnd() % 4));
        CHECK(level >= 0);
        int64_t off = (int64_t)(rnd() % (uint64_t)(len + 1)), size = (int64_t)(rnd() % (uint64_t)(len + 40000));
        if (it % 5 == 0) off = 0, size = len;
        uint8_t *out = malloc((size_t)(size ? size : 1));
        int64_t n = -7, bad = -1;
        uint32_t got = 0, ex = 0;
        const int rc = orc_cache_readat(img, fsize, len, level, off, size, out, &n, &got, &ex, &bad);
        CHECK(rc >= 0 && rc <= 2 && n >= 0 && n <= size);
        if (rc == 1) CHECK(bad >= 0 && got != ex);
        if (rc == 0 && n) CHECK(!memcmp(out, img + off, (size_t)n));
        free(out);
        free(img);
    }
    return 0;
}

int main(void) {
    if (aead_cases() || readat_cases()) return 1;
    uint32_t d1 = 0, d2 = 0;
    CHECK(orc_bench_seal_crc(0, 3, 5, 70000, 11, &d1) >= 0);
    if (evp_load()) {
        CHECK(orc_bench_seal_crc_evp(0, 3, 5, 70000, 11, &d2) >= 0);
        CHECK(d1 == d2);
    }
    printf("oracle sanitizer run ok\n");
    return 0;
}

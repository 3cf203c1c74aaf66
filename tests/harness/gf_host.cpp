// CPU build of juicefs_amd/csrc/jfsx_gf.h (test infrastructure only): the
// integer-multiply GF(2^128) product, checked by tests/test_gf.py against the
// bit-serial product of SP 800-38D Algorithm 1 (the kernels' g_mul, restated
// here on the same reflected words) and against Python.
#include <stdint.h>

#include "../../juicefs_amd/csrc/jfsx_gf.h"

namespace {
// SP 800-38D Algorithm 1 on words w[0..3], w[0] bit 31 = x^0
void mul_serial(const uint32_t x[4], const uint32_t y[4], uint32_t z[4]) {
    uint32_t v[4] = {y[0], y[1], y[2], y[3]};
    z[0] = z[1] = z[2] = z[3] = 0;
    for (int k = 0; k < 4; k++) {
        uint32_t xw = x[k];
        for (int i = 0; i < 32; i++) {
            const uint32_t m = 0u - (xw >> 31);
            xw <<= 1;
            for (int q = 0; q < 4; q++) z[q] ^= v[q] & m;
            const uint32_t lsb = v[3] & 1u;
            v[3] = (v[3] >> 1) | (v[2] << 31);
            v[2] = (v[2] >> 1) | (v[1] << 31);
            v[1] = (v[1] >> 1) | (v[0] << 31);
            v[0] = (v[0] >> 1) ^ (0xE1000000u & (0u - lsb));
        }
    }
}
}  // namespace

extern "C" {
void gf_mul(const uint32_t *x, const uint32_t *y, uint32_t *z) { jfsx_gf::mul(x, y, z); }
void gf_mul_serial(const uint32_t *x, const uint32_t *y, uint32_t *z) { mul_serial(x, y, z); }
uint64_t gf_clmul32(uint32_t x, uint32_t y) { return jfsx_gf::clmul32(x, y); }
// n random products (xorshift from seed), returns the number that differ
int gf_check(uint64_t seed, int n) {
    int bad = 0;
    for (int i = 0; i < n; i++) {
        uint32_t x[4], y[4], a[4], b[4];
        for (int q = 0; q < 8; q++) {
            seed ^= seed << 13;
            seed ^= seed >> 7;
            seed ^= seed << 17;
            (q < 4 ? x[q] : y[q - 4]) = (uint32_t)(seed >> 16);
        }
        if (i % 7 == 0) x[i % 4] = 0xffffffffu;  // dense words
        if (i % 11 == 0) y[(i + 1) % 4] = 0;
        jfsx_gf::mul(x, y, a);
        mul_serial(x, y, b);
        for (int q = 0; q < 4; q++) bad += a[q] != b[q];
    }
    return bad;
}
}

// Host build of the engine's Zstandard decoder (juicefs_amd/csrc/jfsx_zstd.h,
// the code the GPU kernel runs) for the CPU test suite: plain memory behind
// the decoder's Env interface.  Built by tests/test_zstd_host.py with g++.
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../juicefs_amd/csrc/jfsx_zstd.h"

namespace {
struct HostEnv {
    const uint8_t *src;
    int64_t n;
    uint8_t *dst;
    uint8_t *lit;
    uint8_t in8(int64_t i) const { return (i >= 0 && i < n) ? src[i] : 0; }
    uint64_t in64(int64_t i) const {
        uint64_t v = 0;
        for (int k = 0; k < 8; k++) v |= (uint64_t)in8(i + k) << (8 * k);
        return v;
    }
    uint64_t in64u(int64_t i) const {  // the device reads these unchecked
        if (i < 0 || i + 8 > n) abort();
        return in64(i);
    }
    void lit_put(uint64_t i, uint32_t b) const { lit[i] = (uint8_t)b; }
    void lit_put4(uint32_t o0, uint32_t w0, uint32_t o1, uint32_t w1, uint32_t o2, uint32_t w2, uint32_t o3,
                  uint32_t w3) const {
        const uint32_t o[4] = {o0, o1, o2, o3}, w[4] = {w0, w1, w2, w3};
        for (int j = 0; j < 4; j++)
            for (int i = 0; i < 4; i++) lit[o[j] + i] = (uint8_t)(w[j] >> (8 * i));
    }
    void lit_fill(uint64_t i, uint32_t b, uint64_t cnt) { memset(lit + i, (int)b, cnt); }
    void lit_sync() {}
    void stamp(int) {}
    uint16_t *hufg;
    void huf_fill(uint16_t *p, uint16_t v, uint32_t cnt) const {
        for (uint32_t j = 0; j < cnt; j++) p[j] = v;
    }
    uint16_t *huf_g() const { return hufg; }
    void huf_sync() const {}
    uint32_t huf_ld(uint32_t i) const { return hufg[i]; }
    void out_sync() {}
    void out_from_in(uint64_t o, int64_t i, uint64_t cnt) { memcpy(dst + o, src + i, cnt); }
    void out_from_lit(uint64_t o, uint64_t i, uint64_t cnt) { memcpy(dst + o, lit + i, cnt); }
    void out_fill(uint64_t o, uint32_t b, uint64_t cnt) { memset(dst + o, (int)b, cnt); }
    void out_match(uint64_t o, uint64_t off, uint64_t cnt) {
        for (uint64_t j = 0; j < cnt; j++) dst[o + j] = dst[o - off + j];
    }
    uint64_t out64(uint64_t o) const {
        uint64_t v;
        memcpy(&v, dst + o, 8);
        return v;
    }
    uint32_t out32(uint64_t o) const {
        uint32_t v;
        memcpy(&v, dst + o, 4);
        return v;
    }
    uint32_t out8(uint64_t o) const { return dst[o]; }
};
}  // namespace

extern "C" int64_t zstd_host_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
    static thread_local jzd::Tables t;
    std::vector<uint8_t> litbuf(jzd::kBlockMax + 64);
    std::vector<uint16_t> hufbuf(1u << jzd::kHufLogMax);
    HostEnv e{src, n, dst, litbuf.data(), hufbuf.data()};
    // decode into an exactly sized heap copy, so ASan builds of this harness
    // see any read past the output's end
    std::vector<uint8_t> out((size_t)cap);
    e.dst = out.data();
    const int64_t r = jzd::decompress(e, t, (uint64_t)n, (uint64_t)cap);
    if (r > 0) memcpy(dst, out.data(), (size_t)r);
    return r;
}

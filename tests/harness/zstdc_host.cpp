// Host build of the engine's Zstandard level-1 encoder (jfsx_zstdc.h): the
// same source the GPU kernel runs, compiled for the CPU so tests can compare
// its frames byte for byte with the system libzstd (tests/test_zstdc_host.py).
// Test infrastructure only.
#include <stdint.h>
#include <string.h>

#include <vector>

#include "../../juicefs_amd/csrc/jfsx_zstdc.h"

extern "C" int64_t zstdc_host_compress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
    if ((uint64_t)cap < jzc::compress_bound((uint64_t)n)) return -1;
    static thread_local std::vector<uint32_t> htab(1u << jzc::kHashLogMax);
    static thread_local std::vector<jzc::SeqDef> seqs(jzc::kMaxSeq);
    static thread_local std::vector<uint8_t> lits(jzc::kBlockMax + 64), codes(3 * jzc::kMaxSeq), body(jzc::kBodyCap);
    static thread_local jzc::Work w;
    // exactly sized copies, so an ASan build sees any read past the input
    std::vector<uint8_t> in(src, src + n);
    return (int64_t)jzc::compress_frame(in.data(), (uint64_t)n, dst, htab.data(), seqs.data(), lits.data(),
                                        codes.data(), body.data(), w);
}

extern "C" uint64_t zstdc_host_bound(uint64_t n) { return jzc::compress_bound(n); }

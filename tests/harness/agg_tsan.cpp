// ThreadSanitizer driver for the host scheduling code of libjfsx
// (juicefs_amd/csrc/jfsx_agg.cpp: async tickets, the aggregator and its
// per-device dispatchers, the multi-device context) over the stub engine of
// agg_host.cpp.  Built with -fsanitize=thread by tests/test_sanitizers.py and
// run standalone; exit 0 = every caller got its own result and TSan is silent.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "agg_host.cpp"

namespace {
bool tag_ok(const jfsx_blk &b, int algo) {
    for (int k = 0; k < 16; k++)
        if (b.tag[k] != (uint8_t)(b.key[k] ^ (uint8_t)(b.len >> (8 * (k & 7))) ^ (uint8_t)algo)) return false;
    return true;
}
}  // namespace

int main() {
    harness_reset(200);
    std::atomic<int> bad{0};
    // 1) single-context aggregator under 48 threads, mixed ops
    {
        jfsx_agg *a = nullptr;
        if (jfsx_agg_new((jfsx_ctx *)0x1000, 8, 0, 300, &a)) return 1;
        std::vector<std::thread> ts;
        for (int t = 0; t < 48; t++)
            ts.emplace_back([&, t] {
                for (int i = 0; i < 40; i++) {
                    jfsx_blk b{};
                    for (int k = 0; k < 32; k++) b.key[k] = (uint8_t)(t * 31 + i + k);
                    b.len = 100 + t * 7 + i;
                    if (i % 3 == 2) {
                        jfsx_range r{};
                        r.len = b.len;
                        if (jfsx_agg_crc32c(a, &r, JFSX_CRC_VERIFY, JFSX_MEM_HOST)) bad++;
                        continue;
                    }
                    if (jfsx_agg_seal(a, t & 1, &b, JFSX_CRC_NONE, JFSX_MEM_HOST) || !tag_ok(b, t & 1)) bad++;
                }
            });
        for (auto &th : ts) th.join();
        jfsx_agg_free(a);
    }
    // 2) multi-device context: concurrent host batches and the per-device aggregator
    {
        jfsx_mctx *m = nullptr;
        if (jfsx_mctx_open(0, 0, &m)) return 1;
        std::vector<std::thread> ts;
        for (int t = 0; t < 6; t++)
            ts.emplace_back([&, t] {
                std::vector<jfsx_blk> v(37);
                for (size_t i = 0; i < v.size(); i++) {
                    v[i].key[0] = (uint8_t)(i + t);
                    v[i].len = 1000 * (i % 5 + 1);
                }
                if (jfsx_mctx_seal_batch(m, 1, (int)v.size(), v.data(), JFSX_CRC_GEN, JFSX_MEM_HOST)) bad++;
                for (auto &b : v)
                    if (!tag_ok(b, 1)) bad++;
            });
        jfsx_agg *a = nullptr;
        if (jfsx_agg_new_mctx(m, 4, 0, 200, &a)) return 1;
        for (int t = 0; t < 24; t++)
            ts.emplace_back([&, t] {
                for (int i = 0; i < 20; i++) {
                    jfsx_blk b{};
                    b.key[3] = (uint8_t)(t ^ i);
                    b.len = 4096 + i;
                    if (jfsx_agg_seal(a, 0, &b, JFSX_CRC_NONE, JFSX_MEM_HOST) || !tag_ok(b, 0)) bad++;
                }
            });
        for (auto &th : ts) th.join();
        jfsx_agg_free(a);
        jfsx_mctx_close(m);
    }
    // 3) async tickets: submit from several threads, wait from others
    {
        jfsx_ctx *c = (jfsx_ctx *)0x2000;
        std::vector<jfsx_ticket> tk(16);
        std::vector<std::vector<jfsx_blk>> bufs(16, std::vector<jfsx_blk>(3));
        std::vector<std::thread> ts;
        for (int t = 0; t < 16; t++)
            ts.emplace_back([&, t] {
                for (auto &b : bufs[t]) b.len = 50 + t;
                if (jfsx_seal_batch_async(c, 0, 3, bufs[t].data(), 0, JFSX_MEM_DEVICE, &tk[t])) bad++;
            });
        for (auto &th : ts) th.join();
        ts.clear();
        for (int t = 0; t < 16; t++)
            ts.emplace_back([&, t] {
                if (jfsx_wait(c, tk[t], -1)) bad++;
                for (auto &b : bufs[t])
                    if (!tag_ok(b, 0)) bad++;
            });
        for (auto &th : ts) th.join();
        harness_close(c);
    }
    // 4) pageable per-object Seal / Open: 24 callers staging through the
    // shared arenas (slices reserved, copied, released from many threads)
    {
        const int T = 24, PER = 8;
        const uint64_t L = 20000;
        std::vector<uint8_t> buf((size_t)2 * T * PER * L);
        for (size_t i = 0; i < buf.size() / 2; i++) buf[i] = (uint8_t)(i * 131);
        harness_pageable((uintptr_t)buf.data(), (uintptr_t)buf.data() + buf.size());
        jfsx_agg *a = nullptr;
        if (jfsx_agg_new((jfsx_ctx *)0x1000, 0, 1 << 20, 200, &a)) return 1;
        std::vector<std::thread> ts;
        for (int t = 0; t < T; t++)
            ts.emplace_back([&, t] {
                for (int j = 0; j < PER; j++) {
                    const size_t i = (size_t)t * PER + j;
                    uint8_t *src = buf.data() + i * L, *obj = buf.data() + (size_t)T * PER * L + i * L;
                    jfsx_blk b{};
                    for (int k = 0; k < 32; k++) b.key[k] = (uint8_t)(i + k);
                    b.src = src;
                    b.dst = obj;
                    b.len = L;
                    if (jfsx_agg_seal(a, 0, &b, 0, JFSX_MEM_HOST) || !tag_ok(b, 0)) bad++;
                    for (uint64_t x = 0; x < L; x++)
                        if (obj[x] != (uint8_t)(src[x] ^ b.key[x & 31] ^ 0x5A)) {
                            bad++;
                            break;
                        }
                    b.src = b.dst = obj;  // Open in place: the plaintext comes back
                    if (jfsx_agg_open(a, 0, &b, 0, JFSX_MEM_HOST) || b.status != JFSX_OK || memcmp(obj, src, L)) bad++;
                }
            });
        for (auto &th : ts) th.join();
        jfsx_agg_free(a);
        harness_pageable(0, 0);
    }
    if (bad) {
        std::fprintf(stderr, "%d wrong results\n", bad.load());
        return 1;
    }
    std::printf("scheduler sanitizer run ok\n");
    return 0;
}

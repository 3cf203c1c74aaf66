// Host build of the aggregator and the async queue (juicefs_amd/csrc/jfsx_agg.cpp)
// over stub batch entry points, so their scheduling logic -- grouping, windows,
// size caps, error isolation, ordering, shutdown -- is testable without a GPU.
// The stubs record every batch they receive and compute a position-free fake
// "tag" so results can be matched to their requesters.
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "../../juicefs_amd/csrc/jfsx_agg.cpp"

namespace {
std::mutex h_mu;
std::vector<int> h_sizes;   // blocks per batch, in issue order
std::vector<int> h_ops;     // 0 seal, 1 open, 2 crc
std::vector<int> h_modes;
int h_sleep_us = 2000;

int stub(int op, int n, int mode) {
    {
        std::lock_guard<std::mutex> g(h_mu);
        h_sizes.push_back(n);
        h_ops.push_back(op);
        h_modes.push_back(mode);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(h_sleep_us));
    return 0;
}
}  // namespace

extern "C" {

// fake transform: tag[i] = key[i] ^ (len >> 8*(i&7)); reserved != 0 -> EINVAL
int jfsx_seal_batch(jfsx_ctx *, int algo, int n, jfsx_blk *b, int crc_mode, int mem) {
    for (int i = 0; i < n; i++)
        if (b[i].reserved) return JFSX_EINVAL;
    stub(0, n, crc_mode);
    for (int i = 0; i < n; i++) {
        for (int k = 0; k < 16; k++) b[i].tag[k] = b[i].key[k] ^ (uint8_t)(b[i].len >> (8 * (k & 7))) ^ (uint8_t)algo;
        b[i].status = JFSX_OK;
    }
    return 0;
}

int jfsx_open_batch(jfsx_ctx *, int algo, int n, jfsx_blk *b, int crc_mode, int mem) {
    for (int i = 0; i < n; i++)
        if (b[i].reserved) return JFSX_EINVAL;
    stub(1, n, crc_mode);
    for (int i = 0; i < n; i++) {
        bool ok = true;
        for (int k = 0; k < 16; k++)
            ok &= b[i].tag[k] == (uint8_t)(b[i].key[k] ^ (uint8_t)(b[i].len >> (8 * (k & 7))) ^ (uint8_t)algo);
        b[i].status = ok ? JFSX_OK : JFSX_ETAG;
    }
    return 0;
}

int jfsx_crc32c_segments(jfsx_ctx *, int n, jfsx_range *r, int mode, int mem) {
    stub(2, n, mode);
    for (int i = 0; i < n; i++) r[i].status = r[i].len % 7 == 3 ? JFSX_ECRC : JFSX_OK;
    return 0;
}

void harness_reset(int sleep_us) {
    std::lock_guard<std::mutex> g(h_mu);
    h_sizes.clear();
    h_ops.clear();
    h_modes.clear();
    h_sleep_us = sleep_us;
}

int harness_batches(int *sizes, int *ops, int *modes, int cap) {
    std::lock_guard<std::mutex> g(h_mu);
    const int n = (int)h_sizes.size();
    for (int i = 0; i < n && i < cap; i++) {
        sizes[i] = h_sizes[i];
        ops[i] = h_ops[i];
        modes[i] = h_modes[i];
    }
    return n;
}

// ctx_close's hook, for the async queue tests
void harness_close(jfsx_ctx *c) { jfsx::async_detach(c); }
}

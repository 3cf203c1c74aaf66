// Host build of the aggregator, the async queue and the multi-device context
// (juicefs_amd/csrc/jfsx_agg.cpp) over stub batch entry points, so their
// scheduling logic -- grouping, windows, size caps, error isolation, ordering,
// shutdown, the per-device split and the per-device dispatchers -- is testable
// without a GPU.  Fake devices are contexts 0x1000 + 0x100*d.
// The stubs record every batch they receive and compute a position-free fake
// "tag" so results can be matched to their requesters.
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <vector>

#include "../../juicefs_amd/csrc/jfsx_agg.cpp"

namespace {
std::mutex h_mu;
std::vector<int> h_sizes;   // blocks per batch, in issue order
std::vector<int> h_ops;     // 0 seal, 1 open, 2 crc, 3 lz4 compress, 4 lz4 decompress
std::vector<int> h_modes;
std::vector<intptr_t> h_ctxs;  // context of each batch
std::vector<uint64_t> h_first;  // len of the first block of each batch
std::vector<std::vector<uintptr_t>> h_srcs;  // src pointers of each AEAD batch, in order
int h_sleep_us = 2000;
int h_ndev = 4;
int h_open_ctx = 0;  // contexts opened and not closed

int stub(jfsx_ctx *c, int op, int n, int mode, uint64_t first_len = 0, const jfsx_blk *b = nullptr) {
    {
        std::lock_guard<std::mutex> g(h_mu);
        std::vector<uintptr_t> srcs;
        for (int i = 0; b && i < n; i++) srcs.push_back((uintptr_t)b[i].src);
        h_srcs.push_back(srcs);
        h_sizes.push_back(n);
        h_ops.push_back(op);
        h_modes.push_back(mode);
        h_ctxs.push_back((intptr_t)c);
        h_first.push_back(first_len);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(h_sleep_us));
    return 0;
}
}  // namespace

// Fake device memory: device d owns [(d+1) << 40, (d+2) << 40); anything
// below 1 << 40 is host memory.
namespace jfsx {
int device_of(const void *p, uintptr_t *lo, uintptr_t *hi) {
    const uintptr_t a = (uintptr_t)p;
    if (a < ((uintptr_t)1 << 40)) {
        *lo = a;
        *hi = a + 1;
        return -1;
    }
    const int d = (int)(a >> 40) - 1;
    *lo = (uintptr_t)(d + 1) << 40;
    *hi = (uintptr_t)(d + 2) << 40;
    return d;
}
// staging stubs: every host buffer counts as pinned unless the harness marks
// a range pageable (harness_pageable); bounce buffers are malloc'd
uintptr_t h_pg_lo = 0, h_pg_hi = 0;
std::atomic<int> h_bounces{0};
bool host_pinned(const void *p, uint64_t n) {
    const uintptr_t a = (uintptr_t)p;
    return !(a < h_pg_hi && a + n > h_pg_lo);
}
char *bounce_acquire(jfsx_ctx *, size_t need, size_t *cap) {
    h_bounces++;
    *cap = need;
    return (char *)malloc(need ? need : 1);
}
void bounce_release(jfsx_ctx *, char *p, size_t) { free(p); }
bool host_pin(const void *, uint64_t) { return false; }
void host_unpin(const void *) {}
void bounce_count(jfsx_ctx *, uint64_t, uint64_t) {}
}  // namespace jfsx

extern "C" {

// fake bytes of a host block with both pointers set: dst[j] = src[j] ^ key[j % 32]
// ^ 0x5A (its own inverse), so a test sees whether the staged copy reached
// the transform and its output came back to the caller's buffer
void fake_bytes(jfsx_blk &b) {
    const uint8_t *s = (const uint8_t *)b.src;
    uint8_t *d = (uint8_t *)b.dst;
    for (uint64_t j = 0; j < b.len; j++) d[j] = s[j] ^ b.key[j & 31] ^ 0x5A;
}

// fake transform: tag[i] = key[i] ^ (len >> 8*(i&7)); reserved != 0 -> EINVAL
int jfsx_seal_batch(jfsx_ctx *c, int algo, int n, jfsx_blk *b, int crc_mode, int mem) {
    for (int i = 0; i < n; i++)
        if (b[i].reserved) return JFSX_EINVAL;
    // fake device 3 fails device batches of 100-byte blocks
    if (mem == JFSX_MEM_DEVICE && (intptr_t)c == 0x1300 && n && b[0].len == 100) return JFSX_EIO;
    stub(c, 0, n, crc_mode, n ? b[0].len : 0, b);
    for (int i = 0; i < n; i++) {
        for (int k = 0; k < 16; k++) b[i].tag[k] = b[i].key[k] ^ (uint8_t)(b[i].len >> (8 * (k & 7))) ^ (uint8_t)algo;
        b[i].status = JFSX_OK;
        if (mem == JFSX_MEM_HOST && b[i].src && b[i].dst) fake_bytes(b[i]);
    }
    return 0;
}

int jfsx_open_batch(jfsx_ctx *c, int algo, int n, jfsx_blk *b, int crc_mode, int mem) {
    for (int i = 0; i < n; i++)
        if (b[i].reserved) return JFSX_EINVAL;
    stub(c, 1, n, crc_mode, n ? b[0].len : 0, b);
    for (int i = 0; i < n; i++) {
        bool ok = true;
        for (int k = 0; k < 16; k++)
            ok &= b[i].tag[k] == (uint8_t)(b[i].key[k] ^ (uint8_t)(b[i].len >> (8 * (k & 7))) ^ (uint8_t)algo);
        b[i].status = ok ? JFSX_OK : JFSX_ETAG;
        if (mem == JFSX_MEM_HOST && b[i].src && b[i].dst) {
            if (ok) fake_bytes(b[i]);
            else memset(b[i].dst, 0, b[i].len);  // the engine releases nothing of a failed block
        }
    }
    return 0;
}

int jfsx_crc32c_segments(jfsx_ctx *c, int n, jfsx_range *r, int mode, int mem) {
    stub(c, 2, n, mode, n ? r[0].len : 0);
    for (int i = 0; i < n; i++) r[i].status = r[i].len % 7 == 3 ? JFSX_ECRC : JFSX_OK;
    return 0;
}

// fake LZ4: out_len = src_len / 2 + 1 (compress), dst_cap (decompress);
// src_len == 7 -> JFSX_EFORMAT; dst_cap == 1 -> EINVAL (the batch is retried alone)
int jfsx_lz4_compress_batch(jfsx_ctx *c, int n, jfsx_zblk *z, int mem) {
    for (int i = 0; i < n; i++)
        if (z[i].dst_cap == 1) return JFSX_EINVAL;
    stub(c, 3, n, 0, n ? z[0].src_len : 0);
    for (int i = 0; i < n; i++) {
        z[i].out_len = z[i].src_len / 2 + 1;
        z[i].status = JFSX_OK;
    }
    return 0;
}

int jfsx_lz4_decompress_batch(jfsx_ctx *c, int n, jfsx_zblk *z, int mem) {
    stub(c, 4, n, 0, n ? z[0].src_len : 0);
    for (int i = 0; i < n; i++) {
        z[i].status = z[i].src_len == 7 ? JFSX_EFORMAT : JFSX_OK;
        z[i].out_len = z[i].status ? 0 : z[i].dst_cap;
    }
    return 0;
}

int jfsx_zstd_decompress_batch(jfsx_ctx *c, int n, jfsx_zblk *z, int mem) {
    stub(c, 5, n, 0, n ? z[0].src_len : 0);
    for (int i = 0; i < n; i++) {
        z[i].status = z[i].src_len == 7 ? JFSX_EFORMAT : JFSX_OK;
        z[i].out_len = z[i].status ? 0 : z[i].dst_cap;
    }
    return 0;
}

// fake zstd compress: out_len = src_len / 3 + 9
int jfsx_zstd_compress_batch(jfsx_ctx *c, int n, jfsx_zblk *z, int mem) {
    stub(c, 6, n, 0, n ? z[0].src_len : 0);
    for (int i = 0; i < n; i++) {
        z[i].out_len = z[i].src_len / 3 + 9;
        z[i].status = JFSX_OK;
    }
    return 0;
}

int jfsx_device_count(int *n) {
    *n = h_ndev;
    return h_ndev ? 0 : JFSX_ENODEV;
}

int jfsx_ctx_open(int device, uint32_t flags, jfsx_ctx **out) {
    if (device < 0 || device >= h_ndev) return JFSX_ENODEV;
    std::lock_guard<std::mutex> g(h_mu);
    h_open_ctx++;
    *out = (jfsx_ctx *)(intptr_t)(0x1000 + 0x100 * device);
    return 0;
}

int jfsx_ctx_close(jfsx_ctx *) {
    std::lock_guard<std::mutex> g(h_mu);
    h_open_ctx--;
    return 0;
}

void harness_reset(int sleep_us) {
    std::lock_guard<std::mutex> g(h_mu);
    h_srcs.clear();
    h_sizes.clear();
    h_ops.clear();
    h_modes.clear();
    h_ctxs.clear();
    h_first.clear();
    h_sleep_us = sleep_us;
}

void harness_set_ndev(int n) { h_ndev = n; }
// mark [lo, hi) pageable (host_pinned() false there; 0, 0: none); bounce
// buffers (and staging arenas) allocated so far
void harness_pageable(uintptr_t lo, uintptr_t hi) {
    jfsx::h_pg_lo = lo;
    jfsx::h_pg_hi = hi;
}
int harness_bounces(void) { return jfsx::h_bounces.load(); }
int harness_open_ctx(void) { return h_open_ctx; }

// per batch: device index of its context and the len of its first block
int harness_batch_devs(int *dev, uint64_t *first, int cap) {
    std::lock_guard<std::mutex> g(h_mu);
    const int n = (int)h_ctxs.size();
    for (int i = 0; i < n && i < cap; i++) {
        dev[i] = (int)((h_ctxs[i] - 0x1000) / 0x100);
        first[i] = h_first[i];
    }
    return n;
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

// src pointers of AEAD batch `batch` (issue order); returns how many
int harness_batch_srcs(int batch, uintptr_t *out, int cap) {
    std::lock_guard<std::mutex> g(h_mu);
    if (batch < 0 || batch >= (int)h_srcs.size()) return -1;
    const std::vector<uintptr_t> &v = h_srcs[batch];
    for (int i = 0; i < (int)v.size() && i < cap; i++) out[i] = v[i];
    return (int)v.size();
}

// ctx_close's hook, for the async queue tests
void harness_close(jfsx_ctx *c) { jfsx::async_detach(c); }
}

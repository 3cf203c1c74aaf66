// jfsx_agg.cpp -- asynchronous batches, the per-block aggregator and the
// multi-device context (host C++; only the public C-ABI below it is used).
//
// The reference encrypts and decrypts one block per call, synchronously, from
// many goroutines at once: Encrypt from up to max-uploads (default 20,
// cmd/flags.go:126-127) uploaders plus the staging uploader
// (pkg/chunk/cached_store.go:824-826), Decrypt from reader goroutines, the
// prefetcher and warmup workers (cached_store.go:185, :813-821; fill.go:64-90).
// The engine is fast only on batches, so this file provides the two pieces a
// drop-in needs between those callers and jfsx_seal_batch/jfsx_open_batch
// (SURVEY §8b "Sync and _async + jfsx_wait variants", §8f-2 "batching
// aggregator"):
//
//   * jfsx_*_async + jfsx_wait: a batch is queued on the context's worker
//     thread and the call returns a ticket at once.
//   * jfsx_agg: per-block calls that block the calling thread (the shape of
//     dataEncryptor.Encrypt / Decrypt, encrypt.go:164-216, and of the
//     cacheFile.ReadAt verify, disk_cache.go:1315-1327) are coalesced by a
//     dispatcher thread into batches of compatible requests (same op, algo,
//     crc mode, memory kind), bounded by a block count, a byte count and a
//     time window measured from the oldest waiting request.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "jfsx.h"

namespace {

using Clock = std::chrono::steady_clock;

// ---------------------------------------------------------------------------
// per-context worker for the _async entry points

struct Job {
    std::function<int()> fn;
    int rc = 0;
    bool done = false;
};

struct AsyncQ {
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::deque<std::shared_ptr<Job>> q;
    std::map<uint64_t, std::shared_ptr<Job>> live;  // submitted, not yet waited for
    uint64_t next = 1;
    bool stop = false;
    std::thread th;

    void run() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv_work.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;  // stop, and nothing left to run
            std::shared_ptr<Job> j = q.front();
            q.pop_front();
            lk.unlock();
            const int rc = j->fn();
            lk.lock();
            j->rc = rc;
            j->done = true;
            cv_done.notify_all();
        }
    }
};

std::mutex g_mu;
std::map<const jfsx_ctx *, AsyncQ *> g_async;

AsyncQ *async_of(jfsx_ctx *c) {
    std::lock_guard<std::mutex> g(g_mu);
    AsyncQ *&a = g_async[c];
    if (!a) {
        a = new AsyncQ;
        a->th = std::thread([a] { a->run(); });
    }
    return a;
}

int submit(jfsx_ctx *c, std::function<int()> fn, jfsx_ticket *t) {
    if (!c || !t) return JFSX_EINVAL;
    AsyncQ *a = async_of(c);
    auto j = std::make_shared<Job>();
    j->fn = std::move(fn);
    std::lock_guard<std::mutex> g(a->mu);
    if (a->stop) return JFSX_EINVAL;
    *t = a->next++;
    a->live[*t] = j;
    a->q.push_back(j);
    a->cv_work.notify_one();
    return 0;
}

bool valid_algo(int algo) { return algo == JFSX_AES256GCM || algo == JFSX_CHACHA20P1305; }
bool valid_mem(int mem) { return mem == JFSX_MEM_DEVICE || mem == JFSX_MEM_HOST; }

}  // namespace

namespace jfsx {
// jfsx_ctx_close: run what is queued, then stop the worker (before the
// context's streams and buffers go away)
void async_detach(jfsx_ctx *c) {
    AsyncQ *a = nullptr;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_async.find(c);
        if (it == g_async.end()) return;
        a = it->second;
        g_async.erase(it);
    }
    {
        std::lock_guard<std::mutex> g(a->mu);
        a->stop = true;
        a->cv_work.notify_all();
    }
    a->th.join();
    delete a;
}
}  // namespace jfsx

extern "C" {

int jfsx_seal_batch_async(jfsx_ctx *c, int algo, int n, jfsx_blk *blks, int crc_mode, int mem, jfsx_ticket *t) {
    return submit(c, [=] { return jfsx_seal_batch(c, algo, n, blks, crc_mode, mem); }, t);
}

int jfsx_open_batch_async(jfsx_ctx *c, int algo, int n, jfsx_blk *blks, int crc_mode, int mem, jfsx_ticket *t) {
    return submit(c, [=] { return jfsx_open_batch(c, algo, n, blks, crc_mode, mem); }, t);
}

int jfsx_crc32c_segments_async(jfsx_ctx *c, int n, jfsx_range *ranges, int mode, int mem, jfsx_ticket *t) {
    return submit(c, [=] { return jfsx_crc32c_segments(c, n, ranges, mode, mem); }, t);
}

int jfsx_wait(jfsx_ctx *c, jfsx_ticket t, int timeout_ms) {
    if (!c) return JFSX_EINVAL;
    AsyncQ *a;
    {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = g_async.find(c);
        if (it == g_async.end()) return JFSX_EINVAL;
        a = it->second;
    }
    std::unique_lock<std::mutex> lk(a->mu);
    auto it = a->live.find(t);
    if (it == a->live.end()) return JFSX_EINVAL;
    std::shared_ptr<Job> j = it->second;
    auto ready = [&] { return j->done; };
    if (timeout_ms < 0)
        a->cv_done.wait(lk, ready);
    else if (!a->cv_done.wait_for(lk, std::chrono::milliseconds(timeout_ms), ready))
        return JFSX_EAGAIN;
    a->live.erase(t);
    return j->rc;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// aggregator

namespace jfsx {

enum AggOp { kSeal = 0, kOpen = 1, kCrc = 2, kLz4c = 3, kLz4d = 4, kZstdd = 5, kZstdc = 6 };

struct Req {
    int op, algo, mode, mem;
    jfsx_blk *blk;
    jfsx_range *range;
    jfsx_zblk *z;
    uint64_t bytes;
    Clock::time_point t0;
    int rc = 0;
    bool done = false;
    bool same(const Req &o) const { return op == o.op && algo == o.algo && mode == o.mode && mem == o.mem; }
};

}  // namespace jfsx

using jfsx::Req;
using jfsx::kSeal;
using jfsx::kOpen;
using jfsx::kCrc;
using jfsx::kLz4c;
using jfsx::kLz4d;
using jfsx::kZstdd;
using jfsx::kZstdc;

struct jfsx_agg {
    std::vector<jfsx_ctx *> cs;  // one dispatcher thread per context (device)
    int max_blocks;
    uint64_t max_bytes;
    std::chrono::microseconds window;
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::deque<Req *> q;
    bool stop = false;
    uint64_t calls = 0, batches = 0, blocks = 0;
    std::vector<uint64_t> dev_batches;
    std::vector<std::thread> ths;

    int call(jfsx_ctx *c, const std::vector<Req *> &b, size_t i0, size_t n, std::vector<jfsx_blk> &blks,
             std::vector<jfsx_range> &rng, std::vector<jfsx_zblk> &zs) {
        const Req &h = *b[i0];
        if (h.op == kCrc) return jfsx_crc32c_segments(c, (int)n, rng.data() + i0, h.mode, h.mem);
        if (h.op == kLz4c) return jfsx_lz4_compress_batch(c, (int)n, zs.data() + i0, h.mem);
        if (h.op == kLz4d) return jfsx_lz4_decompress_batch(c, (int)n, zs.data() + i0, h.mem);
        if (h.op == kZstdd) return jfsx_zstd_decompress_batch(c, (int)n, zs.data() + i0, h.mem);
        if (h.op == kZstdc) return jfsx_zstd_compress_batch(c, (int)n, zs.data() + i0, h.mem);
        if (h.op == kSeal) return jfsx_seal_batch(c, h.algo, (int)n, blks.data() + i0, h.mode, h.mem);
        return jfsx_open_batch(c, h.algo, (int)n, blks.data() + i0, h.mode, h.mem);
    }

    // one engine call for the whole group; if the engine rejects the batch
    // (an argument error in one request), every request is retried alone so
    // the error reaches only its own caller
    void execute(jfsx_ctx *c, std::vector<Req *> &b) {
        const size_t n = b.size();
        std::vector<jfsx_blk> blks;
        std::vector<jfsx_range> rng;
        std::vector<jfsx_zblk> zs;
        const int op = b[0]->op;
        if (op == kCrc) {
            rng.resize(n);
            for (size_t i = 0; i < n; i++) rng[i] = *b[i]->range;
        } else if (op == kLz4c || op == kLz4d || op == kZstdd || op == kZstdc) {
            zs.resize(n);
            for (size_t i = 0; i < n; i++) zs[i] = *b[i]->z;
        } else {
            blks.resize(n);
            for (size_t i = 0; i < n; i++) blks[i] = *b[i]->blk;
        }
        int rc = call(c, b, 0, n, blks, rng, zs);
        if (rc == JFSX_EINVAL && n > 1) {
            for (size_t i = 0; i < n; i++) b[i]->rc = call(c, b, i, 1, blks, rng, zs);
        } else {
            for (size_t i = 0; i < n; i++) b[i]->rc = rc;
        }
        for (size_t i = 0; i < n; i++) {
            if (op == kCrc)
                *b[i]->range = rng[i];
            else if (op == kLz4c || op == kLz4d || op == kZstdd || op == kZstdc)
                *b[i]->z = zs[i];
            else
                *b[i]->blk = blks[i];
        }
    }

    // Dispatcher k: take the group of the oldest request once it is full (block
    // or byte cap) or its window has closed, run it on context k.  Several
    // dispatchers share the queue: after every wait the head is re-read, since
    // another dispatcher may have taken the group in the meantime.
    void run(int k) {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv_work.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;  // stop, and nothing left to run
            const Req *head = q.front();
            int cnt = 0;
            uint64_t bytes = 0;
            for (Req *r : q)
                if (r->same(*head)) cnt++, bytes += r->bytes;
            const Clock::time_point deadline = head->t0 + window;
            if (!(stop || cnt >= max_blocks || bytes >= max_bytes || Clock::now() >= deadline)) {
                cv_work.wait_until(lk, deadline);
                continue;
            }
            std::vector<Req *> b;
            bytes = 0;
            const Req h = *head;
            for (auto it = q.begin(); it != q.end() && (int)b.size() < max_blocks;) {
                if ((*it)->same(h) && (b.empty() || bytes + (*it)->bytes <= max_bytes)) {
                    bytes += (*it)->bytes;
                    b.push_back(*it);
                    it = q.erase(it);
                } else {
                    ++it;
                }
            }
            if (!q.empty()) cv_work.notify_all();  // the next group may be ready for an idle dispatcher
            lk.unlock();
            execute(cs[k], b);
            lk.lock();
            batches++;
            dev_batches[k]++;
            blocks += b.size();
            for (Req *r : b) r->done = true;
            cv_done.notify_all();
        }
    }

    int submit(Req &r) {
        std::unique_lock<std::mutex> lk(mu);
        if (stop) return JFSX_EINVAL;
        r.t0 = Clock::now();
        q.push_back(&r);
        calls++;
        cv_work.notify_one();
        cv_done.wait(lk, [&] { return r.done; });
        return r.rc;
    }
};

namespace {
int agg_start(std::vector<jfsx_ctx *> cs, int max_blocks, uint64_t max_bytes, uint32_t window_us, jfsx_agg **out) {
    jfsx_agg *a = new (std::nothrow) jfsx_agg;
    if (!a) return JFSX_ENOMEM;
    a->cs = std::move(cs);
    a->max_blocks = max_blocks ? max_blocks : 256;
    a->max_bytes = max_bytes ? max_bytes : (uint64_t)1 << 30;
    a->window = std::chrono::microseconds(window_us);
    a->dev_batches.assign(a->cs.size(), 0);
    for (size_t k = 0; k < a->cs.size(); k++) a->ths.emplace_back([a, k] { a->run((int)k); });
    *out = a;
    return 0;
}
// device pointers belong to one GPU: over a multi-device context any
// dispatcher may take a group, so only host memory is accepted there (as the
// jfsx_mctx_*_batch entry points do)
bool agg_mem_ok(const jfsx_agg *a, int mem) {
    return valid_mem(mem) && !(mem == JFSX_MEM_DEVICE && a->cs.size() > 1);
}
}  // namespace

extern "C" {

int jfsx_agg_new(jfsx_ctx *c, int max_blocks, uint64_t max_bytes, uint32_t window_us, jfsx_agg **out) {
    if (!c || !out || max_blocks < 0) return JFSX_EINVAL;
    return agg_start({c}, max_blocks, max_bytes, window_us, out);
}

int jfsx_agg_free(jfsx_agg *a) {
    if (!a) return JFSX_EINVAL;
    {
        std::lock_guard<std::mutex> g(a->mu);
        a->stop = true;
        a->cv_work.notify_all();
    }
    for (std::thread &t : a->ths) t.join();  // requests already queued run first
    delete a;
    return 0;
}

int jfsx_agg_dev_batches(jfsx_agg *a, int i, uint64_t *batches) {
    if (!a || !batches || i < 0) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(a->mu);
    if ((size_t)i >= a->dev_batches.size()) return JFSX_EINVAL;
    *batches = a->dev_batches[i];
    return 0;
}

int jfsx_agg_seal(jfsx_agg *a, int algo, jfsx_blk *blk, int crc_mode, int mem) {
    if (!a || !blk || !valid_algo(algo) || !agg_mem_ok(a, mem)) return JFSX_EINVAL;
    Req r{kSeal, algo, crc_mode, mem, blk, nullptr, nullptr, blk->len};
    return a->submit(r);
}

int jfsx_agg_open(jfsx_agg *a, int algo, jfsx_blk *blk, int crc_mode, int mem) {
    if (!a || !blk || !valid_algo(algo) || !agg_mem_ok(a, mem)) return JFSX_EINVAL;
    Req r{kOpen, algo, crc_mode, mem, blk, nullptr, nullptr, blk->len};
    return a->submit(r);
}

int jfsx_agg_crc32c(jfsx_agg *a, jfsx_range *range, int mode, int mem) {
    if (!a || !range || !agg_mem_ok(a, mem) || (mode != JFSX_CRC_GEN && mode != JFSX_CRC_VERIFY)) return JFSX_EINVAL;
    Req r{kCrc, 0, mode, mem, nullptr, range, nullptr, range->len};
    return a->submit(r);
}

int jfsx_agg_lz4_compress(jfsx_agg *a, jfsx_zblk *z, int mem) {
    if (!a || !z || !agg_mem_ok(a, mem)) return JFSX_EINVAL;
    Req r{kLz4c, 0, 0, mem, nullptr, nullptr, z, z->src_len};
    return a->submit(r);
}

int jfsx_agg_lz4_decompress(jfsx_agg *a, jfsx_zblk *z, int mem) {
    if (!a || !z || !agg_mem_ok(a, mem)) return JFSX_EINVAL;
    Req r{kLz4d, 0, 0, mem, nullptr, nullptr, z, z->dst_cap};
    return a->submit(r);
}

int jfsx_agg_zstd_decompress(jfsx_agg *a, jfsx_zblk *z, int mem) {
    if (!a || !z || !agg_mem_ok(a, mem)) return JFSX_EINVAL;
    Req r{kZstdd, 0, 0, mem, nullptr, nullptr, z, z->dst_cap};
    return a->submit(r);
}

int jfsx_agg_zstd_compress(jfsx_agg *a, jfsx_zblk *z, int mem) {
    if (!a || !z || !agg_mem_ok(a, mem)) return JFSX_EINVAL;
    Req r{kZstdc, 0, 0, mem, nullptr, nullptr, z, z->src_len};
    return a->submit(r);
}

int jfsx_agg_stats(jfsx_agg *a, uint64_t *calls, uint64_t *batches, uint64_t *blocks) {
    if (!a) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(a->mu);
    if (calls) *calls = a->calls;
    if (batches) *batches = a->batches;
    if (blocks) *blocks = a->blocks;
    return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// multi-device context (SURVEY §8b jfsx_open_ctx(dev_mask), §8e): one jfsx_ctx
// per GPU, built on the public single-device entry points only

struct jfsx_mctx {
    std::vector<jfsx_ctx *> cs;
};

namespace {

// contiguous runs of blocks, one per device, balanced by bytes: run k is
// [cut[k], cut[k+1]).  With n >= nd every device gets at least one block
// (a lone giant block still goes to one device).
std::vector<int> split_runs(int n, int nd, const std::function<uint64_t(int)> &len) {
    std::vector<int> cut(nd + 1, n);
    cut[0] = 0;
    uint64_t total = 0;
    for (int i = 0; i < n; i++) total += len(i) + 1;  // +1: empty blocks still count
    uint64_t acc = 0;
    int i = 0;
    for (int k = 1; k < nd; k++) {
        const uint64_t target = total * (uint64_t)k / (uint64_t)nd;
        const int keep = n - (nd - k);  // leave one block for each later run
        if (i < n && i == cut[k - 1]) acc += len(i) + 1, i++;  // at least one block per run
        while (i < keep && acc + (len(i) + 1) / 2 <= target) acc += len(i) + 1, i++;
        cut[k] = i;
    }
    return cut;
}

// run f(k, b0, b1) for every non-empty run, device 0's on the calling thread
int fan_out(const std::vector<int> &cut, const std::function<int(int, int, int)> &f) {
    const int nd = (int)cut.size() - 1;
    std::vector<int> rc(nd, 0);
    std::vector<std::thread> th;
    for (int k = 1; k < nd; k++)
        if (cut[k + 1] > cut[k]) th.emplace_back([&, k] { rc[k] = f(k, cut[k], cut[k + 1]); });
    if (cut[1] > cut[0]) rc[0] = f(0, cut[0], cut[1]);
    for (std::thread &t : th) t.join();
    for (int k = 0; k < nd; k++)
        if (rc[k]) return rc[k];
    return 0;
}

int mctx_aead(jfsx_mctx *m, bool open, int algo, int n, jfsx_blk *blks, int crc_mode, int mem) {
    if (!m || n < 0 || (n && !blks)) return JFSX_EINVAL;
    if (mem != JFSX_MEM_HOST && !(mem == JFSX_MEM_DEVICE && m->cs.size() == 1)) return JFSX_EINVAL;
    if (n == 0) return 0;
    const std::vector<int> cut = split_runs(n, (int)m->cs.size(), [&](int i) { return blks[i].len; });
    return fan_out(cut, [&](int k, int b0, int b1) {
        return open ? jfsx_open_batch(m->cs[k], algo, b1 - b0, blks + b0, crc_mode, mem)
                    : jfsx_seal_batch(m->cs[k], algo, b1 - b0, blks + b0, crc_mode, mem);
    });
}

}  // namespace

extern "C" {

int jfsx_mctx_open(uint64_t dev_mask, uint32_t flags, jfsx_mctx **out) {
    if (!out) return JFSX_EINVAL;
    *out = nullptr;
    int nd = 0;
    if (jfsx_device_count(&nd) || nd <= 0) return JFSX_ENODEV;
    if (nd < 64 && (dev_mask >> nd)) return JFSX_ENODEV;  // a selected device is not visible
    jfsx_mctx *m = new (std::nothrow) jfsx_mctx;
    if (!m) return JFSX_ENOMEM;
    for (int d = 0; d < nd && d < 64; d++) {
        if (dev_mask && !((dev_mask >> d) & 1)) continue;
        jfsx_ctx *c = nullptr;
        const int rc = jfsx_ctx_open(d, flags, &c);
        if (rc) {
            jfsx_mctx_close(m);
            return rc;
        }
        m->cs.push_back(c);
    }
    *out = m;
    return 0;
}

int jfsx_mctx_close(jfsx_mctx *m) {
    if (!m) return JFSX_EINVAL;
    for (jfsx_ctx *c : m->cs) jfsx_ctx_close(c);
    delete m;
    return 0;
}

int jfsx_mctx_ndev(jfsx_mctx *m) { return m ? (int)m->cs.size() : 0; }

jfsx_ctx *jfsx_mctx_ctx(jfsx_mctx *m, int i) {
    return m && i >= 0 && (size_t)i < m->cs.size() ? m->cs[i] : nullptr;
}

int jfsx_mctx_seal_batch(jfsx_mctx *m, int algo, int n, jfsx_blk *blks, int crc_mode, int mem) {
    return mctx_aead(m, false, algo, n, blks, crc_mode, mem);
}

int jfsx_mctx_open_batch(jfsx_mctx *m, int algo, int n, jfsx_blk *blks, int crc_mode, int mem) {
    return mctx_aead(m, true, algo, n, blks, crc_mode, mem);
}

int jfsx_mctx_crc32c_segments(jfsx_mctx *m, int n, jfsx_range *ranges, int mode, int mem) {
    if (!m || n < 0 || (n && !ranges)) return JFSX_EINVAL;
    if (mem != JFSX_MEM_HOST && !(mem == JFSX_MEM_DEVICE && m->cs.size() == 1)) return JFSX_EINVAL;
    if (n == 0) return 0;
    const std::vector<int> cut = split_runs(n, (int)m->cs.size(), [&](int i) { return ranges[i].len; });
    return fan_out(cut, [&](int k, int b0, int b1) {
        return jfsx_crc32c_segments(m->cs[k], b1 - b0, ranges + b0, mode, mem);
    });
}

static int mctx_lz4(jfsx_mctx *m, int op, int n, jfsx_zblk *z, int mem) {
    if (!m || n < 0 || (n && !z)) return JFSX_EINVAL;
    if (mem != JFSX_MEM_HOST && !(mem == JFSX_MEM_DEVICE && m->cs.size() == 1)) return JFSX_EINVAL;
    if (n == 0) return 0;
    const std::vector<int> cut = split_runs(n, (int)m->cs.size(), [&](int i) { return z[i].src_len; });
    return fan_out(cut, [&](int k, int b0, int b1) {
        return op == kLz4c   ? jfsx_lz4_compress_batch(m->cs[k], b1 - b0, z + b0, mem)
               : op == kLz4d ? jfsx_lz4_decompress_batch(m->cs[k], b1 - b0, z + b0, mem)
               : op == kZstdc ? jfsx_zstd_compress_batch(m->cs[k], b1 - b0, z + b0, mem)
                              : jfsx_zstd_decompress_batch(m->cs[k], b1 - b0, z + b0, mem);
    });
}

int jfsx_mctx_lz4_compress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) { return mctx_lz4(m, kLz4c, n, blks, mem); }
int jfsx_mctx_lz4_decompress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) {
    return mctx_lz4(m, kLz4d, n, blks, mem);
}
int jfsx_mctx_zstd_decompress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) {
    return mctx_lz4(m, kZstdd, n, blks, mem);
}

int jfsx_mctx_zstd_compress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) {
    return mctx_lz4(m, kZstdc, n, blks, mem);
}

int jfsx_agg_new_mctx(jfsx_mctx *m, int max_blocks, uint64_t max_bytes, uint32_t window_us, jfsx_agg **out) {
    if (!m || m->cs.empty() || !out || max_blocks < 0) return JFSX_EINVAL;
    return agg_start(m->cs, max_blocks, max_bytes, window_us, out);
}

}  // extern "C"

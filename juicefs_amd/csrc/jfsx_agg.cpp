// jfsx_agg.cpp -- asynchronous batches and the per-block aggregator (host C++).
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

enum AggOp { kSeal = 0, kOpen = 1, kCrc = 2 };

struct Req {
    int op, algo, mode, mem;
    jfsx_blk *blk;
    jfsx_range *range;
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

struct jfsx_agg {
    jfsx_ctx *c;
    int max_blocks;
    uint64_t max_bytes;
    std::chrono::microseconds window;
    std::mutex mu;
    std::condition_variable cv_work, cv_done;
    std::deque<Req *> q;
    bool stop = false;
    uint64_t calls = 0, batches = 0, blocks = 0;
    std::thread th;

    int call(const std::vector<Req *> &b, size_t i0, size_t n, std::vector<jfsx_blk> &blks,
             std::vector<jfsx_range> &rng) {
        const Req &h = *b[i0];
        if (h.op == kCrc) return jfsx_crc32c_segments(c, (int)n, rng.data() + i0, h.mode, h.mem);
        if (h.op == kSeal) return jfsx_seal_batch(c, h.algo, (int)n, blks.data() + i0, h.mode, h.mem);
        return jfsx_open_batch(c, h.algo, (int)n, blks.data() + i0, h.mode, h.mem);
    }

    // one engine call for the whole group; if the engine rejects the batch
    // (an argument error in one request), every request is retried alone so
    // the error reaches only its own caller
    void execute(std::vector<Req *> &b) {
        const size_t n = b.size();
        std::vector<jfsx_blk> blks;
        std::vector<jfsx_range> rng;
        if (b[0]->op == kCrc) {
            rng.resize(n);
            for (size_t i = 0; i < n; i++) rng[i] = *b[i]->range;
        } else {
            blks.resize(n);
            for (size_t i = 0; i < n; i++) blks[i] = *b[i]->blk;
        }
        int rc = call(b, 0, n, blks, rng);
        if (rc == JFSX_EINVAL && n > 1) {
            for (size_t i = 0; i < n; i++) b[i]->rc = call(b, i, 1, blks, rng);
        } else {
            for (size_t i = 0; i < n; i++) b[i]->rc = rc;
        }
        for (size_t i = 0; i < n; i++) {
            if (b[i]->op == kCrc)
                *b[i]->range = rng[i];
            else
                *b[i]->blk = blks[i];
        }
    }

    void run() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv_work.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;
            // wait for the group of the oldest request to fill, or its window to close
            const Clock::time_point deadline = q.front()->t0 + window;
            for (;;) {
                int cnt = 0;
                uint64_t bytes = 0;
                for (Req *r : q)
                    if (r->same(*q.front())) cnt++, bytes += r->bytes;
                if (stop || cnt >= max_blocks || bytes >= max_bytes || Clock::now() >= deadline) break;
                cv_work.wait_until(lk, deadline);
            }
            std::vector<Req *> b;
            uint64_t bytes = 0;
            const Req head = *q.front();
            for (auto it = q.begin(); it != q.end() && (int)b.size() < max_blocks;) {
                if ((*it)->same(head) && (b.empty() || bytes + (*it)->bytes <= max_bytes)) {
                    bytes += (*it)->bytes;
                    b.push_back(*it);
                    it = q.erase(it);
                } else {
                    ++it;
                }
            }
            lk.unlock();
            execute(b);
            lk.lock();
            batches++;
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

extern "C" {

int jfsx_agg_new(jfsx_ctx *c, int max_blocks, uint64_t max_bytes, uint32_t window_us, jfsx_agg **out) {
    if (!c || !out || max_blocks < 0) return JFSX_EINVAL;
    jfsx_agg *a = new (std::nothrow) jfsx_agg;
    if (!a) return JFSX_ENOMEM;
    a->c = c;
    a->max_blocks = max_blocks ? max_blocks : 256;
    a->max_bytes = max_bytes ? max_bytes : (uint64_t)1 << 30;
    a->window = std::chrono::microseconds(window_us);
    a->th = std::thread([a] { a->run(); });
    *out = a;
    return 0;
}

int jfsx_agg_free(jfsx_agg *a) {
    if (!a) return JFSX_EINVAL;
    {
        std::lock_guard<std::mutex> g(a->mu);
        a->stop = true;
        a->cv_work.notify_all();
    }
    a->th.join();  // requests already queued run first
    delete a;
    return 0;
}

int jfsx_agg_seal(jfsx_agg *a, int algo, jfsx_blk *blk, int crc_mode, int mem) {
    if (!a || !blk || !valid_algo(algo) || !valid_mem(mem)) return JFSX_EINVAL;
    Req r{kSeal, algo, crc_mode, mem, blk, nullptr, blk->len};
    return a->submit(r);
}

int jfsx_agg_open(jfsx_agg *a, int algo, jfsx_blk *blk, int crc_mode, int mem) {
    if (!a || !blk || !valid_algo(algo) || !valid_mem(mem)) return JFSX_EINVAL;
    Req r{kOpen, algo, crc_mode, mem, blk, nullptr, blk->len};
    return a->submit(r);
}

int jfsx_agg_crc32c(jfsx_agg *a, jfsx_range *range, int mode, int mem) {
    if (!a || !range || !valid_mem(mem) || (mode != JFSX_CRC_GEN && mode != JFSX_CRC_VERIFY)) return JFSX_EINVAL;
    Req r{kCrc, 0, mode, mem, nullptr, range, range->len};
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

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
#include <algorithm>
#include <cstdint>
#include <cstdlib>
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
    // completion: each caller sleeps on its own condition variable, so a
    // finished batch wakes only its own callers (not every waiting caller,
    // which would contend on the queue lock the dispatchers need)
    std::mutex m;
    std::condition_variable cv;
    bool fin = false;
    bool same(const Req &o) const { return op == o.op && algo == o.algo && mode == o.mode && mem == o.mem; }
};

}  // namespace jfsx

// A pinned staging arena shared by the pageable per-object requests of one
// aggregator (see Staged): callers take consecutive 256-byte-aligned slices,
// so the blocks of one batch usually sit side by side in one allocation and
// the engine moves them with one H2D and one D2H copy instead of one per block
// (large copies run nearer the link's rate than 4 MiB ones).
struct AggArena {
    char *base;
    size_t cap, used;
    int refs;   // slices still held by requests
    bool open;  // the arena slices are taken from now
};

namespace {
// pipelined batches that may run before small groups start to wait for more
// bytes (JFSX_AGG_INFLIGHT, default 3), and the group size that goes at once
// whatever runs (JFSX_AGG_FILL_MB, default 4: one 4 MiB block)
int pipe_inflight() {
    static const int v = [] {
        const char *e = getenv("JFSX_AGG_INFLIGHT");
        const int t = e ? atoi(e) : 3;  // 2 before the keysetup stream (profiles/r6/ab_small/)
        return t >= 1 ? t : 3;
    }();
    return v;
}
uint64_t pipe_fill() {
    static const uint64_t v = [] {
        const char *e = getenv("JFSX_AGG_FILL_MB");
        return (uint64_t)(e ? atof(e) * 1048576.0 : 4194304.0);
    }();
    return v;
}
}  // namespace

using jfsx::Req;
using jfsx::kSeal;
using jfsx::kOpen;
using jfsx::kCrc;
using jfsx::kLz4c;
using jfsx::kLz4d;
using jfsx::kZstdd;
using jfsx::kZstdc;

struct jfsx_agg {
    std::vector<jfsx_ctx *> cs;  // context of each dispatcher thread
    std::vector<int> dev;        // device slot (jfsx_agg_dev_batches) of each dispatcher
    int max_blocks;
    uint64_t max_bytes;
    std::chrono::microseconds window;
    std::mutex mu;
    std::condition_variable cv_work;
    std::deque<Req *> q;
    bool stop = false;
    int busy = 0;             // dispatchers running a pipelined batch
    Clock::time_point last_done{};  // when the last pipelined batch finished
    std::vector<int> serial;  // per device: dispatchers running a non-pipelined batch
    uint64_t calls = 0, batches = 0, blocks = 0;
    std::vector<uint64_t> dev_batches;
    std::vector<std::thread> ths;
    // staging arenas (arena_reserve / arena_release)
    std::mutex ar_mu;
    AggArena *ar_cur = nullptr;
    std::vector<AggArena *> ar_free, ar_all;

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

    // Host-memory Seal / Open / CRC calls pipeline through the context
    // (jfsx_seal_batch, jfsx_crc32c_segments): several such batches of one
    // device run at once.  Everything else holds its context for the whole
    // call, so a device runs one of those at a time.
    static bool piped(const Req &r) { return (r.op == kSeal || r.op == kOpen || r.op == kCrc) && r.mem == JFSX_MEM_HOST; }

    // Dispatcher k: take the group of the oldest request once it is full (block
    // or byte cap) or its window has closed -- or, for a pipelined group, as
    // soon as the engine is streaming: another pipelined batch is running, or
    // one finished within the window (the time the group spent queued behind
    // that batch was its batching, and holding it longer would only idle the
    // pipeline).  While pipe_inflight() pipelined batches already run, a group
    // of small blocks waits for pipe_fill() bytes, its window or the end of a
    // running batch instead: every group costs the compute stream a fixed
    // keysetup / main / finalize sequence (about 0.14 ms for a handful of
    // 64 KiB blocks), so small blocks travel in fewer, larger groups.  Then
    // run the group on context cs[k].  A
    // non-pipelined group waits while its device runs another one, so requests
    // arriving meanwhile join one batch instead of several small ones.  The
    // dispatchers share the queue: after every wait the head is re-read, since
    // another dispatcher may have taken the group in the meantime.
    void run(int k) {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv_work.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;  // stop, and nothing left to run
            const Req *head = q.front();
            const bool pipe = piped(*head);
            if (!pipe && !stop && serial[dev[k]] > 0) {
                cv_work.wait(lk);
                continue;
            }
            int cnt = 0;
            uint64_t bytes = 0;
            for (Req *r : q)
                if (r->same(*head)) cnt++, bytes += r->bytes;
            const Clock::time_point now = Clock::now(), deadline = head->t0 + window;
            const bool streaming = busy > 0 || (last_done != Clock::time_point{} && now - last_done < window);
            const bool pipe_go = pipe && streaming && (busy < pipe_inflight() || bytes >= pipe_fill());
            if (!(stop || pipe_go || cnt >= max_blocks || bytes >= max_bytes || now >= deadline)) {
                cv_work.wait_until(lk, deadline);
                continue;
            }
            std::vector<Req *> b;
            bytes = 0;
            const Req *h = head;  // still alive: its caller waits until the batch is done
            for (auto it = q.begin(); it != q.end() && (int)b.size() < max_blocks;) {
                if ((*it)->same(*h) && (b.empty() || bytes + (*it)->bytes <= max_bytes)) {
                    bytes += (*it)->bytes;
                    b.push_back(*it);
                    it = q.erase(it);
                } else {
                    ++it;
                }
            }
            int &held = pipe ? busy : serial[dev[k]];
            held++;
            if (!q.empty()) cv_work.notify_all();  // the rest may go to an idle dispatcher now
            lk.unlock();
            execute(cs[k], b);
            // the counters first: a caller that has returned sees its batch
            // counted (jfsx_agg_stats right after the last call returns)
            lk.lock();
            held--;
            if (pipe) last_done = Clock::now();
            batches++;
            dev_batches[dev[k]]++;
            blocks += b.size();
            lk.unlock();
            for (Req *r : b) {
                std::lock_guard<std::mutex> g(r->m);  // r may be gone once fin is seen: notify under its lock
                r->fin = true;
                r->cv.notify_one();
            }
            lk.lock();
            if (!q.empty()) cv_work.notify_all();
        }
    }

    int submit(Req &r) {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (stop) return JFSX_EINVAL;
            r.t0 = Clock::now();
            q.push_back(&r);
            calls++;
            cv_work.notify_one();
        }
        std::unique_lock<std::mutex> l2(r.m);
        r.cv.wait(l2, [&] { return r.fin; });
        return r.rc;
    }
};

namespace jfsx {
// pinned staging of pageable caller memory (jfsx_api.cpp; the host harness
// stubs them)
bool host_pinned(const void *p, uint64_t n);
bool host_pin(const void *p, uint64_t n);
void host_unpin(const void *p);
char *bounce_acquire(jfsx_ctx *c, size_t need, size_t *cap);
void bounce_release(jfsx_ctx *c, char *p, size_t cap);
void bounce_count(jfsx_ctx *c, uint64_t in, uint64_t out);
}  // namespace jfsx

namespace {
// A per-object request on pageable memory (a Go-heap slice: io.ReadAll's
// result, Encrypt's fresh object buffer, encrypt.go:183, :258; a cache page)
// is staged here, on the calling thread: its block is copied into a pinned
// bounce buffer of the engine before the request is queued, and its output
// copied out of it after the request completes.  So max-uploads callers copy
// in parallel, and the dispatchers, which run the batches, never copy.
// Blocks up to a quarter of an arena take a slice of the aggregator's shared
// arena (JFSX_AGG_ARENA_MB, default 64; 0: a bounce buffer of their own, as
// larger blocks always do).
size_t arena_bytes() {
    static const size_t v = [] {
        const char *e = getenv("JFSX_AGG_ARENA_MB");
        return (size_t)(e ? atoll(e) : 64) << 20;
    }();
    return v;
}

// a slice of need bytes of the open arena (a fresh one when it is full).  A
// new arena is allocated outside the lock (pinned allocation takes
// milliseconds), so other callers keep reserving from the open one meanwhile.
char *arena_reserve(jfsx_agg *a, size_t need, AggArena **out) {
    for (;;) {
        {
            std::lock_guard<std::mutex> g(a->ar_mu);
            AggArena *cur = a->ar_cur;
            if (cur && !cur->refs) cur->used = 0;  // nothing of it in flight: start over at its base
            if (cur && cur->used + need > cur->cap) {  // full: close it
                cur->open = false;
                if (!cur->refs) a->ar_free.push_back(cur);
                a->ar_cur = cur = nullptr;
            }
            if (!cur && !a->ar_free.empty()) {
                cur = a->ar_free.back();
                a->ar_free.pop_back();
                cur->used = 0;
                cur->open = true;
                a->ar_cur = cur;
            }
            if (cur) {
                char *p = cur->base + cur->used;
                cur->used += need;
                cur->refs++;
                *out = cur;
                return p;
            }
        }
        size_t cap = 0;
        char *base = jfsx::bounce_acquire(a->cs[0], arena_bytes(), &cap);
        if (!base) return nullptr;
        AggArena *fresh = new (std::nothrow) AggArena{base, cap, 0, 0, false};
        if (!fresh) {
            jfsx::bounce_release(a->cs[0], base, cap);
            return nullptr;
        }
        std::lock_guard<std::mutex> g(a->ar_mu);
        a->ar_all.push_back(fresh);
        a->ar_free.push_back(fresh);  // the next pass takes it (or one another caller freed)
    }
}

void arena_release(jfsx_agg *a, AggArena *ar) {
    std::lock_guard<std::mutex> g(a->ar_mu);
    if (--ar->refs == 0 && !ar->open) a->ar_free.push_back(ar);
}

struct Staged {
    jfsx_agg *a = nullptr;
    jfsx_ctx *c = nullptr;
    char *p = nullptr;
    size_t cap = 0;
    AggArena *ar = nullptr;                   // p is a slice of this arena
    const void *pin[2] = {nullptr, nullptr};  // caller ranges pinned for the call
    ~Staged() {
        if (ar) arena_release(a, ar);
        else if (p) jfsx::bounce_release(c, p, cap);
        for (const void *q : pin)
            if (q) jfsx::host_unpin(q);
    }
    int get(jfsx_agg *agg, uint64_t len) {
        a = agg;
        c = agg->cs[0];
        const size_t need = (size_t)((len + 255) & ~(uint64_t)255);
        if (need <= arena_bytes() / 4 && (p = arena_reserve(agg, need, &ar))) return 0;
        p = jfsx::bounce_acquire(c, need, &cap);
        return p ? 0 : JFSX_ENOMEM;
    }
};

int agg_aead(jfsx_agg *a, int op, int algo, jfsx_blk *blk, int crc_mode, int mem);
int agg_crc(jfsx_agg *a, jfsx_range *range, int mode, int mem);
}  // namespace

namespace {
// dispatcher threads per context (JFSX_AGG_DISPATCHERS overrides)
int dispatchers_per_ctx() {
    static const int d = [] {
        const char *e = getenv("JFSX_AGG_DISPATCHERS");
        const int v = e ? atoi(e) : 0;
        return v >= 1 && v <= 32 ? v : 4;
    }();
    return d;
}

int agg_start(const std::vector<jfsx_ctx *> &cs, int max_blocks, uint64_t max_bytes, uint32_t window_us,
              jfsx_agg **out) {
    jfsx_agg *a = new (std::nothrow) jfsx_agg;
    if (!a) return JFSX_ENOMEM;
    const int per = dispatchers_per_ctx();
    // dispatcher j serves device j % ndev, so the first dispatchers to wake
    // are spread over the devices
    for (int j = 0; j < per * (int)cs.size(); j++) {
        a->cs.push_back(cs[j % cs.size()]);
        a->dev.push_back(j % (int)cs.size());
    }
    a->max_blocks = max_blocks ? max_blocks : 256;
    a->max_bytes = max_bytes ? max_bytes : (uint64_t)1 << 30;
    a->window = std::chrono::microseconds(window_us);
    a->dev_batches.assign(cs.size(), 0);
    a->serial.assign(cs.size(), 0);
    for (size_t k = 0; k < a->cs.size(); k++) a->ths.emplace_back([a, k] { a->run((int)k); });
    *out = a;
    return 0;
}
// device pointers belong to one GPU: over a multi-device context any
// dispatcher may take a group, so only host memory is accepted there (as the
// jfsx_mctx_*_batch entry points do)
bool agg_mem_ok(const jfsx_agg *a, int mem) {
    return valid_mem(mem) && !(mem == JFSX_MEM_DEVICE && a->dev_batches.size() > 1);
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
    for (AggArena *ar : a->ar_all) {  // no request holds a slice any more
        jfsx::bounce_release(a->cs[0], ar->base, ar->cap);
        delete ar;
    }
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
    return agg_aead(a, kSeal, algo, blk, crc_mode, mem);
}

int jfsx_agg_open(jfsx_agg *a, int algo, jfsx_blk *blk, int crc_mode, int mem) {
    if (!a || !blk || !valid_algo(algo) || !agg_mem_ok(a, mem)) return JFSX_EINVAL;
    return agg_aead(a, kOpen, algo, blk, crc_mode, mem);
}

int jfsx_agg_crc32c(jfsx_agg *a, jfsx_range *range, int mode, int mem) {
    if (!a || !range || !agg_mem_ok(a, mem) || (mode != JFSX_CRC_GEN && mode != JFSX_CRC_VERIFY)) return JFSX_EINVAL;
    return agg_crc(a, range, mode, mem);
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

}  // extern "C"

namespace {
int agg_aead(jfsx_agg *a, int op, int algo, jfsx_blk *blk, int crc_mode, int mem) {
    const uint64_t len = blk->len;
    const bool host = mem == JFSX_MEM_HOST && len && blk->src && blk->dst;
    bool in_pg = host && !jfsx::host_pinned(blk->src, len);
    bool out_pg = host && (blk->dst == blk->src ? in_pg : !jfsx::host_pinned(blk->dst, len));
    Staged st;
    // first choice: pin the caller's own pages for the call (no copy)
    if (in_pg && jfsx::host_pin(blk->src, len)) {
        st.pin[0] = blk->src;
        in_pg = false;
        if (blk->dst == blk->src) out_pg = false;
    }
    if (out_pg && jfsx::host_pin(blk->dst, len)) {
        st.pin[1] = blk->dst;
        out_pg = false;
    }
    if (!in_pg && !out_pg) {
        Req r{op, algo, crc_mode, mem, blk, nullptr, nullptr, len};
        return a->submit(r);
    }
    if (st.get(a, len)) return JFSX_ENOMEM;
    jfsx_blk w = *blk;
    if (in_pg) {
        memcpy(st.p, blk->src, len);
        w.src = st.p;
    }
    if (out_pg) w.dst = st.p;  // in place in the bounce buffer when both are pageable
    Req r{op, algo, crc_mode, mem, &w, nullptr, nullptr, len};
    const int rc = a->submit(r);
    const void *src = blk->src;
    void *dst = blk->dst;
    *blk = w;  // results into the caller's record, its own pointers kept
    blk->src = src;
    blk->dst = dst;
    if (rc == 0 && out_pg) {
        // an Open whose tag failed releases nothing (the engine zeroed the
        // bounce copy; the caller's buffer is zeroed here)
        if (op == kOpen && w.status == JFSX_ETAG) memset(dst, 0, len);
        else memcpy(dst, st.p, len);
    }
    jfsx::bounce_count(st.c, in_pg ? len : 0, rc == 0 && out_pg ? len : 0);
    return rc;
}

int agg_crc(jfsx_agg *a, jfsx_range *range, int mode, int mem) {
    const uint64_t len = range->len;
    if (mem != JFSX_MEM_HOST || !len || !range->data || jfsx::host_pinned(range->data, len)) {
        Req r{kCrc, 0, mode, mem, nullptr, range, nullptr, len};
        return a->submit(r);
    }
    Staged st;
    if (jfsx::host_pin(range->data, len)) {
        st.pin[0] = range->data;
        Req r{kCrc, 0, mode, mem, nullptr, range, nullptr, len};
        return a->submit(r);
    }
    if (st.get(a, len)) return JFSX_ENOMEM;
    memcpy(st.p, range->data, len);
    jfsx_range w = *range;
    w.data = st.p;
    Req r{kCrc, 0, mode, mem, nullptr, &w, nullptr, len};
    const int rc = a->submit(r);
    const void *data = range->data;
    *range = w;
    range->data = data;
    jfsx::bounce_count(st.c, len, 0);
    return rc;
}
}  // namespace

extern "C" {

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

namespace jfsx {
// device owning a device pointer, with its allocation's bounds; -1 for host
// memory (jfsx_api.cpp; the host harness stubs it)
int device_of(const void *p, uintptr_t *lo, uintptr_t *hi);
}  // namespace jfsx

namespace {
// persistent worker threads running one device's parts of the batches: a
// few per device (JFSX_MCTX_WORKERS, default 4), so concurrent callers of a
// multi-device context overlap on every device, as they do on the first one,
// whose part runs on each calling thread
int mctx_workers() {
    static const int v = [] {
        const char *e = getenv("JFSX_MCTX_WORKERS");
        const int t = e ? atoi(e) : 4;
        return t >= 1 && t <= 64 ? t : 4;
    }();
    return v;
}

struct MWorker {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    bool stop = false;
    std::vector<std::thread> ths;

    void run() {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return stop || !q.empty(); });
            if (q.empty()) return;
            std::function<void()> f = std::move(q.front());
            q.pop_front();
            lk.unlock();
            f();
            lk.lock();
        }
    }
    void post(std::function<void()> f) {
        std::lock_guard<std::mutex> g(mu);
        q.push_back(std::move(f));
        cv.notify_one();
    }
};
}  // namespace

struct jfsx_mctx {
    std::vector<jfsx_ctx *> cs;
    std::vector<int> devs;                      // device ordinal of cs[k]
    std::vector<std::unique_ptr<MWorker>> ws;   // ws[k] runs device k's parts (k >= 1)
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

// run f(k) for every device k with work (has[k]): device parts 1.. on their
// persistent workers, the first on the calling thread; the first error in
// device order is returned
int fan_out(jfsx_mctx *m, const std::vector<char> &has, const std::function<int(int)> &f) {
    const int nd = (int)m->cs.size();
    std::vector<int> rc(nd, 0);
    std::mutex mu;
    std::condition_variable cv;
    int left = 0, first = -1;
    for (int k = 0; k < nd; k++)
        if (has[k]) {
            if (first < 0) first = k;
            else left++;
        }
    if (first < 0) return 0;
    for (int k = first + 1; k < nd; k++) {
        if (!has[k]) continue;
        m->ws[k]->post([&, k] {
            const int r = f(k);
            std::lock_guard<std::mutex> g(mu);
            rc[k] = r;
            if (--left == 0) cv.notify_all();
        });
    }
    rc[first] = f(first);
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return left == 0; });
    }
    for (int k = 0; k < nd; k++)
        if (rc[k]) return rc[k];
    return 0;
}

// Per-device parts of a batch of T items.  Host memory: contiguous runs
// balanced by bytes.  Device memory: each item goes to the device that owns
// the pointers ptrs(item) lists (all on one member device, else JFSX_EINVAL).
// A device whose items are one contiguous run of the caller's array runs it in
// place; otherwise its items are gathered, run, and scattered back.
template <class T>
int mctx_run(jfsx_mctx *m, int n, T *items, int mem, const std::function<uint64_t(const T &)> &bytes,
             const std::function<int(const T &, const void **)> &ptrs,
             const std::function<int(jfsx_ctx *, int, T *)> &run) {
    if (!m || n < 0 || (n && !items) || (mem != JFSX_MEM_HOST && mem != JFSX_MEM_DEVICE)) return JFSX_EINVAL;
    if (n == 0) return 0;
    const int nd = (int)m->cs.size();
    std::vector<char> has(nd, 0);
    if (mem == JFSX_MEM_HOST || nd == 1) {
        const std::vector<int> cut = nd == 1 ? std::vector<int>{0, n}
                                             : split_runs(n, nd, [&](int i) { return bytes(items[i]); });
        for (int k = 0; k < nd; k++) has[k] = cut[k + 1] > cut[k];
        return fan_out(m, has, [&](int k) { return run(m->cs[k], cut[k + 1] - cut[k], items + cut[k]); });
    }
    // ownership routing
    int maxdev = 0;
    for (int d : m->devs) maxdev = std::max(maxdev, d);
    std::vector<int> slot_of(maxdev + 1, -1);
    for (int k = 0; k < nd; k++) slot_of[m->devs[k]] = k;
    std::vector<int> owner(n);
    uintptr_t lo = 1, hi = 0;
    int cdev = -1;  // allocation of the last lookup
    for (int i = 0; i < n; i++) {
        const void *p[4];
        const int np = ptrs(items[i], p);
        int d = -2;
        for (int j = 0; j < np; j++) {
            const uintptr_t a = (uintptr_t)p[j];
            if (!(a >= lo && a < hi)) cdev = jfsx::device_of(p[j], &lo, &hi);
            if (cdev < 0 || cdev > maxdev || slot_of[cdev] < 0 || (d != -2 && d != cdev)) return JFSX_EINVAL;
            d = cdev;
        }
        owner[i] = d == -2 ? 0 : slot_of[d];  // an item with no buffers runs anywhere
        has[owner[i]] = 1;
    }
    std::vector<std::vector<int>> idx(nd);
    for (int i = 0; i < n; i++) idx[owner[i]].push_back(i);
    return fan_out(m, has, [&](int k) {
        const std::vector<int> &ix = idx[k];
        if (ix.back() - ix.front() + 1 == (int)ix.size()) return run(m->cs[k], (int)ix.size(), items + ix.front());
        std::vector<T> tmp(ix.size());
        for (size_t j = 0; j < ix.size(); j++) tmp[j] = items[ix[j]];
        const int rc = run(m->cs[k], (int)ix.size(), tmp.data());
        for (size_t j = 0; j < ix.size(); j++) items[ix[j]] = tmp[j];
        return rc;
    });
}

int blk_ptrs(const jfsx_blk &b, int crc_mode, const void **p) {
    int np = 0;
    if (b.len) {
        p[np++] = b.src;
        p[np++] = b.dst;
    }
    if (crc_mode && b.crc) p[np++] = b.crc;
    return np;
}

int mctx_aead(jfsx_mctx *m, bool open, int algo, int n, jfsx_blk *blks, int crc_mode, int mem) {
    return mctx_run<jfsx_blk>(
        m, n, blks, mem, [](const jfsx_blk &b) { return b.len; },
        [&](const jfsx_blk &b, const void **p) { return blk_ptrs(b, crc_mode, p); },
        [&](jfsx_ctx *c, int cnt, jfsx_blk *part) {
            return open ? jfsx_open_batch(c, algo, cnt, part, crc_mode, mem)
                        : jfsx_seal_batch(c, algo, cnt, part, crc_mode, mem);
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
        m->devs.push_back(d);
    }
    for (size_t k = 0; k < m->cs.size(); k++) {
        m->ws.emplace_back(new MWorker);
        if (k) {
            MWorker *w = m->ws.back().get();
            for (int t = 0; t < mctx_workers(); t++) w->ths.emplace_back([w] { w->run(); });
        }
    }
    *out = m;
    return 0;
}

int jfsx_mctx_close(jfsx_mctx *m) {
    if (!m) return JFSX_EINVAL;
    for (auto &w : m->ws) {
        if (w->ths.empty()) continue;
        {
            std::lock_guard<std::mutex> g(w->mu);
            w->stop = true;
            w->cv.notify_all();
        }
        for (std::thread &t : w->ths) t.join();
    }
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
    return mctx_run<jfsx_range>(
        m, n, ranges, mem, [](const jfsx_range &r) { return r.len; },
        [](const jfsx_range &r, const void **p) {
            int np = 0;
            if (r.len) p[np++] = r.data;
            if (r.crc) p[np++] = r.crc;
            return np;
        },
        [&](jfsx_ctx *c, int cnt, jfsx_range *part) { return jfsx_crc32c_segments(c, cnt, part, mode, mem); });
}

static int mctx_codec(jfsx_mctx *m, int op, int n, jfsx_zblk *z, int mem) {
    return mctx_run<jfsx_zblk>(
        m, n, z, mem, [](const jfsx_zblk &b) { return b.src_len; },
        [](const jfsx_zblk &b, const void **p) {
            int np = 0;
            if (b.src_len) p[np++] = b.src;
            if (b.dst_cap) p[np++] = b.dst;
            return np;
        },
        [&](jfsx_ctx *c, int cnt, jfsx_zblk *part) {
            return op == kLz4c    ? jfsx_lz4_compress_batch(c, cnt, part, mem)
                   : op == kLz4d  ? jfsx_lz4_decompress_batch(c, cnt, part, mem)
                   : op == kZstdc ? jfsx_zstd_compress_batch(c, cnt, part, mem)
                                  : jfsx_zstd_decompress_batch(c, cnt, part, mem);
        });
}

int jfsx_mctx_lz4_compress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) {
    return mctx_codec(m, kLz4c, n, blks, mem);
}
int jfsx_mctx_lz4_decompress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) {
    return mctx_codec(m, kLz4d, n, blks, mem);
}
int jfsx_mctx_zstd_decompress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) {
    return mctx_codec(m, kZstdd, n, blks, mem);
}

int jfsx_mctx_zstd_compress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem) {
    return mctx_codec(m, kZstdc, n, blks, mem);
}

int jfsx_agg_new_mctx(jfsx_mctx *m, int max_blocks, uint64_t max_bytes, uint32_t window_us, jfsx_agg **out) {
    if (!m || m->cs.empty() || !out || max_blocks < 0) return JFSX_EINVAL;
    return agg_start(m->cs, max_blocks, max_bytes, window_us, out);
}

}  // extern "C"

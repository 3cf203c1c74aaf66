// jfsx_api.cpp -- C-ABI of libjfsx.so (include/jfsx.h): contexts, tables,
// batch planning, staging, launches.  Host code, compiled by hipcc.
//
// A batch runs as: H2D of descriptors (one pinned copy) -> keysetup kernel ->
// main transform kernel (one workgroup per task) -> finalize kernel -> D2H of
// per-block results (tags, status, first failing CRC) -> stream sync.
#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "jfsx_internal.h"

#define JFSX_HD static inline
#include "jfsx_rsa.h"

using namespace jfsx;

// Every HIP failure is recorded with its call site before the engine returns
// JFSX_EIO, so a caller can tell a device fault from an out-of-resources
// launch or a bad copy (jfsx_last_error).
#define HIP_OK(x)                                                      \
    do {                                                               \
        const hipError_t e_ = (x);                                     \
        if (e_ != hipSuccess) {                                        \
            note_hip_error(e_, __FILE__, __LINE__, #x);                \
            return JFSX_EIO;                                           \
        }                                                              \
    } while (0)

namespace {

// last failure: per calling thread, and per context for calls made on one
struct ErrRec {
    int hip = 0;
    char msg[320] = {0};
};
thread_local ErrRec tl_err;
thread_local jfsx_ctx *tl_ctx = nullptr;  // context of the entry point running on this thread
void note_ctx_error(jfsx_ctx *c, const ErrRec &e);

void note_hip_error(hipError_t e, const char *file, int line, const char *expr) {
    const char *base = strrchr(file, '/');
    snprintf(tl_err.msg, sizeof(tl_err.msg), "%s (%s) at %s:%d in %s", hipGetErrorName(e), hipGetErrorString(e),
             base ? base + 1 : file, line, expr);
    tl_err.hip = (int)e;
    if (tl_ctx) note_ctx_error(tl_ctx, tl_err);
    (void)hipGetLastError();  // a handled failure must not resurface at the next launch check
}

// hipGetLastError() after a launch also returns the error of any earlier
// failed HIP call of this thread (a handled hipMalloc failure, say): clear the
// slot before launching, so the check that follows sees only the launch
inline void launch_begin() { (void)hipGetLastError(); }

// an entry point's scope: failures inside it are also kept on the context
struct CtxScope {
    jfsx_ctx *prev;
    explicit CtxScope(jfsx_ctx *c) : prev(tl_ctx) { tl_ctx = c; }
    ~CtxScope() { tl_ctx = prev; }
};

// Device allocations made through jfsx_alloc_device, by address: a
// multi-device context routes each block of a device-memory batch to the GPU
// that owns its buffers (jfsx_mctx_seal_batch and friends).
std::shared_mutex g_alloc_mu;
std::map<uintptr_t, std::pair<uintptr_t, int>> g_allocs;  // base -> (end, device)

void note_alloc(void *p, size_t bytes, int device) {
    std::unique_lock<std::shared_mutex> g(g_alloc_mu);
    g_allocs[(uintptr_t)p] = {(uintptr_t)p + bytes, device};
}
void forget_alloc(void *p) {
    std::unique_lock<std::shared_mutex> g(g_alloc_mu);
    g_allocs.erase((uintptr_t)p);
}

// Page-locked host allocations made through jfsx_alloc_pinned(_node), by
// address: a host call streams such blocks with no bounce copy.
std::shared_mutex g_pin_mu;
std::map<uintptr_t, uintptr_t> g_pinned;  // base -> end

void note_pinned(void *p, size_t bytes) {
    std::unique_lock<std::shared_mutex> g(g_pin_mu);
    g_pinned[(uintptr_t)p] = (uintptr_t)p + bytes;
}
void forget_pinned(void *p) {
    std::unique_lock<std::shared_mutex> g(g_pin_mu);
    g_pinned.erase((uintptr_t)p);
}
// base of the engine-pinned allocation holding p, 0 if none
uintptr_t pinned_base(const void *p) {
    const uintptr_t a = (uintptr_t)p;
    std::shared_lock<std::shared_mutex> g(g_pin_mu);
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return 0;
    --it;
    return a < it->second ? it->first : 0;
}

// JFSX_HOST_STAGE: how a pageable host block reaches the DMA engines.
//   bounce (default)    copy it into the context's pinned bounce buffers on
//                       the calling thread (20 per-object callers: 41.7 GB/s,
//                       0.22 host CPU-s per GB, profiles/r6)
//   register            pin the caller's own pages for the call
//                       (hipHostRegister / hipHostUnregister around it), and
//                       bounce where the runtime refuses; no copies (0.10 CPU-s
//                       per GB) but 28-31 GB/s: under 20 concurrent callers
//                       the runtime's registration and lookup calls contend
//   none                hand the pageable pointer to hipMemcpyAsync as it is
//                       (the runtime's own staged copy: 15.3 GB/s, A/B only)
//   all                 bounce every host block, pinned or not (tests)
enum { kStageNone = 0, kStageRegister = 1, kStageBounce = 2, kStageAll = 3 };
int stage_policy() {
    static const int v = [] {
        const char *e = getenv("JFSX_HOST_STAGE");
        if (!e || !strcmp(e, "bounce")) return (int)kStageBounce;
        if (!strcmp(e, "register")) return (int)kStageRegister;
        if (!strcmp(e, "none")) return (int)kStageNone;
        return (int)kStageAll;
    }();
    return v;
}
}  // namespace

namespace jfsx {
// true when [p, p + n) may be handed to the DMA engines as it is: engine-pinned
// memory, or host memory the HIP runtime reports as registered (another
// library's pinned buffers).  Everything else -- the Go heap, malloc, numpy --
// is pageable and goes through the context's bounce pool.
bool host_pinned(const void *p, uint64_t n) {
    const int pol = stage_policy();
    if (pol == kStageNone || pol == kStageAll || !n) return pol != kStageAll || !n;
    const uintptr_t a = (uintptr_t)p;
    {
        std::shared_lock<std::shared_mutex> g(g_pin_mu);
        auto it = g_pinned.upper_bound(a);
        if (it != g_pinned.begin()) {
            --it;
            if (a < it->second) return a + n <= it->second;
        }
    }
    hipPointerAttribute_t at;
    const bool reg = hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    return reg;
}

// Pin a pageable caller range for the duration of one call (JFSX_HOST_STAGE
// register): true when it is now page-locked and must be released with
// host_unpin once the call's DMA has finished; false where the policy is not
// register or the runtime refuses (the caller then bounces the block).  The
// Go heap does not move objects, and the range is released before the call
// returns, so cgo's rule that C keeps no Go pointer past the call holds.
bool host_pin(const void *p, uint64_t n) {
    if (stage_policy() != kStageRegister || !n) return false;
    const hipError_t e = hipHostRegister(const_cast<void *>(p), n, hipHostRegisterPortable);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    note_pinned(const_cast<void *>(p), n);  // host_pinned() then answers from the registry
    return true;
}
void host_unpin(const void *p) {
    forget_pinned(const_cast<void *>(p));
    if (hipHostUnregister(const_cast<void *>(p)) != hipSuccess) (void)hipGetLastError();
}
}  // namespace jfsx

namespace {

// ---------------------------------------------------------------------------
// table construction (host)
// ---------------------------------------------------------------------------
uint8_t gf8_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0));
        b >>= 1;
    }
    return p;
}

void make_aes_table(std::vector<uint32_t> &t) {
    // S-box = affine(inverse) over GF(2^8) (FIPS-197 5.1.1)
    uint8_t sbox[256];
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) {
            uint8_t r = 1, base = (uint8_t)x;
            for (int e = 254; e; e >>= 1) {
                if (e & 1) r = gf8_mul(r, base);
                base = gf8_mul(base, base);
            }
            inv = r;
        }
        uint8_t s = inv, v = inv;
        for (int k = 1; k <= 4; k++) v ^= (uint8_t)((s << k) | (s >> (8 - k)));
        sbox[x] = v ^ 0x63;
    }
    t.assign(256 * 64, 0);
    for (int x = 0; x < 256; x++) {
        uint32_t s = sbox[x];
        uint32_t t0 = gf8_mul((uint8_t)s, 2) | (s << 8) | (s << 16) | ((uint32_t)gf8_mul((uint8_t)s, 3) << 24);
        uint32_t t2 = (t0 << 16) | (t0 >> 16);
        for (int r = 0; r < 32; r++) {
            t[x * 64 + r] = t0;
            t[x * 64 + 32 + r] = t2;
        }
    }
}

uint32_t crc_mulmod_h(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & 0x80000000u) p ^= b;
        a <<= 1;
        b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
    }
    return p;
}

void make_crc_tables(std::vector<uint32_t> &crc, std::vector<uint32_t> &crcx) {
    uint32_t T[256];
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
        T[i] = c;
    }
    uint32_t x8[32];
    x8[0] = 0x00800000u;  // x^8
    for (int k = 1; k < 32; k++) x8[k] = crc_mulmod_h(x8[k - 1], x8[k - 1]);
    auto xpow8 = [&](uint64_t n) {
        uint32_t r = 0x80000000u;
        for (int k = 0; n; k++, n >>= 1)
            if (n & 1) r = crc_mulmod_h(x8[k], r);
        return r;
    };
    crc.assign(32 * 256, 0);
    for (int j = 0; j < 16; j++) {
        const uint32_t xp = xpow8(15 - j);
        for (int b = 0; b < 256; b++) crc[j * 256 + b] = crc_mulmod_h(xp, T[b]);
    }
    // S tables: shift a lane CRC across the gap to its next piece -- 1008 B for
    // 16-B pieces at 1 KiB row stride (GCM), 4032 B for 64-B chunks at 4 KiB (ChaCha)
    // (and 1024 B / 4096 B: a whole row / a whole 4 KiB span of 64-B lane chunks,
    // for the CRC-only kernel's A' = S(A) ^ crc_raw(0, chunk))
#ifndef JFSX_CRC_SPAN
#define JFSX_CRC_SPAN 64
#endif
    // (the CRC-only kernel's span: 64 lanes x JFSX_CRC_SPAN bytes, jfsx_crc.hip)
    const uint32_t x1008 = xpow8(1008), x4032 = xpow8(4032), x1024 = xpow8(1024),
                   x4096 = xpow8(64 * (JFSX_CRC_SPAN >= 64 ? JFSX_CRC_SPAN : 64));
    for (int k = 0; k < 4; k++)
        for (uint32_t v = 0; v < 256; v++) {
            crc[(16 + k) * 256 + v] = crc_mulmod_h(x1008, v << (8 * k));
            crc[(20 + k) * 256 + v] = crc_mulmod_h(x4032, v << (8 * k));
            crc[(24 + k) * 256 + v] = crc_mulmod_h(x1024, v << (8 * k));
            crc[(28 + k) * 256 + v] = crc_mulmod_h(x4096, v << (8 * k));
        }
    crcx.assign(192, 0);
    for (int l = 0; l < 64; l++) crcx[l] = xpow8(16 * (63 - l));
    for (int k = 0; k < 32; k++) crcx[64 + k] = x8[k];
    crcx[96] = crc_mulmod_h(xpow8(kSeg), 0xffffffffu);
    // x^(8 * 1024 k), k = 1..31: whole-row shifts (crc_xpow8_fast, jfsx_internal.h)
    for (int k = 1; k < 32; k++) crcx[96 + k] = xpow8(1024 * (uint64_t)k);
    for (int l = 0; l < 64; l++) crcx[128 + l] = xpow8(64 * (63 - l));
}

inline uint64_t nseg_of(uint64_t len) { return len ? (len + kSeg - 1) / kSeg : 1; }

struct Plan {
    std::vector<Task> tasks;
    uint64_t nslots = 0;
};

// Device + pinned-host scratch for one in-flight batch.
struct Workspace {
    char *d = nullptr;  // descriptors, schedules, partials, results (device)
    size_t dcap = 0;
    char *h = nullptr;  // pinned mirror: descriptors up, results down
    size_t hcap = 0;
    char *stage = nullptr;  // host-ingest staging for block data (device)
    size_t scap = 0;
    int n = 0;              // blocks of the batch in flight
    uint64_t nt = 0;        // tasks of the batch in flight
    const void *dout = nullptr;  // device BlkOut[n] of the batch in flight
    size_t down = 0;        // bytes of the result download (BlkOut[n], then the CRC words with host_crc)
    size_t crc_off = 0;     // host_crc GEN: offset of the CRC words in that download
    size_t res_off = 0;     // offset of the results (BlkOut[n], CRC words) in h
    bool crc_back = false;  // host_crc GEN: finish_aead copies the CRC words to the callers' arrays
    int crc_mult = 1;       // CRC arrays per block (2 with JFSX_CRC_BOTH)
    bool timed = false;     // the batch's main kernel is bracketed by timing events
};

constexpr int kRing = 1;  // workspace of the synchronous paths (device batches, CRC, codecs, generator)
#ifndef JFSX_PIPE
#define JFSX_PIPE 8
#endif
// Host-memory AEAD pipeline (run_aead_host): kPipe staging slots shared by every
// thread that calls on the context.  A batch is cut into groups; each group
// takes the next slot, is enqueued as H2D (s_in) -> keysetup/main/finalize
// (stream) -> D2H (s_out) and the call moves on; it then waits for its own
// groups' D2H events only.  The ring never drains between calls: while one
// caller waits for its results, the next caller's H2D is already running
// (per-object callers: the aggregator's dispatchers, cached_store.go:415-472).
constexpr int kPipe = JFSX_PIPE;

struct PipeGroup;
struct PipeSlot {
    std::mutex mu;               // held while the slot is completed or refilled
    Workspace w;
    hipEvent_t ev_in = nullptr, ev_comp = nullptr, ev_out = nullptr;
    hipEvent_t ev_k0 = nullptr, ev_k1 = nullptr;  // main-kernel timing
    hipEvent_t ev_ks = nullptr;                   // descriptors pulled and keysetup done (s_ks)
    PipeGroup *owner = nullptr;  // group in flight in this slot (its results not yet collected)
};
// one group of one host batch: where its results go once its D2H is done
struct PipeGroup {
    PipeSlot *slot = nullptr;
    jfsx_blk *dv = nullptr;  // the call's per-block result records of this group
    bool open = false;
    int rc = 0;
    char *bounce = nullptr;  // pinned bounce region of the group's pageable blocks (owner only)
    size_t bcap = 0;
    std::vector<const void *> pins;  // caller ranges pinned for the group (owner only)
};

// Engine-owned pinned staging for callers' pageable memory (SURVEY §8b
// "Ownership": the reference's pages and objects are Go-heap slices,
// pkg/chunk/page.go:42-50, pkg/object/encrypt.go:183, :258).  A host call
// copies its pageable blocks into a bounce buffer on its own thread before it
// enqueues them, and out of it on its own thread after its D2H, so concurrent
// callers copy in parallel and the DMA engines only ever see page-locked
// memory.  Grow-only per context: idle buffers are kept (up to a retention
// cap) and handed to the next call whose group fits.
struct BouncePool {
    std::mutex mu;
    std::multimap<size_t, char *> idle;  // capacity -> buffer
    size_t idle_bytes = 0;
    std::atomic<uint64_t> allocs{0}, bytes_in{0}, bytes_out{0};
};

}  // namespace

struct jfsx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;  // transform stream
    hipStream_t s_in = nullptr;    // host-ingest H2D
    hipStream_t s_out = nullptr;   // host-ingest D2H
    hipStream_t s_ks = nullptr;    // host pipeline: descriptor pull + keysetup of the next group
    std::mutex mu;                 // enqueue order on the streams; the synchronous paths' workspace
    uint32_t *d_tab = nullptr;  // aes | crc | crcx
    DevTables tabs{};
    Workspace ws[kRing];
    hipEvent_t ev_k0[kRing] = {}, ev_k1[kRing] = {};  // main-kernel timing of the synchronous paths
    PipeSlot pipe[kPipe];
    int pipe_next = 0;  // next pipeline slot (under mu)
    // JFSX_PIPE_STATS=1: where host batches spend their time, printed at close
    // (groups, us enqueueing under mu, us waiting for a busy slot, us waiting
    // for one's own groups)
    std::atomic<uint64_t> ps_groups{0}, ps_enq_us{0}, ps_slot_us{0}, ps_own_us{0};
    // host-memory checks, bounce copies in (with the buffer's acquisition) and
    // out, waits for one's own groups (us, summed over callers)
    std::atomic<uint64_t> ps_pin_us{0}, ps_bin_us{0}, ps_bout_us{0}, ps_wait_us{0};
    std::atomic<uint64_t> ps_blocks{0}, ps_h2d{0}, ps_d2h{0};  // blocks, data copies up / down (coalesced runs)
    std::mutex stat_mu; // met, ms_total, launches
    std::atomic<size_t> slot_bytes{(size_t)256 << 20};
    int ncu = 256;  // compute units: persistent transform kernels launch one workgroup per CU
    size_t zstd_arena_budget = 0;  // device bytes the block-parallel zstd decoder may hold (see run_codec)
    bool timing = false;
    bool bitslice = false;  // JFSX_CTX_BITSLICE
    char *rsa_d = nullptr;  // batched RSA unwrap: ct | halves | em | len (device, grow-only)
    size_t rsa_dcap = 0;
    char *rsa_h = nullptr;  // pinned mirror of ct in / em + len out
    size_t rsa_hcap = 0;
    double ms_total = 0;
    uint64_t launches = 0;
    BouncePool bounce;       // pinned staging of pageable caller memory (host calls)
    int numa_node = -1;      // host NUMA node of the device (bounce buffers are placed there)
    std::mutex err_mu;     // last HIP failure on this context (jfsx_last_error)
    ErrRec err;
    jfsx_metrics met{};      // jfsx_ctx_metrics (updated under mu)
};

namespace {
void add_kernel_ms(jfsx_ctx *c, float ms) {
    std::lock_guard<std::mutex> g(c->stat_mu);
    c->ms_total += ms;
    c->launches += 1;
}
// jfsx_ctx_metrics tallies after a batch returned 0
void tally_aead(jfsx_ctx *c, bool open, int n, const jfsx_blk *b) {
    std::lock_guard<std::mutex> g(c->stat_mu);
    jfsx_metrics &m = c->met;
    uint64_t bytes = 0, fail = 0;
    for (int i = 0; i < n; i++) {
        bytes += b[i].len;
        fail += b[i].status != JFSX_OK;
    }
    if (open) {
        m.open_batches++;
        m.open_blocks += n;
        m.open_bytes += bytes;
        m.open_fail += fail;
    } else {
        m.seal_batches++;
        m.seal_blocks += n;
        m.seal_bytes += bytes;
    }
}
void tally_crc(jfsx_ctx *c, int n, const jfsx_range *r) {
    std::lock_guard<std::mutex> g(c->stat_mu);
    jfsx_metrics &m = c->met;
    m.crc_batches++;
    m.crc_ranges += n;
    for (int i = 0; i < n; i++) {
        m.crc_bytes += r[i].len;
        m.crc_fail += r[i].status != JFSX_OK;
    }
}
void tally_codec(jfsx_ctx *c, uint64_t &blocks, uint64_t &in, uint64_t &out, uint64_t *fail, int n,
                 const jfsx_zblk *z) {
    std::lock_guard<std::mutex> g(c->stat_mu);
    blocks += n;
    for (int i = 0; i < n; i++) {
        in += z[i].src_len;
        out += z[i].out_len;
        if (fail) *fail += z[i].status != JFSX_OK;
    }
}
void note_ctx_error(jfsx_ctx *c, const ErrRec &e) {
    std::lock_guard<std::mutex> g(c->err_mu);
    c->err = e;
}
}  // namespace

namespace {

int ensure_dev(jfsx_ctx *c, char **buf, size_t *cap, size_t need) {
    if (need <= *cap) return 0;
    if (*buf) {
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipFree(*buf));
        *buf = nullptr;
        *cap = 0;
    }
    size_t n = std::max(need, (size_t)1 << 20);
    n = (n + 0xFFFFF) & ~(size_t)0xFFFFF;
    const hipError_t e = hipMalloc((void **)buf, n);
    if (e != hipSuccess) {
        note_hip_error(e, __FILE__, __LINE__, "hipMalloc(workspace)");
        return JFSX_ENOMEM;
    }
    *cap = n;
    return 0;
}

int ensure_host(char **buf, size_t *cap, size_t need) {
    if (need <= *cap) return 0;
    if (*buf) {
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipHostFree(*buf));
        *buf = nullptr;
        *cap = 0;
    }
    size_t n = std::max(need, (size_t)1 << 20);
    n = (n + 0xFFFFF) & ~(size_t)0xFFFFF;
    const hipError_t e = hipHostMalloc((void **)buf, n, hipHostMallocDefault);
    if (e != hipSuccess) {
        note_hip_error(e, __FILE__, __LINE__, "hipHostMalloc(staging)");
        return JFSX_ENOMEM;
    }
    *cap = n;
    return 0;
}

inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Split each block into <= max_bytes tasks (a multiple of waves segments), one
// workgroup each; `slots` partial slots per task.
Plan plan_tasks(const std::vector<uint64_t> &lens, uint64_t max_bytes, uint32_t waves, uint32_t slots,
                uint64_t want, uint64_t min_task = 0) {
    Plan p;
    uint64_t total = 0;
    for (uint64_t l : lens) total += l;
    // tasks are whole segments; min_task (GCM: its row split keeps all 16
    // waves busy on any task) or else one segment per wave
    const uint64_t unit = min_task ? min_task : (uint64_t)waves * kSeg;
    uint64_t ch = max_bytes;
    // enough workgroups to fill the 256 CUs when the batch is small
    if (total / ch < want) {
        uint64_t c = (total / want + unit - 1) / unit * unit;
        ch = std::max(unit, std::min(ch, c));
    }
    for (size_t b = 0; b < lens.size(); b++) {
        for (uint64_t c0 = 0; c0 < lens[b]; c0 += ch) {
            Task t;
            t.blk = (uint32_t)b;
            t.slot0 = (uint32_t)p.nslots;
            t.c0 = c0;
            t.c1 = std::min(c0 + ch, lens[b]);
            p.tasks.push_back(t);
            p.nslots += slots;
        }
    }
    return p;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15) == 0; }

// tasks reordered by size, largest first, in units of 4 KiB (stable within a unit)
void order_largest_first(Task *t, size_t n, size_t max_units) {
    bool sorted = true;
    for (size_t i = 1; i < n && sorted; i++) sorted = ((t[i - 1].c1 - t[i - 1].c0) >> 12) >= ((t[i].c1 - t[i].c0) >> 12);
    if (sorted) return;
    std::vector<size_t> start(max_units + 2, 0);
    for (size_t i = 0; i < n; i++) start[max_units - std::min<size_t>((t[i].c1 - t[i].c0) >> 12, max_units) + 1]++;
    for (size_t u = 1; u < start.size(); u++) start[u] += start[u - 1];
    std::vector<Task> tmp(t, t + n);
    for (size_t i = 0; i < n; i++) t[start[max_units - std::min<size_t>((tmp[i].c1 - tmp[i].c0) >> 12, max_units)]++] = tmp[i];
}

constexpr uint64_t kGcmMaxLen = (((uint64_t)1 << 32) - 2) * 16;
constexpr uint64_t kGcmMinTask = 2 * (uint64_t)kSeg;  // 64 KiB
constexpr uint64_t kCpMaxLen = ((uint64_t)1 << 38) - 64;

// bytes per task of crc_segments_k: up to kCrcTaskBytes, but small enough that
// a small batch still spreads over every CU (~2 tasks per CU), and a whole
// number of 16-segment rounds (one 16-wave workgroup per task, jfsx_crc.hip)
uint64_t crc_task_bytes(uint64_t total) {
    const uint64_t round = 16 * (uint64_t)kSeg;
    return std::min<uint64_t>(kCrcTaskBytes, std::max<uint64_t>(round, (total / 512 + round - 1) / round * round));
}

int check_aead_args(int algo, int n, const jfsx_blk *blks, int crc_mode, bool device) {
    if (algo != JFSX_AES256GCM && algo != JFSX_CHACHA20P1305) return JFSX_EINVAL;
    // NONE, GEN, VERIFY, GEN|CT, VERIFY|CT, GEN|BOTH
    if (crc_mode < 0 || (crc_mode & ~(3 | JFSX_CRC_CT | JFSX_CRC_BOTH)) || (crc_mode & 3) == 3 ||
        crc_mode == JFSX_CRC_CT || ((crc_mode & JFSX_CRC_BOTH) && crc_mode != (JFSX_CRC_GEN | JFSX_CRC_BOTH)) || n < 0)
        return JFSX_EINVAL;
    for (int i = 0; i < n; i++) {
        const jfsx_blk &b = blks[i];
        if (b.len && (!b.src || !b.dst)) return JFSX_EINVAL;
        if (device && b.len && (!aligned16(b.src) || !aligned16(b.dst))) return JFSX_EINVAL;
        // the ciphers' own limits: GCM's 32-bit counter runs from 2, so past
        // (2^32 - 2) blocks it would wrap onto J0 (the tag mask) -- Go's Seal
        // panics there (gcmMaxPlaintext); ChaCha20's 32-bit block counter runs
        // from 1 (x/crypto v0.19.0: (1<<38) - 64)
        if (algo == JFSX_AES256GCM && b.len > kGcmMaxLen) return JFSX_EINVAL;
        if (algo == JFSX_CHACHA20P1305 && b.len > kCpMaxLen) return JFSX_EINVAL;
        if (crc_mode && !b.crc) return JFSX_EINVAL;
    }
    return 0;
}

// Enqueue keysetup -> transform -> finalize -> result copy for n device-resident
// blocks on stream s, using workspace w.  Results land in w.h (BlkOut[n]) once
// the stream reaches that point; finish_aead() copies them into blks.
// Stages the batch's metadata and enqueues keysetup / main / finalize on s.
// Host ingest passes up = (s_in, ev): the metadata upload then rides the
// upload stream behind the data, ev is recorded there and s waits on it; with
// collect = false the caller downloads the BlkOut results on its own stream.
// The compute stream then carries kernels only, so the H2D and D2H DMA of
// neighbouring slots run concurrently (full duplex).
// host_crc: the blocks' CRC pointers are host arrays.  VERIFY arrays ride the
// descriptor upload (copied into the pinned mirror) and GEN arrays come back
// behind the BlkOut records in the same download, so a group of per-object
// blocks costs one small copy each way instead of one per block.
// With fin = (s_out, ev) the keysetup kernel also rides the upload stream
// (after the data and descriptors) and the finalize kernel runs on fin after
// ev marks the main kernel's end: the compute stream then carries only the
// main kernels, so a small batch's keysetup and finalize -- a few waves each,
// latency-bound -- overlap the neighbouring batches' main kernels instead of
// running between them.
int enqueue_aead(jfsx_ctx *c, Workspace &w, hipStream_t s, hipEvent_t k0, hipEvent_t k1, int algo, bool open, int n,
                 const jfsx_blk *blks, int crc_mode, hipStream_t up = nullptr, hipEvent_t up_ev = nullptr,
                 bool collect = true, hipStream_t fin = nullptr, hipEvent_t main_ev = nullptr,
                 bool host_crc = false, bool zc = false, hipStream_t ksst = nullptr, hipEvent_t ks_ev = nullptr) {
    const bool gcm = algo == JFSX_AES256GCM;
    // JFSX_CRC_BOTH: the AEAD kernels checksum the plaintext (CRC_GEN) into the
    // first half of each CRC array and crc_segments_k checksums the ciphertext
    // in device memory into the second half -- before an in-place Open
    // overwrites it, after a Seal wrote it
    const bool both = (crc_mode & JFSX_CRC_BOTH) != 0;
    const int mult = both ? 2 : 1;
    crc_mode &= ~JFSX_CRC_BOTH;
    std::vector<uint64_t> lens(n);
    uint64_t crc_calc_words = 0, crc_words = 0;
    for (int i = 0; i < n; i++) {
        lens[i] = blks[i].len;
        if ((crc_mode & 3) == JFSX_CRC_VERIFY) crc_calc_words += nseg_of(blks[i].len);
        crc_words += mult * nseg_of(blks[i].len);
    }
    std::vector<Task> ctasks;  // the ciphertext pass (BOTH)
    if (both) {
        uint64_t total = 0;
        for (int i = 0; i < n; i++) total += lens[i];
        const uint64_t per = crc_task_bytes(total);
        for (int i = 0; i < n; i++)
            for (uint64_t c0 = 0; c0 < lens[i]; c0 += per) ctasks.push_back(Task{(uint32_t)i, 0, c0, std::min(c0 + per, lens[i])});
    }
    const bool hc_in = host_crc && (crc_mode & 3) == JFSX_CRC_VERIFY;
    const bool hc_out = host_crc && (crc_mode & 3) == JFSX_CRC_GEN;
    const uint32_t slots = gcm ? kSlotsPerTask : kCpWaves;
    // a small batch (the per-object path) is cut into tasks down to 64 KiB so
    // that it still spreads over the CUs (2 tasks per CU); a 64 GiB batch keeps
    // 4 MiB tasks
    Plan plan = gcm ? plan_tasks(lens, kMaxTaskBytes, kWaves, slots, 512, kGcmMinTask)
                    : plan_tasks(lens, kCpTaskBytes, kCpWaves, slots, 2048);
    const size_t nt = plan.tasks.size();
    // device workspace layout
    size_t off = 0;
    const size_t o_keys = off; off = align256(off + sizeof(KeyIn) * n);
    const size_t o_blk = off; off = align256(off + sizeof(BlkDev) * n);
    const size_t o_task = off; off = align256(off + sizeof(Task) * std::max<size_t>(nt, 1));
    const size_t o_tagin = off; off = align256(off + 16 * (size_t)n);
    const size_t o_queue = off; off = align256(off + 4);  // persistent kernel's task counter (uploaded as 0)
    const size_t o_crcin = off; if (hc_in) off = align256(off + 4 * crc_words);
    const size_t o_cblk = off; if (both) off = align256(off + sizeof(BlkDev) * n);
    const size_t o_ctask = off; if (both) off = align256(off + sizeof(Task) * std::max<size_t>(ctasks.size(), 1));
    const size_t h_bytes = off;  // everything above is uploaded from the pinned mirror
    const size_t o_out = off; off = align256(off + sizeof(BlkOut) * n);
    const size_t o_crcout = off; if (hc_out) off = align256(off + 4 * crc_words);
    const size_t down = hc_out ? o_crcout + 4 * crc_words - o_out : sizeof(BlkOut) * n;
    const size_t o_sched = off; off = align256(off + (gcm ? sizeof(GcmSched) : sizeof(CpSched)) * n);
    const size_t o_part = off; off = align256(off + 32 * std::max<uint64_t>(plan.nslots, 1));
    const size_t o_pexp = off; off = align256(off + 4 * std::max<uint64_t>(plan.nslots, 1));
    const size_t o_calc = off; off = align256(off + 4 * std::max<uint64_t>(crc_calc_words, 1));
    int rc;
    if ((rc = ensure_dev(c, &w.d, &w.dcap, off))) return rc;
    // zc: the results go straight to the pinned mirror, after the descriptors
    const size_t o_hres = zc ? h_bytes : 0;
    if ((rc = ensure_host(&w.h, &w.hcap, zc ? h_bytes + down : std::max(h_bytes, down)))) return rc;
    char *h = w.h, *d = w.d;
    KeyIn *hk = (KeyIn *)(h + o_keys);
    BlkDev *hb = (BlkDev *)(h + o_blk);
    *(uint32_t *)(h + o_queue) = 0;
    uint64_t calc = 0, cw = 0;
    for (int i = 0; i < n; i++) {
        const jfsx_blk &b = blks[i];
        memcpy(hk[i].key, b.key, 32);
        memcpy(hk[i].nonce, b.nonce, 12);
        hk[i].pad = 0;
        hb[i].src = (const uint8_t *)b.src;
        hb[i].dst = (uint8_t *)b.dst;
        hb[i].len = b.len;
        hb[i].crc = b.crc;
        if (hc_in) {
            memcpy(h + o_crcin + 4 * cw, b.crc, 4 * nseg_of(b.len));
            hb[i].crc = (uint8_t *)(d + o_crcin + 4 * cw);
        } else if (hc_out) {
            hb[i].crc = zc ? (uint8_t *)(h + o_hres + (o_crcout - o_out) + 4 * cw) : (uint8_t *)(d + o_crcout + 4 * cw);
            if (zc && b.len == 0) memset(hb[i].crc, 0, 4 * mult);  // checksum() of nothing: one zero word
        }
        if (both) {
            BlkDev &cb = ((BlkDev *)(h + o_cblk))[i];
            memset(&cb, 0, sizeof(cb));
            cb.src = open ? hb[i].src : hb[i].dst;
            cb.len = b.len;
            cb.crc = hb[i].crc + 4 * nseg_of(b.len);
        }
        cw += mult * nseg_of(b.len);
        hb[i].crc_calc = nullptr;
        if ((crc_mode & 3) == JFSX_CRC_VERIFY) {
            hb[i].crc_calc = (uint32_t *)(d + o_calc) + calc;
            calc += nseg_of(b.len);
        }
        hb[i].slot0 = 0;
        hb[i].nslots = 0;
        hb[i].tag_in = open ? (const uint8_t *)(d + o_tagin + 16 * (size_t)i) : nullptr;
        memcpy(h + o_tagin + 16 * (size_t)i, b.tag, 16);
    }
    uint32_t max_slots = 0;
    for (size_t t = 0; t < nt; t++) {
        BlkDev &bd = hb[plan.tasks[t].blk];
        if (bd.nslots == 0) bd.slot0 = plan.tasks[t].slot0;
        bd.nslots += slots;
        max_slots = std::max(max_slots, bd.nslots);
    }
    if (nt) {
        Task *ht = (Task *)(h + o_task);
        memcpy(ht, plan.tasks.data(), sizeof(Task) * nt);
#ifdef JFSX_ABLATE_TRACE
        for (size_t t = 0; t < nt; t++) ht[t].trace = (uint32_t)t;
#endif
        // the persistent transform kernels take tasks in array order: largest
        // first, so that the last tasks handed out are short (slots stay per
        // task).  A counting sort on 4 KiB units: O(n), on the host's
        // critical path for every batch
        order_largest_first(ht, nt, (size_t)(gcm ? kMaxTaskBytes : kCpTaskBytes) >> 12);
    }
    if (!ctasks.empty()) memcpy(h + o_ctask, ctasks.data(), sizeof(Task) * ctasks.size());
    // the ciphertext pass of BOTH on stream st
    auto ct_pass = [&](hipStream_t st) {
        launch_crc_segments(st, (int)ctasks.size(), (const Task *)(d + o_ctask), (const BlkDev *)(d + o_cblk), c->tabs);
    };
    const KeyIn *dk = (const KeyIn *)(d + o_keys);
    const BlkDev *db = (const BlkDev *)(d + o_blk);
    const Task *dt = (const Task *)(d + o_task);
    uint32_t *dpart = (uint32_t *)(d + o_part);
    uint32_t *dpexp = (uint32_t *)(d + o_pexp);
    uint32_t *dq = (uint32_t *)(d + o_queue);
    BlkOut *dout = zc ? (BlkOut *)(h + o_hres) : (BlkOut *)(d + o_out);
    // keysetup on the upload stream when one is given (fin set), on the
    // keysetup stream ksst (with zc: the pull too) when given, else on s
    const bool kss = zc && ksst && ks_ev;
    hipStream_t ks = kss ? ksst : (up && fin) ? up : s, fs = fin ? fin : s;
    launch_begin();
    if (zc) {
        // the compute stream (or the keysetup stream) pulls the descriptors
        // out of the pinned mirror itself, so the upload stream carries only
        // the blocks' data
        launch_pull(kss ? ksst : s, d, h, h_bytes);
    } else {
        HIP_OK(hipMemcpyAsync(d, h, h_bytes, hipMemcpyHostToDevice, up ? up : s));
    }
    // the compute stream waits for the upload before the first kernel that
    // reads what it carries: keysetup when the descriptors ride it, else main
    if (up && ks == s && !zc) {
        HIP_OK(hipEventRecord(up_ev, up));
        HIP_OK(hipStreamWaitEvent(s, up_ev, 0));
    }
    if (gcm) launch_gcm_keysetup(ks, n, dk, db, (GcmSched *)(d + o_sched), c->tabs, c->bitslice);
    else launch_cp_keysetup(ks, n, dk, db, (CpSched *)(d + o_sched));
    if (kss) {  // the descriptors and schedules are ready for the compute stream
        HIP_OK(hipEventRecord(ks_ev, ksst));
        HIP_OK(hipStreamWaitEvent(s, ks_ev, 0));
    }
    if (up && (ks != s || zc)) {
        HIP_OK(hipEventRecord(up_ev, up));
        HIP_OK(hipStreamWaitEvent(s, up_ev, 0));
    }
    if ((crc_mode & 3) == JFSX_CRC_GEN && !(zc && hc_out))
        for (int i = 0; i < n; i++)
            if (blks[i].len == 0) HIP_OK(hipMemsetAsync(hb[i].crc, 0, 4 * mult, s));
    if (both && open) ct_pass(s);
    if (c->timing) HIP_OK(hipEventRecord(k0, s));
    if (gcm)
        launch_gcm_main(s, (int)nt, c->ncu, dq, open, crc_mode, c->bitslice, dt, db, (const GcmSched *)(d + o_sched),
                        dpart, dpexp, c->tabs);
    else
        launch_cp_main(s, (int)nt, c->ncu, dq, open, crc_mode, dt, db, (const CpSched *)(d + o_sched), dpart, dpexp,
                       c->tabs);
    if (c->timing) HIP_OK(hipEventRecord(k1, s));
    if (both && !open) ct_pass(s);
    if (fin) {
        HIP_OK(hipEventRecord(main_ev, s));
        HIP_OK(hipStreamWaitEvent(fs, main_ev, 0));
    }
    if (gcm)
        launch_gcm_finalize(fs, n, open, crc_mode, db, (const GcmSched *)(d + o_sched), dpart, dpexp, dout, max_slots);
    else
        launch_cp_finalize(fs, n, open, crc_mode, db, (const CpSched *)(d + o_sched), dpart, dpexp, dout);
    HIP_OK(hipGetLastError());
    w.dout = dout;
    w.down = zc ? 0 : down;
    w.crc_off = o_crcout - o_out;
    w.crc_back = hc_out;
    w.crc_mult = mult;
    w.res_off = o_hres;
    if (collect && !zc) HIP_OK(hipMemcpyAsync(h, dout, down, hipMemcpyDeviceToHost, fs));
    w.n = n;
    w.nt = nt;
    w.timed = c->timing;
    return 0;
}

// After the batch's stream work completed: per-block results into blks.
int finish_aead(jfsx_ctx *c, Workspace &w, hipEvent_t k0, hipEvent_t k1, bool open, jfsx_blk *blks) {
    if (w.timed && w.nt) {
        float ms = 0;
        w.timed = false;
        HIP_OK(hipEventElapsedTime(&ms, k0, k1));
        add_kernel_ms(c, ms);
    }
    const BlkOut *ho = (const BlkOut *)(w.h + w.res_off);
    for (int i = 0; i < w.n; i++) {
        jfsx_blk &b = blks[i];
        if (!open) memcpy(b.tag, ho[i].tag, 16);
        b.status = ho[i].status;
        b.crc_bad_seg = ho[i].bad_seg;
        b.crc_got = ho[i].got;
        b.crc_expect = ho[i].expect;
    }
    if (w.crc_back) {
        const char *hw = w.h + w.res_off + w.crc_off;
        for (int i = 0; i < w.n; i++) {
            const size_t cb = 4 * (size_t)w.crc_mult * nseg_of(blks[i].len);
            memcpy(blks[i].crc, hw, cb);
            hw += cb;
        }
        w.crc_back = false;
    }
    w.n = 0;
    w.nt = 0;
    return 0;
}

// Open releases nothing of a block whose tag failed: Go's in-place Open
// (encrypt.go:215; crypto/cipher gcm.go and x/crypto chacha20poly1305 both
// clear `out` on a mismatch) leaves zeros, and so does the engine -- dst, and
// a plaintext CRC_GEN array (it is a function of the unauthenticated
// plaintext).  Ciphertext CRCs (JFSX_CRC_CT) stay: the object checksum is
// checked before the tag (checksum.go:55-82).  Device memory: zeroed on s.
int wipe_failed(hipStream_t s, int n, const jfsx_blk *blks, int crc_mode, bool device) {
    const bool crc_pt = (crc_mode & 3) == JFSX_CRC_GEN && !(crc_mode & JFSX_CRC_CT);
    bool any = false;
    for (int i = 0; i < n; i++) {
        const jfsx_blk &b = blks[i];
        if (b.status != JFSX_ETAG) continue;
        any = true;
        if (device) {
            if (b.len) HIP_OK(hipMemsetAsync(b.dst, 0, b.len, s));
            if (crc_pt) HIP_OK(hipMemsetAsync(b.crc, 0, 4 * nseg_of(b.len), s));
        } else {
            if (b.len) memset(b.dst, 0, b.len);
            if (crc_pt) memset(b.crc, 0, 4 * nseg_of(b.len));
        }
    }
    if (any && device) HIP_OK(hipStreamSynchronize(s));
    return 0;
}

// Device-resident batch: one enqueue, one sync (under c->mu).
int run_aead(jfsx_ctx *c, int algo, bool open, int n, jfsx_blk *blks, int crc_mode) {
    int rc = check_aead_args(algo, n, blks, crc_mode, true);
    if (rc || n == 0) return rc;
    if ((rc = enqueue_aead(c, c->ws[0], c->stream, c->ev_k0[0], c->ev_k1[0], algo, open, n, blks, crc_mode))) {
        (void)hipStreamSynchronize(c->stream);  // nothing of this batch left in flight
        c->ws[0].timed = false;
        return rc;
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    if ((rc = finish_aead(c, c->ws[0], c->ev_k0[0], c->ev_k1[0], open, blks))) return rc;
    return open ? wipe_failed(c->stream, n, blks, crc_mode, true) : 0;
}

// staging bytes of one host block in a pipeline slot (its CRC array rides the
// slot's descriptor upload / result download instead)
inline size_t host_need(const jfsx_blk &b, int) { return align256(b.len); }

// The groups of a host batch: runs of blocks of up to slot_bytes; a batch
// smaller than a few slots is cut into about 6 groups (>= 16 MiB each) so that
// its own copies and transforms overlap too.
std::vector<std::pair<int, int>> host_groups(const jfsx_ctx *c, int n, const jfsx_blk *blks, int crc_mode) {
    std::vector<std::pair<int, int>> groups;  // [b0, b1)
    size_t total = 0;
    for (int i = 0; i < n; i++) total += host_need(blks[i], crc_mode);
    const size_t slot = std::min(c->slot_bytes.load(), std::max<size_t>((size_t)16 << 20, total / 6));
    int b0 = 0;
    size_t acc = 0;
    for (int i = 0; i < n; i++) {
        const size_t need = host_need(blks[i], crc_mode);
        if (i > b0 && acc + need > slot) {
            groups.push_back({b0, i});
            b0 = i;
            acc = 0;
        }
        acc += need;
    }
    groups.push_back({b0, n});
    return groups;
}

// Enqueue the CRC-only transform (crc_segments_k + crc_finalize_k) for n
// ranges of device memory, given as block records (src, len, crc), on stream
// s with workspace w: the counterpart of enqueue_aead for checksum() and the
// ReadAt verify (disk_cache.go:1218-1231, :1315-1327).  up / up_ev, collect,
// host_crc and zc mean what they mean for enqueue_aead: the host pipeline
// passes the data's upload stream, keeps the CRC arrays in the descriptor
// upload (VERIFY) and the result download (GEN), and lets the compute stream
// pull the descriptors out of the pinned mirror.
int enqueue_crc(jfsx_ctx *c, Workspace &w, hipStream_t s, hipEvent_t k0, hipEvent_t k1, int n, const jfsx_blk *blks,
                int mode, hipStream_t up = nullptr, hipEvent_t up_ev = nullptr, bool collect = true,
                bool host_crc = false, bool zc = false) {
    uint64_t total = 0, calc_words = 0, crc_words = 0;
    for (int i = 0; i < n; i++) {
        total += blks[i].len;
        crc_words += nseg_of(blks[i].len);
        if (mode == JFSX_CRC_VERIFY) calc_words += nseg_of(blks[i].len);
    }
    const uint64_t per = crc_task_bytes(total);
    std::vector<Task> tasks;
    for (int i = 0; i < n; i++)
        for (uint64_t c0 = 0; c0 < blks[i].len; c0 += per)
            tasks.push_back(Task{(uint32_t)i, 0, c0, std::min(c0 + per, blks[i].len)});
    const bool hc_in = host_crc && mode == JFSX_CRC_VERIFY, hc_out = host_crc && mode == JFSX_CRC_GEN;
    const size_t nt = tasks.size();
    size_t off = 0;
    const size_t o_blk = off; off = align256(off + sizeof(BlkDev) * n);
    const size_t o_task = off; off = align256(off + sizeof(Task) * std::max<size_t>(nt, 1));
    const size_t o_crcin = off; if (hc_in) off = align256(off + 4 * crc_words);
    const size_t h_bytes = off;
    const size_t o_out = off; off = align256(off + sizeof(BlkOut) * n);
    const size_t o_crcout = off; if (hc_out) off = align256(off + 4 * crc_words);
    const size_t down = hc_out ? o_crcout + 4 * crc_words - o_out : sizeof(BlkOut) * n;
    const size_t o_calc = off; off = align256(off + 4 * std::max<uint64_t>(calc_words, 1));
    int rc;
    if ((rc = ensure_dev(c, &w.d, &w.dcap, off))) return rc;
    const size_t o_hres = zc ? h_bytes : 0;
    if ((rc = ensure_host(&w.h, &w.hcap, zc ? h_bytes + down : std::max(h_bytes, down)))) return rc;
    char *h = w.h, *d = w.d;
    BlkDev *hb = (BlkDev *)(h + o_blk);
    uint64_t calc = 0, cw = 0;
    for (int i = 0; i < n; i++) {
        const jfsx_blk &b = blks[i];
        memset(&hb[i], 0, sizeof(BlkDev));
        hb[i].src = (const uint8_t *)b.src;
        hb[i].len = b.len;
        hb[i].crc = b.crc;
        if (hc_in) {
            memcpy(h + o_crcin + 4 * cw, b.crc, 4 * nseg_of(b.len));
            hb[i].crc = (uint8_t *)(d + o_crcin + 4 * cw);
        } else if (hc_out) {
            hb[i].crc = zc ? (uint8_t *)(h + o_hres + (o_crcout - o_out) + 4 * cw) : (uint8_t *)(d + o_crcout + 4 * cw);
        }
        cw += nseg_of(b.len);
        if (mode == JFSX_CRC_VERIFY) {
            hb[i].crc_calc = (uint32_t *)(d + o_calc) + calc;
            calc += nseg_of(b.len);
        }
    }
    if (nt) memcpy(h + o_task, tasks.data(), sizeof(Task) * nt);
    BlkOut *dout = zc ? (BlkOut *)(h + o_hres) : (BlkOut *)(d + o_out);
    launch_begin();
    if (zc) launch_pull(s, d, h, h_bytes);
    else HIP_OK(hipMemcpyAsync(d, h, h_bytes, hipMemcpyHostToDevice, up ? up : s));
    if (up) {
        HIP_OK(hipEventRecord(up_ev, up));
        HIP_OK(hipStreamWaitEvent(s, up_ev, 0));
    }
    if (c->timing) HIP_OK(hipEventRecord(k0, s));
    launch_crc_segments(s, (int)nt, (const Task *)(d + o_task), (const BlkDev *)(d + o_blk), c->tabs);
    if (c->timing) HIP_OK(hipEventRecord(k1, s));
    launch_crc_finalize(s, n, mode, (const BlkDev *)(d + o_blk), dout);
    HIP_OK(hipGetLastError());
    w.dout = dout;
    w.down = zc ? 0 : down;
    w.crc_off = o_crcout - o_out;
    w.crc_back = hc_out;
    w.crc_mult = 1;
    w.res_off = o_hres;
    if (collect && !zc) HIP_OK(hipMemcpyAsync(h, dout, down, hipMemcpyDeviceToHost, s));
    w.n = n;
    w.nt = nt;
    w.timed = c->timing;
    return 0;
}

// How a host thread waits for a pipeline slot's D2H (JFSX_WAIT_POLL_US): by
// default it queries the event and sleeps 20 us between queries; 0 =
// hipEventSynchronize, the runtime's wait, which keeps a core busy for the
// whole wait (with or without hipEventBlockingSync).  A group's wait is about
// a millisecond and several dispatchers wait at once: 20 per-object callers on
// pinned blocks kept 5.0 cores busy with the runtime's wait and 1.25 with the
// sleeping one, at the same 41.6-41.9 GB/s (profiles/r6/wait_poll/).
int wait_poll_us() {
    static const int v = [] {
        const char *e = getenv("JFSX_WAIT_POLL_US");
        return e ? atoi(e) : 20;
    }();
    return v;
}

hipError_t wait_event(hipEvent_t ev) {
    const int us = wait_poll_us();
    if (us <= 0) return hipEventSynchronize(ev);
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e != hipErrorNotReady) return e;
        (void)hipGetLastError();  // hipErrorNotReady is not a failure
        std::this_thread::sleep_for(std::chrono::microseconds(us));
    }
}

// Collect the group in flight in slot s (s.mu held; called by the group's own
// caller, or by any caller that needs the slot next): wait for its D2H and
// write its per-block results into the owner's records.  Only results: the
// owner copies its bounced outputs out itself.
void pipe_collect(jfsx_ctx *c, PipeSlot &s) {
    PipeGroup *g = s.owner;
    if (!g) return;
    s.owner = nullptr;
    const hipError_t e = wait_event(s.ev_out);
    if (e != hipSuccess) {
        note_hip_error(e, __FILE__, __LINE__, "hipEventSynchronize(pipeline slot)");
        g->rc = JFSX_EIO;
        s.w.crc_back = false;
        s.w.n = 0;
        s.w.nt = 0;
        s.w.timed = false;
        return;
    }
    g->rc = finish_aead(c, s.w, s.ev_k0, s.ev_k1, g->open, g->dv);
}

// The host pipeline's metadata path: with it (the default) the compute stream
// pulls each group's descriptors out of the pinned mirror with a small kernel
// and finalize writes the per-block results (and GEN CRC words) straight into
// it, so the copy streams carry only block data -- small copies on them run as
// blit kernels between the SDMA transfers.  JFSX_PIPE_META=copy restores the
// metadata copies.
bool zero_copy_meta() {
    static const bool v = [] {
        const char *e = getenv("JFSX_PIPE_META");
        return !(e && !strcmp(e, "copy"));
    }();
    return v;
}

// The host pipeline's keysetup stream (JFSX_KS_STREAM, default on): each
// group's descriptor pull and keysetup kernel run on a fourth stream, so they
// overlap the previous group's main kernel instead of queueing behind it on
// the compute stream (the compute stream waits for them before the main
// kernel).  For a group of a few small blocks keysetup is most of the
// compute stream's time (54 us of 137 per group of 64 KiB blocks, rocprof).
bool ks_stream() {
    static const bool v = [] {
        const char *e = getenv("JFSX_KS_STREAM");
        return !(e && !strcmp(e, "0"));
    }();
    return v;
}

enum PipeOp { kPipeSeal, kPipeOpen, kPipeCrc };

// One group into an empty slot (s.mu and c->mu held): the blocks' data runs up
// on s_in into the slot's staging (coalesced where the blocks are adjacent in
// host memory -- a group's bounced blocks always are), then the transform on
// the compute stream (AEAD: keysetup / main / finalize; CRC: crc_segments /
// crc_finalize); the AEAD outputs run down on s_out, chained by the slot's
// events.  blks hold page-locked host addresses only (run_host substituted the
// bounce buffer for pageable ones); dv[i] (the call's copy of the caller's
// record) is pointed at the staging copy.  (A variant whose kernel wrote the
// outputs straight into engine-pinned caller memory over PCIe ran at 25 GB/s
// against 38.7 staged and was removed.)
int pipe_enqueue(jfsx_ctx *c, PipeSlot &s, PipeOp op, int algo, int nb, const jfsx_blk *blks, jfsx_blk *dv,
                 int crc_mode, const uintptr_t *in_id, const uintptr_t *out_id) {
    Workspace &w = s.w;
    size_t need = 0;
    for (int i = 0; i < nb; i++) need += host_need(blks[i], crc_mode);
    int rc;
    if ((rc = ensure_dev(c, &w.stage, &w.scap, std::max<size_t>(need, 256)))) return rc;
    size_t off = 0;
    // staging in the order of the source addresses: blocks that are
    // neighbours in host memory (pages of one pinned pool, or one bounce
    // buffer) then sit side by side in staging too, and their copies coalesce
    // both ways whatever order the callers submitted them in
    std::vector<int> ord(nb);
    for (int i = 0; i < nb; i++) ord[i] = i;
    if (nb > 1)
        std::stable_sort(ord.begin(), ord.end(),
                         [&](int a, int b) { return (uintptr_t)blks[a].src < (uintptr_t)blks[b].src; });
    const char *run_h = nullptr;
    char *run_d = nullptr;
    size_t run_n = 0;
    uintptr_t run_id = 0;
    auto flush_in = [&]() -> int {
        if (run_n) {
            HIP_OK(hipMemcpyAsync(run_d, run_h, run_n, hipMemcpyHostToDevice, c->s_in));
            c->ps_h2d++;
        }
        run_n = 0;
        return 0;
    };
    for (int k = 0; k < nb; k++) {
        const int i = ord[k];
        char *buf = w.stage + off;
        off += align256(blks[i].len);
        if (blks[i].len) {
            const char *hs = (const char *)blks[i].src;
            // one copy may only span one host allocation (a pinned pool, a
            // bounce buffer): in_id names the allocation, 0 = the block's own
            if (!(run_n && run_h + run_n == hs && run_d + run_n == buf && in_id[i] && in_id[i] == run_id) &&
                (rc = flush_in()))
                return rc;
            if (!run_n) {
                run_h = hs;
                run_d = buf;
                run_id = in_id[i];
            }
            run_n += blks[i].len;
            if (align256(blks[i].len) != blks[i].len && (rc = flush_in())) return rc;
        }
        dv[i].src = buf;
        dv[i].dst = op == kPipeCrc ? nullptr : buf;
    }
    if ((rc = flush_in())) return rc;
    // the transform on the compute stream.  (Moving keysetup onto s_in and
    // finalize onto s_out, to overlap them with neighbouring groups' main
    // kernels, measured 30-33 GB/s against 38-40 at 20 per-object callers:
    // the copy engines then wait behind those kernels.)  The CRC arrays pass
    // through the descriptor upload and the result download (host_crc).
    if (op == kPipeCrc)
        rc = enqueue_crc(c, w, c->stream, s.ev_k0, s.ev_k1, nb, dv, crc_mode, c->s_in, s.ev_in, false, true,
                         zero_copy_meta());
    else
        rc = enqueue_aead(c, w, c->stream, s.ev_k0, s.ev_k1, algo, op == kPipeOpen, nb, dv, crc_mode, c->s_in,
                          s.ev_in, false, nullptr, nullptr, true, zero_copy_meta(), ks_stream() ? c->s_ks : nullptr,
                          s.ev_ks);
    if (rc) return rc;
    HIP_OK(hipEventRecord(s.ev_comp, c->stream));
    HIP_OK(hipStreamWaitEvent(c->s_out, s.ev_comp, 0));
    char *oh = nullptr;
    const char *od = nullptr;
    size_t on = 0;
    uintptr_t oid = 0;
    auto flush_out = [&]() -> int {
        if (on) {
            HIP_OK(hipMemcpyAsync(oh, od, on, hipMemcpyDeviceToHost, c->s_out));
            c->ps_d2h++;
        }
        on = 0;
        return 0;
    };
    for (int k = 0; k < nb && op != kPipeCrc; k++) {
        const int i = ord[k];
        if (!blks[i].len) continue;
        char *hd = (char *)blks[i].dst;
        const char *dd = (const char *)dv[i].dst;
        if (!(on && oh + on == hd && od + on == dd && out_id[i] && out_id[i] == oid) && (rc = flush_out())) return rc;
        if (!on) {
            oh = hd;
            od = dd;
            oid = out_id[i];
        }
        on += blks[i].len;
        if (align256(blks[i].len) != blks[i].len && (rc = flush_out())) return rc;
    }
    if ((rc = flush_out())) return rc;
    if (w.down) HIP_OK(hipMemcpyAsync(w.h, w.dout, w.down, hipMemcpyDeviceToHost, c->s_out));
    HIP_OK(hipEventRecord(s.ev_out, c->s_out));
    return 0;
}

// A pipeline slot for the next group, locked.  Under c->mu only the choice is
// made: the first slot from the ring position on that is unlocked and whose
// group (if any) has finished its D2H, else the next slot in ring order.  The
// wait for a busy slot then happens under that slot's lock alone, so a caller
// waiting for another caller's group holds up nothing else on the context
// (device batches, CRC and codec calls, other callers' enqueues).
PipeSlot *claim_slot(jfsx_ctx *c) {
    PipeSlot *s = nullptr;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        for (int k = 0; k < kPipe && !s; k++) {
            PipeSlot &q = c->pipe[(c->pipe_next + k) % kPipe];
            if (!q.mu.try_lock()) continue;
            bool idle = !q.owner;
            if (!idle) {
                idle = hipEventQuery(q.ev_out) == hipSuccess;
                (void)hipGetLastError();  // hipErrorNotReady is not a failure of this call
            }
            if (idle) {
                s = &q;
                c->pipe_next = (c->pipe_next + k + 1) % kPipe;
            } else {
                q.mu.unlock();
            }
        }
        if (s) return s;
        s = &c->pipe[c->pipe_next];
        c->pipe_next = (c->pipe_next + 1) % kPipe;
    }
    s->mu.lock();
    return s;
}

// bounce buffers: capacity classes of 1 MiB up to 16 MiB, then 16 MiB
size_t bounce_class(size_t need) {
    const size_t mib = (size_t)1 << 20, step = need <= 16 * mib ? mib : 16 * mib;
    return (std::max<size_t>(need, 1) + step - 1) / step * step;
}

// idle buffers kept per context (JFSX_BOUNCE_RETAIN_MB, default 1 GiB)
size_t bounce_retain() {
    static const size_t v = [] {
        const char *e = getenv("JFSX_BOUNCE_RETAIN_MB");
        return (e ? (size_t)atoll(e) : (size_t)1024) << 20;
    }();
    return v;
}

int alloc_pinned_on(int node, size_t bytes, void **p);

char *bounce_get(jfsx_ctx *c, size_t need, size_t *cap) {
    BouncePool &b = c->bounce;
    {
        std::lock_guard<std::mutex> g(b.mu);
        auto it = b.idle.lower_bound(need);
        if (it != b.idle.end() && it->first <= std::max(2 * need, need + ((size_t)1 << 20))) {
            char *p = it->second;
            *cap = it->first;
            b.idle_bytes -= it->first;
            b.idle.erase(it);
            return p;
        }
    }
    const size_t n = bounce_class(need);
    void *p = nullptr;
    if (alloc_pinned_on(c->numa_node, n, &p)) return nullptr;
    note_pinned(p, n);  // so host_pinned() knows a bounced block at once
    b.allocs++;
    *cap = n;
    return (char *)p;
}

// Back to the idle list.  Over the retention cap the largest idle buffers go
// first, so one big pageable host-ingest call's buffers do not crowd out the
// per-object ones (which would then be allocated and freed on every call).
void bounce_put(jfsx_ctx *c, char *p, size_t cap) {
    BouncePool &b = c->bounce;
    std::vector<char *> drop;
    {
        std::lock_guard<std::mutex> g(b.mu);
        b.idle.emplace(cap, p);
        b.idle_bytes += cap;
        while (b.idle_bytes > bounce_retain() && !b.idle.empty()) {
            auto it = std::prev(b.idle.end());
            b.idle_bytes -= it->first;
            drop.push_back(it->second);
            b.idle.erase(it);
        }
    }
    for (char *q : drop) {
        forget_pinned(q);
        (void)hipHostFree(q);
    }
}

}  // namespace

namespace jfsx {
// the aggregator stages pageable per-object requests on the calling thread
// with these (jfsx_agg.cpp)
char *bounce_acquire(jfsx_ctx *c, size_t need, size_t *cap) {
    CtxScope es_(c);
    (void)hipSetDevice(c->device);
    return bounce_get(c, need, cap);
}
void bounce_release(jfsx_ctx *c, char *p, size_t cap) { bounce_put(c, p, cap); }
void bounce_count(jfsx_ctx *c, uint64_t in, uint64_t out) {
    c->bounce.bytes_in += in;
    c->bounce.bytes_out += out;
}
}  // namespace jfsx

namespace {

// memcpy of a group's blocks into / out of its bounce buffer: on the calling
// thread (each per-object caller copies its own block, so max-uploads callers
// copy in parallel); one caller's big group (a host-ingest batch from pageable
// memory) is split over helper threads so the host copy keeps up with PCIe
int copy_threads() {  // JFSX_COPY_THREADS (default 8)
    static const int v = [] {
        const char *e = getenv("JFSX_COPY_THREADS");
        const int t = e ? atoi(e) : 8;
        return t >= 1 && t <= 64 ? t : 8;
    }();
    return v;
}

void par_copy(std::vector<std::pair<char *, const char *>> &ds, const std::vector<size_t> &lens) {
    size_t total = 0;
    for (size_t l : lens) total += l;
    const size_t mib = (size_t)1 << 20;
    const int nt = total >= 32 * mib ? (int)std::min<size_t>((size_t)copy_threads(), total / (8 * mib)) : 1;
    // bytes [lo, hi) of the concatenated items
    auto work = [&](size_t lo, size_t hi) {
        size_t base = 0;
        for (size_t k = 0; k < ds.size() && base < hi; base += lens[k], k++) {
            const size_t a = std::max(lo, base), b = std::min(hi, base + lens[k]);
            if (a < b) memcpy(ds[k].first + (a - base), ds[k].second + (a - base), b - a);
        }
    };
    if (nt <= 1) {
        work(0, total);
        return;
    }
    std::vector<std::thread> ts;
    for (int t = 1; t < nt; t++) ts.emplace_back(work, total * t / nt, total * (t + 1) / nt);
    work(0, total / nt);
    for (std::thread &t : ts) t.join();
}

// Host-memory call (host ingest, the per-object shim, checksum() / ReadAt
// verify on host memory).  The call is cut into groups; for each group the
// calling thread (1) copies its pageable blocks into a bounce buffer, (2)
// claims a pipeline slot, collects whatever group still occupies it, (3)
// enqueues the group under c->mu and moves on.  It then waits for its own
// groups' D2H events only, copying each group's bounced outputs out as it
// completes (after at most a few groups in flight, when it holds bounce
// buffers, so one big pageable call pins no more than that).  So concurrent
// callers keep the H2D and D2H engines busy back to back instead of filling
// and draining the ring once per call.  Open releases no plaintext of a block
// whose tag failed: its destination is wiped before the call returns.  On an
// enqueue error the three streams are drained first, so an error return means
// nothing of the call is still copying into the caller's buffers.
int run_host(jfsx_ctx *c, PipeOp op, int algo, int n, jfsx_blk *blks, int crc_mode) {
    int rc = 0;
    const bool open = op == kPipeOpen;
    const std::vector<std::pair<int, int>> groups = host_groups(c, n, blks, crc_mode);
    std::vector<jfsx_blk> dv(blks, blks + n), hv(blks, blks + n);
    std::vector<char> out_b(n, 0);  // block i's output sits in the bounce buffer
    // the host allocation of each block's source / destination copy, for
    // coalescing (pinned_base; the bounce buffer; 0: copy the block alone)
    std::vector<uintptr_t> in_id(n, 0), out_id(n, 0);
    std::vector<PipeGroup> recs(groups.size());
    size_t issued = 0, done = 0, held = 0;  // groups enqueued / finished; bounce bytes held
    size_t pinned_held = 0;                 // caller ranges pinned by groups in flight
    using SClock = std::chrono::steady_clock;
    auto us = [](SClock::time_point a, SClock::time_point b) {
        return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
    };
    std::vector<std::pair<char *, const char *>> cp;
    std::vector<size_t> cl;
    // wait for group g, copy its bounced outputs out, release its bounce buffer
    auto finish = [&](size_t g) {
        PipeGroup &r = recs[g];
        const SClock::time_point f0 = SClock::now();
        {
            std::lock_guard<std::mutex> sl(r.slot->mu);
            if (r.slot->owner == &r) pipe_collect(c, *r.slot);
        }
        const SClock::time_point f1 = SClock::now();
        c->ps_wait_us += us(f0, f1);
        if (!r.rc) {
            cp.clear();
            cl.clear();
            for (int i = groups[g].first; i < groups[g].second; i++)
                if (out_b[i] && !(open && dv[i].status == JFSX_ETAG)) {
                    cp.push_back({(char *)blks[i].dst, (const char *)hv[i].dst});
                    cl.push_back(blks[i].len);
                    c->bounce.bytes_out += blks[i].len;
                }
            par_copy(cp, cl);
            c->ps_bout_us += us(f1, SClock::now());
        }
        if (r.bounce) {
            bounce_put(c, r.bounce, r.bcap);
            held -= r.bcap;
            r.bounce = nullptr;
        }
        for (const void *q : r.pins) host_unpin(q);
        r.pins.clear();
        if (r.rc && !rc) rc = r.rc;
    };
    for (size_t g = 0; g < groups.size() && !rc; g++) {
        const int b0 = groups[g].first, b1 = groups[g].second;
        PipeGroup &r = recs[g];
        // (1) bounce the group's pageable blocks: one region per block, used
        // by its input (copied in here) and / or its output (copied out by
        // finish); in place when src == dst
        const SClock::time_point p0 = SClock::now();
        size_t need = 0;
        std::vector<size_t> boff(b1 - b0, SIZE_MAX);
        std::vector<char> in_pg(b1 - b0, 0);
        for (int i = b0; i < b1; i++) {
            const jfsx_blk &b = blks[i];
            if (!b.len) continue;
            in_pg[i - b0] = !host_pinned(b.src, b.len);
            out_b[i] = op != kPipeCrc && (b.dst == b.src ? in_pg[i - b0] : !host_pinned(b.dst, b.len));
            // pin the caller's own pages for the call where the runtime
            // allows it; what stays unpinned is bounced
            if (in_pg[i - b0] && host_pin(b.src, b.len)) {
                r.pins.push_back(b.src);
                in_pg[i - b0] = 0;
                if (b.dst == b.src) out_b[i] = 0;
            }
            if (out_b[i] && host_pin(b.dst, b.len)) {
                r.pins.push_back(b.dst);
                out_b[i] = 0;
            }
            in_id[i] = pinned_base(b.src);
            out_id[i] = op == kPipeCrc ? 0 : pinned_base(b.dst);
            if (!in_pg[i - b0] && !out_b[i]) continue;
            boff[i - b0] = need;
            need += align256(b.len);
        }
        const SClock::time_point p1 = SClock::now();
        c->ps_pin_us += us(p0, p1);
        if (need) {
            if (!(r.bounce = bounce_get(c, need, &r.bcap))) {
                for (const void *q : r.pins) host_unpin(q);
                r.pins.clear();
                rc = JFSX_ENOMEM;
                break;
            }
            held += r.bcap;
            cp.clear();
            cl.clear();
            for (int i = b0; i < b1; i++) {
                if (boff[i - b0] == SIZE_MAX) continue;
                char *q = r.bounce + boff[i - b0];
                if (in_pg[i - b0]) {
                    cp.push_back({q, (const char *)blks[i].src});
                    cl.push_back(blks[i].len);
                    hv[i].src = q;
                    in_id[i] = (uintptr_t)r.bounce;
                    c->bounce.bytes_in += blks[i].len;
                }
                if (out_b[i]) {
                    hv[i].dst = q;
                    out_id[i] = (uintptr_t)r.bounce;
                }
            }
            par_copy(cp, cl);
            c->ps_bin_us += us(p1, SClock::now());
        }
        // (2) a slot, (3) the enqueue
        const SClock::time_point t0 = SClock::now();
        PipeSlot &s = *claim_slot(c);
        pipe_collect(c, s);
        const SClock::time_point t1 = SClock::now();
        {
            std::lock_guard<std::mutex> lk(c->mu);
            rc = pipe_enqueue(c, s, op, algo, b1 - b0, hv.data() + b0, dv.data() + b0, crc_mode, in_id.data() + b0,
                              out_id.data() + b0);
            if (rc) {
                (void)hipStreamSynchronize(c->s_in);
                (void)hipStreamSynchronize(c->stream);
                (void)hipStreamSynchronize(c->s_out);
                s.w.n = 0;
                s.w.nt = 0;
                s.w.timed = false;
                s.w.crc_back = false;
            }
        }
        c->ps_slot_us += us(t0, t1);
        c->ps_enq_us += us(t1, SClock::now());
        c->ps_groups++;
        c->ps_blocks += (uint64_t)(b1 - b0);
        if (rc) {
            s.mu.unlock();
            if (r.bounce) {
                bounce_put(c, r.bounce, r.bcap);
                held -= r.bcap;
                r.bounce = nullptr;
            }
            for (const void *q : r.pins) host_unpin(q);
            r.pins.clear();
            break;
        }
        r.slot = &s;
        r.dv = dv.data() + b0;
        r.open = open;
        s.owner = &r;
        s.mu.unlock();
        issued++;
        // a call holding bounce buffers or pinned caller pages keeps at most
        // 4 groups / 1 GiB of them in flight
        pinned_held += r.pins.size();
        while ((held || pinned_held) && (issued - done > 4 || held > ((size_t)1 << 30))) {
            pinned_held -= recs[done].pins.size();
            finish(done++);
        }
    }
    const SClock::time_point tw = SClock::now();
    while (done < issued) finish(done++);
    c->ps_own_us += us(tw, SClock::now());
    if (rc) return rc;
    for (int i = 0; i < n; i++) {
        blks[i].status = dv[i].status;
        blks[i].crc_bad_seg = dv[i].crc_bad_seg;
        blks[i].crc_got = dv[i].crc_got;
        blks[i].crc_expect = dv[i].crc_expect;
        if (op != kPipeOpen && op != kPipeCrc) memcpy(blks[i].tag, dv[i].tag, 16);
    }
    return open ? wipe_failed(c->stream, n, blks, crc_mode, false) : 0;
}

int run_aead_host(jfsx_ctx *c, int algo, bool open, int n, jfsx_blk *blks, int crc_mode) {
    int rc = check_aead_args(algo, n, blks, crc_mode, false);
    if (rc || n == 0) return rc;
    return run_host(c, open ? kPipeOpen : kPipeSeal, algo, n, blks, crc_mode);
}

int check_crc_args(int n, const jfsx_range *r, int mode, bool device) {
    if (n < 0 || (mode != JFSX_CRC_GEN && mode != JFSX_CRC_VERIFY)) return JFSX_EINVAL;
    for (int i = 0; i < n; i++) {
        if (r[i].len && (!r[i].data || (device && !aligned16(r[i].data)))) return JFSX_EINVAL;
        if (!r[i].crc) return JFSX_EINVAL;
    }
    return 0;
}

// ranges as the block records the pipeline and enqueue_crc take
std::vector<jfsx_blk> ranges_as_blocks(int n, const jfsx_range *r) {
    std::vector<jfsx_blk> b(n);
    for (int i = 0; i < n; i++) {
        memset(&b[i], 0, sizeof(jfsx_blk));
        b[i].src = r[i].data;
        b[i].len = r[i].len;
        b[i].crc = r[i].crc;
    }
    return b;
}

void blocks_to_ranges(int n, const jfsx_blk *b, jfsx_range *r) {
    for (int i = 0; i < n; i++) {
        r[i].status = b[i].status;
        r[i].bad_seg = b[i].crc_bad_seg;
        r[i].got = b[i].crc_got;
        r[i].expect = b[i].crc_expect;
    }
}

// Device-memory CRC batch: one enqueue, one sync (under c->mu).
int run_crc(jfsx_ctx *c, int n, jfsx_range *r, int mode) {
    int rc = check_crc_args(n, r, mode, true);
    if (rc || n == 0) return rc;
    std::vector<jfsx_blk> b = ranges_as_blocks(n, r);
    if ((rc = enqueue_crc(c, c->ws[0], c->stream, c->ev_k0[0], c->ev_k1[0], n, b.data(), mode))) {
        (void)hipStreamSynchronize(c->stream);
        c->ws[0].timed = false;
        return rc;
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    if ((rc = finish_aead(c, c->ws[0], c->ev_k0[0], c->ev_k1[0], true, b.data()))) return rc;
    blocks_to_ranges(n, b.data(), r);
    return 0;
}

// Host-memory CRC call: through the host pipeline, like a host AEAD call (no
// context lock held while it waits; pageable ranges bounced by the caller).
int run_crc_host(jfsx_ctx *c, int n, jfsx_range *r, int mode) {
    int rc = check_crc_args(n, r, mode, false);
    if (rc || n == 0) return rc;
    std::vector<jfsx_blk> b = ranges_as_blocks(n, r);
    if ((rc = run_host(c, kPipeCrc, 0, n, b.data(), mode))) return rc;
    blocks_to_ranges(n, b.data(), r);
    return 0;
}

constexpr uint64_t kLz4MaxInput = 0x7E000000ull;  // LZ4_MAX_INPUT_SIZE
uint64_t lz4_bound(uint64_t n) { return n > kLz4MaxInput ? 0 : n + n / 255 + 16; }
// ZSTD_compressBound
uint64_t zstd_bound(uint64_t n) { return n + (n >> 8) + (n < (128u << 10) ? ((128u << 10) - n) >> 11 : 0); }

enum CodecOp { kLz4Comp, kLz4Decomp, kZstdDecomp, kZstdComp };

// The codec stages (jfsx_lz4.hip, jfsx_zstd.hip, jfsx_zstdc.hip): one wave per
// object.  Host-memory batches are staged through the context's slot-0
// staging buffer (inputs up, the out_len bytes of each output down).
int run_codec(jfsx_ctx *c, int n, jfsx_zblk *z, int mem, CodecOp op) {
    if (n < 0 || (mem != JFSX_MEM_DEVICE && mem != JFSX_MEM_HOST)) return JFSX_EINVAL;
    for (int i = 0; i < n; i++) {
        if ((z[i].src_len && !z[i].src) || (z[i].dst_cap && !z[i].dst) || z[i].src_len > kLz4MaxInput ||
            z[i].dst_cap >= ((uint64_t)1 << 32))
            return JFSX_EINVAL;
        if (op == kLz4Comp && z[i].dst_cap < lz4_bound(z[i].src_len)) return JFSX_EINVAL;
        if (op == kZstdComp && z[i].dst_cap < zstd_bound(z[i].src_len)) return JFSX_EINVAL;
        if (op == kZstdDecomp && z[i].dst_cap >= ((uint64_t)1 << 31)) return JFSX_EINVAL;  // 32-bit frame positions
    }
    if (n == 0) return 0;
    int rc;
    Workspace &w = c->ws[0];
    // zstd compression: persistent waves per CU (JFSX_ZC_WAVES overrides the
    // default for A/B; LDS and VGPRs allow 16)
    static const int zc_per_cu = getenv("JFSX_ZC_WAVES") ? std::max(1, std::min(16, atoi(getenv("JFSX_ZC_WAVES"))))
                                                         : kZcWavesPerCu;
    const int zc_waves = std::min(n, c->ncu * zc_per_cu);
    static const bool zc_queue = getenv("JFSX_ZC_QUEUE") && atoi(getenv("JFSX_ZC_QUEUE")) == 1;
    // zstd decompression: block-parallel persistent waves unless
    // JFSX_ZSTD_SERIAL=1 selects the one-wave-per-object serial kernel (A/B)
    static const bool zd_serial = getenv("JFSX_ZSTD_SERIAL") && atoi(getenv("JFSX_ZSTD_SERIAL")) == 1;
    // the block-parallel decoder's waves are capped by the context's arena
    // budget (a 64-object batch needs 64 arenas, not 8 per CU); if the
    // workspace cannot grow to that many, fewer waves are tried, then the
    // serial kernel, whose scratch is n x kZstdScratch (128 KiB per object)
    int zd_waves = op == kZstdDecomp && !zd_serial ? zstd_par_waves(n, c->ncu) : 0;
    if (zd_waves) zd_waves = (int)std::min<size_t>((size_t)zd_waves, std::max<size_t>(c->zstd_arena_budget / kZstdArena, 1));
    const size_t o_out = align256(sizeof(ZDev) * n), o_tab = o_out + align256(sizeof(ZOut) * n);
    ErrRec before;  // a hipMalloc failure the arena fallback recovers from is not recorded
    {
        std::lock_guard<std::mutex> g(c->err_mu);
        before = c->err;
    }
    for (;;) {
        size_t extra = 0;
        if (op == kLz4Comp) extra = kLz4TabBytes * (size_t)n;
        else if (op == kZstdDecomp) extra = zd_waves ? kZstdArena * (size_t)zd_waves : kZstdScratch * (size_t)n;
        else if (op == kZstdComp) extra = 256 + kZstdcScratch * (size_t)zc_waves;  // per-wave scratch
        rc = ensure_dev(c, &w.d, &w.dcap, o_tab + extra);
        if (rc != JFSX_ENOMEM || op != kZstdDecomp || zd_waves == 0) break;
        zd_waves = zd_waves > c->ncu ? std::max(zd_waves / 2, c->ncu) : 0;  // fewer waves, then serial
        (void)hipGetLastError();  // the failed hipMalloc is not this batch's error
        {
            std::lock_guard<std::mutex> g(c->err_mu);
            c->err = before;
        }
    }
    if (rc) return rc;
    if ((rc = ensure_host(&w.h, &w.hcap, o_tab))) return rc;  // descriptors and results only
    hipStream_t s = c->stream;
    ZDev *hz = (ZDev *)w.h;
    std::vector<char *> sdst(n, nullptr);
    if (mem == JFSX_MEM_HOST) {
        size_t need = 0;
        for (int i = 0; i < n; i++) need += align256(z[i].src_len) + align256(z[i].dst_cap);
        if ((rc = ensure_dev(c, &w.stage, &w.scap, std::max<size_t>(need, 256)))) return rc;
        size_t off = 0;
        for (int i = 0; i < n; i++) {
            char *in = w.stage + off;
            off += align256(z[i].src_len);
            sdst[i] = w.stage + off;
            off += align256(z[i].dst_cap);
            if (z[i].src_len) HIP_OK(hipMemcpyAsync(in, z[i].src, z[i].src_len, hipMemcpyHostToDevice, s));
            hz[i] = ZDev{(const uint8_t *)in, (uint8_t *)sdst[i], z[i].src_len, z[i].dst_cap};
        }
    } else {
        for (int i = 0; i < n; i++)
            hz[i] = ZDev{(const uint8_t *)z[i].src, (uint8_t *)z[i].dst, z[i].src_len, z[i].dst_cap};
    }
    HIP_OK(hipMemcpyAsync(w.d, w.h, sizeof(ZDev) * n, hipMemcpyHostToDevice, s));
    if (c->timing) HIP_OK(hipEventRecord(c->ev_k0[0], s));
    const ZDev *dz = (const ZDev *)w.d;
    ZOut *dout = (ZOut *)(w.d + o_out);
    launch_begin();
    switch (op) {
    case kLz4Comp:
        launch_lz4_compress(s, n, c->ncu, dz, dout, (uint32_t *)(w.d + o_tab));
        break;
    case kLz4Decomp:
        launch_lz4_decompress(s, n, dz, dout);
        break;
    case kZstdDecomp:
        launch_zstd_decompress(s, n, dz, dout, (uint8_t *)(w.d + o_tab), zd_waves);
        break;
    case kZstdComp:
        // JFSX_ZC_QUEUE=1: ticket-queue object assignment (A/B; the word
        // before the scratch is the ticket counter)
        launch_zstd_compress(s, n, zc_waves, dz, dout, (uint8_t *)(w.d + o_tab + 256),
                             zc_queue ? (uint32_t *)(w.d + o_tab) : nullptr);
        break;
    }
    if (c->timing) HIP_OK(hipEventRecord(c->ev_k1[0], s));
    HIP_OK(hipGetLastError());
    ZOut *ho = (ZOut *)(w.h + o_out);
    HIP_OK(hipMemcpyAsync(ho, dout, sizeof(ZOut) * n, hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamSynchronize(s));
    if (c->timing) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, c->ev_k0[0], c->ev_k1[0]));
        add_kernel_ms(c, ms);
    }
    for (int i = 0; i < n; i++) {
        z[i].out_len = ho[i].out_len;
        z[i].status = ho[i].status;
        if (op == kZstdDecomp) {
            z[i].reserved = zd_waves ? ho[i].fallback : 0;
            if (zd_waves && ho[i].fallback) {
                std::lock_guard<std::mutex> g(c->stat_mu);
                c->met.zstd_serial++;
            }
        }
        if (mem == JFSX_MEM_HOST && ho[i].out_len)
            HIP_OK(hipMemcpyAsync(z[i].dst, sdst[i], ho[i].out_len, hipMemcpyDeviceToHost, s));
    }
    if (mem == JFSX_MEM_HOST) HIP_OK(hipStreamSynchronize(s));
    return 0;
}

}  // namespace

namespace jfsx {
// The device that owns p, with the bounds [lo, hi) of the allocation it lies
// in (so a caller can skip lookups for neighbouring pointers); -1 when p is
// not device memory.  jfsx_alloc_device allocations are found in the
// registry (an allocation must then be released with jfsx_free_device, which
// drops its entry; one released with hipFree leaves a stale range behind);
// other pointers are asked of the HIP runtime, which also reports the
// allocation's bounds, so the caller's range cache covers their neighbours.
int device_of(const void *p, uintptr_t *lo, uintptr_t *hi) {
    const uintptr_t a = (uintptr_t)p;
    {
        std::shared_lock<std::shared_mutex> g(g_alloc_mu);
        auto it = g_allocs.upper_bound(a);
        if (it != g_allocs.begin()) {
            --it;
            if (a < it->second.first) {
                *lo = it->first;
                *hi = it->second.first;
                return it->second.second;
            }
        }
    }
    *lo = a;
    *hi = a + 1;
    hipPointerAttribute_t at;
    if (p && hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeDevice) {
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) == hipSuccess && base && size &&
            (uintptr_t)base <= a && a < (uintptr_t)base + size) {
            *lo = (uintptr_t)base;
            *hi = (uintptr_t)base + size;
        }
        (void)hipGetLastError();
        return at.device;
    }
    (void)hipGetLastError();
    return -1;
}
}  // namespace jfsx

// ===========================================================================
// exported C-ABI
// ===========================================================================
extern "C" {

int jfsx_abi_version(void) { return JFSX_ABI_VERSION; }

int jfsx_last_error(jfsx_ctx *c, int *hip_error, char *msg, size_t cap) {
    ErrRec e;
    if (c) {
        std::lock_guard<std::mutex> g(c->err_mu);
        e = c->err;
    } else {
        e = tl_err;
    }
    if (hip_error) *hip_error = e.hip;
    if (msg && cap) {
        strncpy(msg, e.msg, cap - 1);
        msg[cap - 1] = 0;
    }
    return 0;
}

int jfsx_device_count(int *n) {
    if (!n) return JFSX_EINVAL;
    if (hipGetDeviceCount(n) != hipSuccess) {
        *n = 0;
        return JFSX_ENODEV;
    }
    return 0;
}

int jfsx_ctx_open(int device, uint32_t flags, jfsx_ctx **out) {
    if (!out || (flags & ~JFSX_CTX_BITSLICE)) return JFSX_EINVAL;
    *out = nullptr;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return JFSX_ENODEV;
    HIP_OK(hipSetDevice(device));
    jfsx_ctx *c = new jfsx_ctx();
    c->device = device;
    c->bitslice = (flags & JFSX_CTX_BITSLICE) != 0;
    (void)jfsx_device_numa_node(device, &c->numa_node);
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
        c->ncu = ncu;
    {
        // the block-parallel zstd decoder's arenas (kZstdArena per wave) may
        // take at most an eighth of the device's memory (JFSX_ZSTD_ARENA_MB
        // overrides): 8 waves per CU on a 256-CU, 288 GB part fit (28 GiB)
        size_t total = 0;
        (void)hipDeviceTotalMem(&total, device);
        c->zstd_arena_budget = total ? total / 8 : (size_t)4 << 30;
        if (const char *e = getenv("JFSX_ZSTD_ARENA_MB")) c->zstd_arena_budget = (size_t)atoll(e) << 20;
    }
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->s_ks, hipStreamNonBlocking) != hipSuccess) {
        jfsx_ctx_close(c);
        return JFSX_EIO;
    }
    std::vector<uint32_t> aes, crc, crcx;
    make_aes_table(aes);
    make_crc_tables(crc, crcx);
    const size_t nbytes = 4 * (aes.size() + crc.size() + crcx.size());
    if (hipMalloc((void **)&c->d_tab, nbytes) != hipSuccess) {
        c->d_tab = nullptr;
        jfsx_ctx_close(c);  // the streams made above
        return JFSX_ENOMEM;
    }
    std::vector<uint32_t> all;
    all.insert(all.end(), aes.begin(), aes.end());
    all.insert(all.end(), crc.begin(), crc.end());
    all.insert(all.end(), crcx.begin(), crcx.end());
    if (hipMemcpy(c->d_tab, all.data(), nbytes, hipMemcpyHostToDevice) != hipSuccess) {
        jfsx_ctx_close(c);
        return JFSX_EIO;
    }
    c->tabs.aes = c->d_tab;
    c->tabs.crc = c->d_tab + aes.size();
    c->tabs.crcx = c->d_tab + aes.size() + crc.size();
    for (int k = 0; k < kRing; k++) {
        if (hipEventCreate(&c->ev_k0[k]) != hipSuccess || hipEventCreate(&c->ev_k1[k]) != hipSuccess) {
            jfsx_ctx_close(c);
            return JFSX_EIO;
        }
    }
    for (PipeSlot &p : c->pipe) {
        if (hipEventCreateWithFlags(&p.ev_in, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&p.ev_comp, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&p.ev_out, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&p.ev_ks, hipEventDisableTiming) != hipSuccess ||
            hipEventCreate(&p.ev_k0) != hipSuccess || hipEventCreate(&p.ev_k1) != hipSuccess) {
            jfsx_ctx_close(c);
            return JFSX_EIO;
        }
    }
    *out = c;
    return 0;
}

int jfsx_ctx_close(jfsx_ctx *c) {
    if (!c) return JFSX_EINVAL;
    if (getenv("JFSX_PIPE_STATS") && c->ps_groups)
        fprintf(stderr, "jfsx pipe stats (device %d): %llu groups, %llu blocks, %llu H2D / %llu D2H data copies, "
                "enqueue %.1f us/group, slot wait %.1f us/group, own wait %.1f us/group\n", c->device,
                (unsigned long long)c->ps_groups.load(), (unsigned long long)c->ps_blocks.load(),
                (unsigned long long)c->ps_h2d.load(), (unsigned long long)c->ps_d2h.load(),
                c->ps_enq_us.load() / (double)c->ps_groups, c->ps_slot_us.load() / (double)c->ps_groups,
                c->ps_own_us.load() / (double)c->ps_groups);
    if (getenv("JFSX_PIPE_STATS") && c->ps_groups)
        fprintf(stderr, "jfsx pipe stats (device %d): per group: host-memory checks %.1f us, bounce in %.1f us, "
                "bounce out %.1f us, own-group wait %.1f us; bounce: %llu allocations, %.1f MB in, %.1f MB out\n",
                c->device, c->ps_pin_us.load() / (double)c->ps_groups, c->ps_bin_us.load() / (double)c->ps_groups,
                c->ps_bout_us.load() / (double)c->ps_groups, c->ps_wait_us.load() / (double)c->ps_groups,
                (unsigned long long)c->bounce.allocs.load(), c->bounce.bytes_in.load() / 1e6,
                c->bounce.bytes_out.load() / 1e6);
    async_detach(c);  // queued _async batches run first (jfsx_agg.cpp)
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    if (c->d_tab) (void)hipFree(c->d_tab);
    if (c->rsa_d) (void)hipFree(c->rsa_d);
    if (c->rsa_h) (void)hipHostFree(c->rsa_h);
    for (auto &kv : c->bounce.idle) {
        forget_pinned(kv.second);
        (void)hipHostFree(kv.second);
    }
    c->bounce.idle.clear();
    for (int k = 0; k < kRing; k++) {
        Workspace &w = c->ws[k];
        if (w.d) (void)hipFree(w.d);
        if (w.stage) (void)hipFree(w.stage);
        if (w.h) (void)hipHostFree(w.h);
        hipEvent_t evs[2] = {c->ev_k0[k], c->ev_k1[k]};
        for (hipEvent_t e : evs)
            if (e) (void)hipEventDestroy(e);
    }
    for (PipeSlot &p : c->pipe) {
        if (p.w.d) (void)hipFree(p.w.d);
        if (p.w.stage) (void)hipFree(p.w.stage);
        if (p.w.h) (void)hipHostFree(p.w.h);
        hipEvent_t evs[6] = {p.ev_in, p.ev_comp, p.ev_out, p.ev_k0, p.ev_k1, p.ev_ks};
        for (hipEvent_t e : evs)
            if (e) (void)hipEventDestroy(e);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->s_in) (void)hipStreamDestroy(c->s_in);
    if (c->s_ks) (void)hipStreamDestroy(c->s_ks);
    if (c->s_out) (void)hipStreamDestroy(c->s_out);
    delete c;
    return 0;
}

int jfsx_ctx_sync(jfsx_ctx *c) {
    if (!c) return JFSX_EINVAL;
    CtxScope es_(c);
    HIP_OK(hipStreamSynchronize(c->stream));
    HIP_OK(hipStreamSynchronize(c->s_in));
    HIP_OK(hipStreamSynchronize(c->s_out));
    return 0;
}

int jfsx_ctx_set_slot_bytes(jfsx_ctx *c, uint64_t bytes) {
    if (!c || bytes < (1u << 20)) return JFSX_EINVAL;
    c->slot_bytes = (size_t)bytes;
    return 0;
}

void *jfsx_ctx_stream(jfsx_ctx *c) { return c ? (void *)c->stream : nullptr; }

int jfsx_ctx_set_timing(jfsx_ctx *c, int enable) {
    if (!c) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    c->timing = enable != 0;
    return 0;
}

int jfsx_ctx_kernel_time(jfsx_ctx *c, double *ms_total, uint64_t *launches, int reset) {
    if (!c) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->stat_mu);
    if (ms_total) *ms_total = c->ms_total;
    if (launches) *launches = c->launches;
    if (reset) {
        c->ms_total = 0;
        c->launches = 0;
    }
    return 0;
}

int jfsx_pcie_probe(jfsx_ctx *c, uint64_t bytes, double out[4]) {
    if (!c || !out || bytes < 8 * 4096) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    const int chunks = 8;
    const size_t ch = (bytes / chunks) & ~(size_t)4095, tot = ch * chunks;
    char *hA = nullptr, *hB = nullptr, *dA = nullptr, *dB = nullptr;
    int rc = 0;
    auto fail = [&](hipError_t e, int line, const char *what) {
        note_hip_error(e, __FILE__, line, what);
        rc = JFSX_EIO;
    };
    hipError_t e;
    // host buffers exactly as jfsx_alloc_pinned makes the ring's staging
    if ((e = hipHostMalloc((void **)&hA, tot, hipHostMallocPortable)) != hipSuccess ||
        (e = hipHostMalloc((void **)&hB, tot, hipHostMallocPortable)) != hipSuccess ||
        (e = hipMalloc((void **)&dA, tot)) != hipSuccess || (e = hipMalloc((void **)&dB, tot)) != hipSuccess) {
        fail(e, __LINE__, "pcie probe buffers");
    } else {
        memset(hA, 1, tot);
        memset(hB, 2, tot);
        hipEvent_t ea, eb;
        (void)hipEventCreate(&ea);
        (void)hipEventCreate(&eb);
        for (int mode = 0; mode < 3 && !rc; mode++) {  // 0 H2D, 1 D2H, 2 both
            float best_a = 1e30f, best_b = 1e30f;
            for (int it = 0; it < 4 && !rc; it++) {
                // the ring's own two streams only: other contexts' work on the
                // device is not waited for (a diagnostic for an idle context)
                if ((e = hipStreamSynchronize(c->s_in)) != hipSuccess || (e = hipStreamSynchronize(c->s_out)) != hipSuccess) {
                    fail(e, __LINE__, "pcie probe sync");
                    break;
                }
                const auto t0 = std::chrono::steady_clock::now();
                for (int k = 0; k < chunks; k++) {
                    if (mode != 1) (void)hipMemcpyAsync(dA + k * ch, hA + k * ch, ch, hipMemcpyHostToDevice, c->s_in);
                    if (mode != 0) (void)hipMemcpyAsync(hB + k * ch, dB + k * ch, ch, hipMemcpyDeviceToHost, c->s_out);
                }
                if (mode != 1) (void)hipEventRecord(ea, c->s_in);
                if (mode != 0) (void)hipEventRecord(eb, c->s_out);
                if (mode != 1) (void)hipEventSynchronize(ea);
                const float ta = std::chrono::duration<float>(std::chrono::steady_clock::now() - t0).count();
                if (mode != 0) (void)hipEventSynchronize(eb);
                const float tb = std::chrono::duration<float>(std::chrono::steady_clock::now() - t0).count();
                if ((e = hipGetLastError()) != hipSuccess) { fail(e, __LINE__, "pcie probe copies"); break; }
                if (it == 0) continue;  // warm-up
                if (ta < best_a) best_a = ta;
                if (tb < best_b) best_b = tb;
            }
            if (mode == 0) out[0] = tot / (double)best_a / 1e9;
            if (mode == 1) out[1] = tot / (double)best_b / 1e9;
            if (mode == 2) {
                out[2] = tot / (double)best_a / 1e9;
                out[3] = tot / (double)best_b / 1e9;
            }
        }
        (void)hipEventDestroy(ea);
        (void)hipEventDestroy(eb);
    }
    if (hA) (void)hipHostFree(hA);
    if (hB) (void)hipHostFree(hB);
    if (dA) (void)hipFree(dA);
    if (dB) (void)hipFree(dB);
    return rc;
}

int jfsx_ctx_metrics(jfsx_ctx *c, jfsx_metrics *out, int reset) {
    if (!c || !out) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->stat_mu);
    *out = c->met;
    out->kernel_ms = c->ms_total;
    out->kernel_launches = c->launches;
    if (reset) {
        c->met = jfsx_metrics{};
        c->ms_total = 0;
        c->launches = 0;
    }
    return 0;
}

int jfsx_alloc_pinned(jfsx_ctx *c, size_t bytes, void **p) {
    if (!c || !p) return JFSX_EINVAL;
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    // portable: the multi-device context's other GPUs DMA from it as well
    const hipError_t e = hipHostMalloc(p, bytes, hipHostMallocPortable);
    if (e == hipSuccess) {
        note_pinned(*p, bytes);
        return 0;
    }
    note_hip_error(e, __FILE__, __LINE__, "hipHostMalloc(pinned)");
    return JFSX_ENOMEM;
}
int jfsx_device_numa_node(int device, int *node) {
    if (!node) return JFSX_EINVAL;
    *node = -1;
    int nd = 0;
    if (hipGetDeviceCount(&nd) != hipSuccess || device < 0 || device >= nd) return JFSX_ENODEV;
    int v = -1;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeHostNumaId, device) == hipSuccess && v >= 0) {
        *node = v;
        return 0;
    }
    (void)hipGetLastError();
    // the PCI function's node, as the kernel reports it
    char bus[64] = {0}, path[160];
    if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return 0;
    for (char *q = bus; *q; q++) *q = (char)tolower(*q);
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
    if (FILE *f = fopen(path, "r")) {
        if (fscanf(f, "%d", &v) == 1 && v >= 0) *node = v;
        fclose(f);
    }
    return 0;
}

namespace {
// set_mempolicy / get_mempolicy (numaif.h modes), called directly so the
// library needs no libnuma
constexpr int kMpolDefault = 0, kMpolBind = 2, kMpolFNode = 1, kMpolFAddr = 2;
constexpr unsigned long kMaxNodes = 1024;
}  // namespace

namespace {
// pinned portable host memory whose pages are bound to `node` (-1: default
// placement).  Binds this thread's allocations to the node while the runtime
// allocates and pins the pages (hipHostMallocNumaUser: they follow the
// caller's policy), then restores the thread's own policy.  Where the node
// cannot be bound (a cpuset without it), the default placement is used.
int alloc_pinned_on(int node, size_t bytes, void **p) {
    unsigned long old_mask[kMaxNodes / 64] = {0}, mask[kMaxNodes / 64] = {0};
    int old_mode = kMpolDefault;
    bool bound = false;
    if (node >= 0 && node < (int)kMaxNodes && syscall(SYS_get_mempolicy, &old_mode, old_mask, kMaxNodes, nullptr, 0) == 0) {
        mask[node / 64] = 1ul << (node % 64);
        bound = syscall(SYS_set_mempolicy, kMpolBind, mask, kMaxNodes) == 0;
    }
    const hipError_t e = hipHostMalloc(p, bytes, hipHostMallocPortable | (bound ? hipHostMallocNumaUser : 0));
    if (bound) (void)syscall(SYS_set_mempolicy, old_mode, old_mode == kMpolDefault ? nullptr : old_mask, kMaxNodes);
    if (e == hipSuccess) return 0;
    note_hip_error(e, __FILE__, __LINE__, "hipHostMalloc(pinned, NUMA node)");
    return JFSX_ENOMEM;
}
}  // namespace

int jfsx_alloc_pinned_node(jfsx_ctx *c, size_t bytes, int node, void **p) {
    if (!c || !p || node < -1 || node >= (int)kMaxNodes) return JFSX_EINVAL;
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    if (node < 0 && jfsx_device_numa_node(c->device, &node)) node = -1;
    const int rc = alloc_pinned_on(node, bytes, p);
    if (rc == 0) note_pinned(*p, bytes);
    return rc;
}

int jfsx_host_numa_node(const void *p, size_t bytes, int *node) {
    if (!p || !node) return JFSX_EINVAL;
    *node = -1;
    const size_t page = 4096, step = (size_t)64 << 20;
    for (size_t o = 0; o < std::max<size_t>(bytes, 1); o += step) {
        int nd = -1;
        void *a = (void *)(((uintptr_t)p + o) & ~(uintptr_t)(page - 1));
        if (syscall(SYS_get_mempolicy, &nd, nullptr, 0, a, kMpolFNode | kMpolFAddr) != 0) return 0;
        if (*node == -1) *node = nd;
        else if (*node != nd) {
            *node = -2;
            return 0;
        }
    }
    return 0;
}

int jfsx_free_pinned(jfsx_ctx *c, void *p) {
    if (!c) return JFSX_EINVAL;
    forget_pinned(p);
    HIP_OK(hipHostFree(p));
    return 0;
}
int jfsx_alloc_device(jfsx_ctx *c, size_t bytes, void **p) {
    if (!c || !p) return JFSX_EINVAL;
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    const hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) {
        note_alloc(*p, bytes, c->device);
        return 0;
    }
    note_hip_error(e, __FILE__, __LINE__, "hipMalloc(device buffer)");
    return JFSX_ENOMEM;
}
int jfsx_free_device(jfsx_ctx *c, void *p) {
    if (!c) return JFSX_EINVAL;
    forget_alloc(p);
    HIP_OK(hipFree(p));
    return 0;
}
int jfsx_memcpy_h2d(jfsx_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!c) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}
int jfsx_memcpy_d2h(jfsx_ctx *c, void *dst, const void *src, size_t bytes) {
    if (!c) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    return 0;
}

namespace {
// host batches lock per group inside the pipeline (the call waits unlocked);
// device batches hold the context for the whole call
int aead_entry(jfsx_ctx *c, int algo, bool open, int n, jfsx_blk *blks, int crc_mode, int mem) {
    if (!c || (n > 0 && !blks)) return JFSX_EINVAL;
    if (mem != JFSX_MEM_HOST && mem != JFSX_MEM_DEVICE) return JFSX_EINVAL;
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    int rc;
    if (mem == JFSX_MEM_HOST) {
        rc = run_aead_host(c, algo, open, n, blks, crc_mode);
    } else {
        std::lock_guard<std::mutex> g(c->mu);
        rc = run_aead(c, algo, open, n, blks, crc_mode);
    }
    if (rc == 0) tally_aead(c, open, n, blks);
    return rc;
}
}  // namespace

int jfsx_seal_batch(jfsx_ctx *c, int algo, int n, jfsx_blk *blks, int crc_mode, int mem) {
    return aead_entry(c, algo, false, n, blks, crc_mode, mem);
}

int jfsx_open_batch(jfsx_ctx *c, int algo, int n, jfsx_blk *blks, int crc_mode, int mem) {
    return aead_entry(c, algo, true, n, blks, crc_mode, mem);
}

int jfsx_crc32c_segments(jfsx_ctx *c, int n, jfsx_range *ranges, int mode, int mem) {
    if (!c || (n > 0 && !ranges)) return JFSX_EINVAL;
    if (mem != JFSX_MEM_HOST && mem != JFSX_MEM_DEVICE) return JFSX_EINVAL;
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    int rc;
    if (mem == JFSX_MEM_HOST) {
        rc = run_crc_host(c, n, ranges, mode);  // the host pipeline locks per group
    } else {
        std::lock_guard<std::mutex> g(c->mu);
        rc = run_crc(c, n, ranges, mode);
    }
    if (rc == 0) tally_crc(c, n, ranges);
    return rc;
}

uint64_t jfsx_lz4_bound(uint64_t n) { return lz4_bound(n); }

int jfsx_lz4_compress_batch(jfsx_ctx *c, int n, jfsx_zblk *blks, int mem) {
    if (!c || (n > 0 && !blks)) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    const int rc = run_codec(c, n, blks, mem, kLz4Comp);
    if (rc == 0) tally_codec(c, c->met.lz4c_blocks, c->met.lz4c_in, c->met.lz4c_out, nullptr, n, blks);
    return rc;
}

int jfsx_lz4_decompress_batch(jfsx_ctx *c, int n, jfsx_zblk *blks, int mem) {
    if (!c || (n > 0 && !blks)) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    const int rc = run_codec(c, n, blks, mem, kLz4Decomp);
    if (rc == 0) tally_codec(c, c->met.lz4d_blocks, c->met.lz4d_in, c->met.lz4d_out, &c->met.lz4d_fail, n, blks);
    return rc;
}

int jfsx_zstd_decompress_batch(jfsx_ctx *c, int n, jfsx_zblk *blks, int mem) {
    if (!c || (n > 0 && !blks)) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    const int rc = run_codec(c, n, blks, mem, kZstdDecomp);
    if (rc == 0) tally_codec(c, c->met.zstdd_blocks, c->met.zstdd_in, c->met.zstdd_out, &c->met.zstdd_fail, n, blks);
    return rc;
}

uint64_t jfsx_zstd_bound(uint64_t n) { return zstd_bound(n); }

int jfsx_zstd_compress_batch(jfsx_ctx *c, int n, jfsx_zblk *blks, int mem) {
    if (!c || (n > 0 && !blks)) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    const int rc = run_codec(c, n, blks, mem, kZstdComp);
    if (rc == 0) tally_codec(c, c->met.zstdc_blocks, c->met.zstdc_in, c->met.zstdc_out, nullptr, n, blks);
    return rc;
}

int jfsx_checksum(jfsx_ctx *c, const void *data, uint64_t len, uint8_t *out) {
    if (!c || !out || (len && !data)) return JFSX_EINVAL;
    jfsx_range r;
    memset(&r, 0, sizeof(r));
    r.data = data;
    r.len = len;
    r.crc = out;
    if (len == 0) {
        memset(out, 0, 4);  // disk_cache.go:1221: (0-1)/csBlock+1 = 1 entry, loop body never runs
        return 0;
    }
    return jfsx_crc32c_segments(c, 1, &r, JFSX_CRC_GEN, JFSX_MEM_HOST);
}

int jfsx_cache_verify(jfsx_ctx *c, const void *file, uint64_t file_size, uint64_t length, int level, uint64_t off,
                      uint64_t size, void *out, uint64_t *n_out, uint32_t *got, uint32_t *expect,
                      int64_t *bad_seg) {
    // cacheFile.ReadAt, disk_cache.go:1255-1329 -- range logic on the host,
    // the CRC work on the GPU.
    if (!c || !file || !n_out || level < 0 || level > 3) return JFSX_EINVAL;
    const uint8_t *f = (const uint8_t *)file;
    *n_out = 0;
    *bad_seg = -1;
    auto pread = [&](uint8_t *dst, uint64_t sz, uint64_t o, bool *eof) -> uint64_t {
        uint64_t nn = 0;
        *eof = false;
        if (o < file_size) {
            nn = std::min(sz, file_size - o);
            if (nn) memcpy(dst, f + o, nn);
        }
        if (nn < sz) *eof = true;
        return nn;
    };
    bool eof = false;
    if (level == 0 || (level == 1 && (off != 0 || size != length))) {
        *n_out = pread((uint8_t *)out, size, off, &eof);
        return eof ? JFSX_EOF : 0;
    }
    std::vector<uint8_t> tmp;
    uint8_t *rb = (uint8_t *)out;
    uint64_t rbsize = size, roff = off;
    if (level == 3) {
        roff = off / kSeg * kSeg;
        uint64_t rend = off + size;
        if (rend % kSeg != 0) {
            rend = (rend / kSeg + 1) * kSeg;
            if (rend > length) rend = length;
        }
        if (rend - roff != size) {
            rbsize = rend - roff;
            tmp.resize(std::max<uint64_t>(rbsize, 1));
            rb = tmp.data();
        }
    }
    const uint64_t nread = pread(rb, rbsize, roff, &eof);
    int rc = 0;
    if (eof) {
        rc = JFSX_EOF;
    } else {
        uint64_t ioff = roff / kSeg, cstart = 0, clen = rbsize;
        bool check = true;
        if (level == 2) {
            if (roff % kSeg != 0) {
                const uint64_t o = kSeg - roff % kSeg;
                if (clen <= o) check = false;
                else {
                    cstart += o;
                    clen -= o;
                    ioff += 1;
                }
            }
            const uint64_t end = roff + nread;
            if (check && end != length && end % kSeg != 0) {
                if (clen <= end % kSeg) check = false;
                else clen -= end % kSeg;
            }
        }
        if (check) {
            const uint64_t nexp = clen ? (clen - 1) / kSeg + 1 : 1;
            std::vector<uint8_t> ebuf(4 * nexp);
            bool eof2 = false;
            pread(ebuf.data(), 4 * nexp, length + ioff * 4, &eof2);
            if (eof2) {
                rc = JFSX_EOF;
            } else if (clen) {
                // the window goes to the host pipeline as it is: a pageable
                // window (the caller's buffer, or the widened read of the
                // extend level) is bounced by this thread, a pinned one
                // streams directly; concurrent readers share the pipeline
                int e;
                jfsx_range r;
                memset(&r, 0, sizeof(r));
                r.data = rb + cstart;
                r.len = clen;
                r.crc = ebuf.data();
                e = jfsx_crc32c_segments(c, 1, &r, JFSX_CRC_VERIFY, JFSX_MEM_HOST);
                if (e) return e;
                if (r.status == JFSX_ECRC) {
                    rc = JFSX_ECRC;
                    if (got) *got = r.got;
                    if (expect) *expect = r.expect;
                    *bad_seg = (int64_t)ioff + r.bad_seg;
                }
            }
        }
    }
    if (!tmp.empty() || (level == 3 && rb != (uint8_t *)out)) {
        if (rc == 0) {
            const uint64_t avail = rbsize - (off - roff);
            const uint64_t cpy = std::min(avail, size);
            if (cpy) memcpy(out, rb + (off - roff), cpy);
            *n_out = cpy;
        } else {
            *n_out = 0;
        }
    } else {
        *n_out = nread;
    }
    return rc;
}

int jfsx_parse_header(const void *obj, uint64_t olen, int *klen, int *nlen) {
    const uint8_t *o = (const uint8_t *)obj;
    if (!o || olen < 3) return JFSX_EMISFORMED;
    const int kl = ((int)o[0] << 8) + o[1], nl = o[2];
    if (klen) *klen = kl;
    if (nlen) *nlen = nl;
    if ((uint64_t)(3 + kl + nl) >= olen) return JFSX_EMISFORMED;  // encrypt.go:199-201
    return 0;
}

// ---------------------------------------------------------------------------
// host CRC32C helpers for the object checksum (pkg/object/checksum.go)
// ---------------------------------------------------------------------------
namespace {
const uint32_t *crc_table1() {
    static uint32_t t[256];
    static std::once_flag once;
    std::call_once(once, [] {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t v = i;
            for (int k = 0; k < 8; k++) v = v & 1 ? (v >> 1) ^ kCrcPoly : v >> 1;
            t[i] = v;
        }
    });
    return t;
}
uint32_t h_xpow8(uint64_t n) {  // x^(8n) mod P
    uint32_t r = 1u << 31, p = 1u << 23;
    for (; n; n >>= 1) {
        if (n & 1) r = crc_mulmod_h(p, r);
        p = crc_mulmod_h(p, p);
    }
    return r;
}
uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
}  // namespace

uint32_t jfsx_crc32c_update(uint32_t crc, const void *data, uint64_t n) {
    // hash/crc32.Update(crc, MakeTable(Castagnoli), p): pre/post-inverted
    const uint32_t *t = crc_table1();
    const uint8_t *p = (const uint8_t *)data;
    crc = ~crc;
    for (uint64_t i = 0; i < n; i++) crc = t[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
    return ~crc;
}

uint32_t jfsx_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return len_b ? crc_mulmod_h(h_xpow8(len_b), crc_a) ^ crc_b : crc_a;
}

int jfsx_object_crc32c(const void *hdr, uint64_t hlen, const uint8_t *seg_crcs, uint64_t clen, const uint8_t *tag,
                       uint32_t *out) {
    // generateChecksum(header || C || tag) (checksum.go:31-53) from the
    // engine's big-endian 32 KiB segment CRCs of C (crc_mode GEN|CT)
    if (!out || (hlen && !hdr) || (clen && !seg_crcs) || !tag) return JFSX_EINVAL;
    uint32_t crc = jfsx_crc32c_update(0, hdr, hlen);
    const uint64_t ns = clen ? (clen - 1) / kSeg + 1 : 0;
    for (uint64_t j = 0; j < ns; j++) {
        const uint64_t lj = std::min<uint64_t>(kSeg, clen - j * kSeg);
        crc = jfsx_crc32c_combine(crc, be32(seg_crcs + 4 * j), lj);
    }
    *out = jfsx_crc32c_update(crc, tag, 16);
    return 0;
}

}  // extern "C"

namespace {
// dataEncryptor.Encrypt / Decrypt around one Seal / Open, issued either as a
// one-block batch on a context or through the aggregator (jfsx_agg_data_*)
using AeadFn = std::function<int(jfsx_blk *, int crc_mode)>;

int data_encrypt(const AeadFn &seal, int algo, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *wrapped,
                 int wlen, const void *plaintext, uint64_t len, void *out, uint64_t out_cap, uint64_t *out_len,
                 uint32_t *obj_crc, uint8_t *seg_crc) {
    // encrypt.go:182-193: [BE16 klen][nlen][wrapped key][nonce][Seal(plaintext)]
    if (!key || !nonce || wlen < 0 || wlen > 65535 || (wlen && !wrapped) || !out) return JFSX_EINVAL;
    if (algo != JFSX_AES256GCM && algo != JFSX_CHACHA20P1305) return JFSX_EINVAL;
    const uint64_t hdr = 3 + (uint64_t)wlen + 12;
    if (out_cap < hdr + len + 16) return JFSX_EINVAL;
    uint8_t *o = (uint8_t *)out;
    o[0] = (uint8_t)(wlen >> 8);
    o[1] = (uint8_t)(wlen & 0xff);
    o[2] = 12;
    if (wlen) memcpy(o + 3, wrapped, wlen);
    memcpy(o + 3 + wlen, nonce, 12);
    jfsx_blk b;
    memset(&b, 0, sizeof(b));
    memcpy(b.key, key, 32);
    memcpy(b.nonce, nonce, 12);
    b.src = plaintext;
    b.dst = o + hdr;
    b.len = len;
    // the checksums the call asks for, in one pass: checksum() of the
    // plaintext (seg_crc, straight into the caller's array), the ciphertext
    // segment CRCs the object checksum is folded from (obj_crc), or both
    const uint64_t ns = nseg_of(len);
    std::vector<uint8_t> segs;
    int mode = JFSX_CRC_NONE;
    if (obj_crc && seg_crc) {
        segs.resize(8 * ns);
        b.crc = segs.data();
        mode = JFSX_CRC_GEN | JFSX_CRC_BOTH;
    } else if (obj_crc) {
        segs.resize(4 * ns);
        b.crc = segs.data();
        mode = JFSX_CRC_GEN | JFSX_CRC_CT;
    } else if (seg_crc) {
        b.crc = seg_crc;
        mode = JFSX_CRC_GEN;
    }
    int rc = seal(&b, mode);
    if (rc) return rc;
    memcpy(o + hdr + len, b.tag, 16);
    const uint8_t *ct_segs = obj_crc && seg_crc ? segs.data() + 4 * ns : segs.data();
    if (obj_crc && seg_crc) memcpy(seg_crc, segs.data(), 4 * ns);
    if (obj_crc && (rc = jfsx_object_crc32c(o, hdr, ct_segs, len, b.tag, obj_crc))) return rc;
    if (out_len) *out_len = hdr + len + 16;
    return 0;
}

int data_decrypt(const AeadFn &open, const uint8_t key[32], const void *obj, uint64_t olen, void *out,
                 uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc, uint32_t *got_crc,
                 uint8_t *seg_crc) {
    // encrypt.go:196-216; with expect_crc, the object checksum the store kept
    // (checksum.go:55-82) is verified in the same pass over C; with seg_crc,
    // checksum() of the plaintext for the cache file the load path writes next
    // (cached_store.go:745 -> disk_cache.go:469) comes out of the same pass
    if (!key || !obj || !out) return JFSX_EINVAL;
    int kl = 0, nl = 0;
    int rc = jfsx_parse_header(obj, olen, &kl, &nl);
    if (rc) return rc;
    const uint8_t *o = (const uint8_t *)obj;
    if (expect_crc && !got_crc) return JFSX_EINVAL;
    if (nl != 12) return JFSX_ETAG;  // aead.Open rejects a wrong nonce size (recovered as an error upstream)
    const uint64_t hdr = 3 + (uint64_t)kl + nl;
    if (olen - hdr < 16) return JFSX_ETAG;  // shorter than the tag: cipher: message authentication failed
    const uint64_t len = olen - hdr - 16;
    if (out_cap < len) return JFSX_EINVAL;
    jfsx_blk b;
    memset(&b, 0, sizeof(b));
    memcpy(b.key, key, 32);
    memcpy(b.nonce, o + 3 + kl, 12);
    b.src = o + hdr;
    b.dst = out;
    b.len = len;
    memcpy(b.tag, o + hdr + len, 16);
    const uint64_t ns = nseg_of(len);
    std::vector<uint8_t> segs;
    int mode = JFSX_CRC_NONE;
    if (expect_crc && seg_crc) {
        segs.resize(8 * ns);
        b.crc = segs.data();
        mode = JFSX_CRC_GEN | JFSX_CRC_BOTH;
    } else if (expect_crc) {
        segs.resize(4 * ns);
        b.crc = segs.data();
        mode = JFSX_CRC_GEN | JFSX_CRC_CT;
    } else if (seg_crc) {
        b.crc = seg_crc;
        mode = JFSX_CRC_GEN;
    }
    rc = open(&b, mode);
    if (rc) return rc;
    if (expect_crc) {
        // the store's read fails first ("verify checksum failed"), before Decrypt sees the bytes
        const uint8_t *ct_segs = seg_crc ? segs.data() + 4 * ns : segs.data();
        if ((rc = jfsx_object_crc32c(o, hdr, ct_segs, len, o + hdr + len, got_crc))) return rc;
        if (*got_crc != *expect_crc) {
            if (len) memset(out, 0, len);
            if (seg_crc) memset(seg_crc, 0, 4 * ns);
            return JFSX_ECRC;
        }
        if (seg_crc) memcpy(seg_crc, segs.data(), 4 * ns);  // zeros when the tag failed
    }
    if (b.status == JFSX_ETAG) return JFSX_ETAG;
    if (out_len) *out_len = len;
    return 0;
}
}  // namespace

extern "C" {

int jfsx_data_encrypt_ex(jfsx_ctx *c, int algo, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *wrapped,
                         int wlen, const void *plaintext, uint64_t len, void *out, uint64_t out_cap, uint64_t *out_len,
                         uint32_t *obj_crc, uint8_t *seg_crc) {
    if (!c) return JFSX_EINVAL;
    return data_encrypt([&](jfsx_blk *b, int m) { return jfsx_seal_batch(c, algo, 1, b, m, JFSX_MEM_HOST); }, algo,
                        key, nonce, wrapped, wlen, plaintext, len, out, out_cap, out_len, obj_crc, seg_crc);
}

int jfsx_data_decrypt_ex(jfsx_ctx *c, int algo, const uint8_t key[32], const void *obj, uint64_t olen, void *out,
                         uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc, uint32_t *got_crc,
                         uint8_t *seg_crc) {
    if (!c || (algo != JFSX_AES256GCM && algo != JFSX_CHACHA20P1305)) return JFSX_EINVAL;
    return data_decrypt([&](jfsx_blk *b, int m) { return jfsx_open_batch(c, algo, 1, b, m, JFSX_MEM_HOST); }, key,
                        obj, olen, out, out_cap, out_len, expect_crc, got_crc, seg_crc);
}

int jfsx_data_encrypt(jfsx_ctx *c, int algo, const uint8_t key[32], const uint8_t nonce[12], const uint8_t *wrapped,
                      int wlen, const void *plaintext, uint64_t len, void *out, uint64_t out_cap, uint64_t *out_len,
                      uint32_t *obj_crc) {
    return jfsx_data_encrypt_ex(c, algo, key, nonce, wrapped, wlen, plaintext, len, out, out_cap, out_len, obj_crc,
                                nullptr);
}

int jfsx_data_decrypt(jfsx_ctx *c, int algo, const uint8_t key[32], const void *obj, uint64_t olen, void *out,
                      uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc, uint32_t *got_crc) {
    return jfsx_data_decrypt_ex(c, algo, key, obj, olen, out, out_cap, out_len, expect_crc, got_crc, nullptr);
}

int jfsx_agg_data_encrypt_ex(jfsx_agg *a, int algo, const uint8_t key[32], const uint8_t nonce[12],
                             const uint8_t *wrapped, int wlen, const void *plaintext, uint64_t len, void *out,
                             uint64_t out_cap, uint64_t *out_len, uint32_t *obj_crc, uint8_t *seg_crc) {
    if (!a) return JFSX_EINVAL;
    return data_encrypt([&](jfsx_blk *b, int m) { return jfsx_agg_seal(a, algo, b, m, JFSX_MEM_HOST); }, algo, key,
                        nonce, wrapped, wlen, plaintext, len, out, out_cap, out_len, obj_crc, seg_crc);
}

int jfsx_agg_data_decrypt_ex(jfsx_agg *a, int algo, const uint8_t key[32], const void *obj, uint64_t olen, void *out,
                             uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc, uint32_t *got_crc,
                             uint8_t *seg_crc) {
    if (!a || (algo != JFSX_AES256GCM && algo != JFSX_CHACHA20P1305)) return JFSX_EINVAL;
    return data_decrypt([&](jfsx_blk *b, int m) { return jfsx_agg_open(a, algo, b, m, JFSX_MEM_HOST); }, key, obj,
                        olen, out, out_cap, out_len, expect_crc, got_crc, seg_crc);
}

int jfsx_agg_data_encrypt(jfsx_agg *a, int algo, const uint8_t key[32], const uint8_t nonce[12],
                          const uint8_t *wrapped, int wlen, const void *plaintext, uint64_t len, void *out,
                          uint64_t out_cap, uint64_t *out_len, uint32_t *obj_crc) {
    return jfsx_agg_data_encrypt_ex(a, algo, key, nonce, wrapped, wlen, plaintext, len, out, out_cap, out_len,
                                    obj_crc, nullptr);
}

int jfsx_agg_data_decrypt(jfsx_agg *a, int algo, const uint8_t key[32], const void *obj, uint64_t olen, void *out,
                          uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc, uint32_t *got_crc) {
    return jfsx_agg_data_decrypt_ex(a, algo, key, obj, olen, out, out_cap, out_len, expect_crc, got_crc, nullptr);
}

int jfsx_gen_synthetic(jfsx_ctx *c, void *dst, uint64_t len, uint64_t seed, uint64_t block) {
    if (!c || (len && !dst) || !aligned16(dst)) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    launch_begin();
    if (len) launch_gen_synthetic(c->stream, (uint8_t *)dst, len, seed, block);
    HIP_OK(hipGetLastError());
    return 0;
}

int jfsx_gen_synthetic_batch(jfsx_ctx *c, void *dst, uint64_t stride, int n, const uint64_t *lens, uint64_t seed,
                             uint64_t block0) {
    if (!c || n < 0 || (n && (!dst || !lens)) || !aligned16(dst) || (n > 1 && (stride & 15))) return JFSX_EINVAL;
    for (int i = 0; i < n; i++)
        if (lens[i] > stride && n > 1) return JFSX_EINVAL;
    if (n == 0) return 0;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    Workspace &w = c->ws[0];
    int rc;
    if ((rc = ensure_dev(c, &w.d, &w.dcap, 8 * (size_t)n))) return rc;
    if ((rc = ensure_host(&w.h, &w.hcap, 8 * (size_t)n))) return rc;
    memcpy(w.h, lens, 8 * (size_t)n);
    HIP_OK(hipMemcpyAsync(w.d, w.h, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    launch_begin();
    launch_gen_synthetic_batch(c->stream, (uint8_t *)dst, stride, n, (const uint64_t *)w.d, seed, block0);
    HIP_OK(hipGetLastError());
    HIP_OK(hipStreamSynchronize(c->stream));  // w.h/w.d are reused by the next batch
    return 0;
}

void jfsx_gen_key(uint64_t seed, uint64_t b, uint8_t key[32], uint8_t nonce[12]) {
    auto mix64 = [](uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    const uint64_t G = 0x9E3779B97F4A7C15ULL;
    for (int i = 0; i < 4; i++) {
        uint64_t w = mix64((seed ^ 0x4B4559ULL) + G * ((b << 8) + i + 1));
        memcpy(key + 8 * i, &w, 8);
    }
    uint64_t w0 = mix64((seed ^ 0x4E4F4E4345ULL) + G * ((b << 8) + 1));
    uint64_t w1 = mix64((seed ^ 0x4E4F4E4345ULL) + G * ((b << 8) + 2));
    memcpy(nonce, &w0, 8);
    memcpy(nonce + 8, &w1, 4);
}

int jfsx_debug_tables(uint32_t *aes, uint32_t *crc, uint32_t *crcx) {
    std::vector<uint32_t> a, c, x;
    make_aes_table(a);  // 16384 / 8192 / 192 dwords
    make_crc_tables(c, x);
    if (aes) memcpy(aes, a.data(), 4 * a.size());
    if (crc) memcpy(crc, c.data(), 4 * c.size());
    if (crcx) memcpy(crcx, x.data(), 4 * x.size());
    return 0;
}

// ---------------------------------------------------------------------------
// batched RSA-OAEP key unwrap (rsaEncryptor.Decrypt,
// pkg/object/encrypt.go:124-134 and :207-210)
// ---------------------------------------------------------------------------
struct jfsx_rsa_key {
    int device = 0;
    jfsx_rsa::Key *d_key = nullptr;
};

int jfsx_rsa_key_new(jfsx_ctx *c, const uint8_t *p, const uint8_t *q, const uint8_t *dp, const uint8_t *dq,
                     const uint8_t *qinv, int prime_bytes, const uint8_t *label, int label_len, jfsx_rsa_key **out) {
    if (!c || !out || !p || !q || !dp || !dq || !qinv || label_len < 0 || (label_len && !label)) return JFSX_EINVAL;
    *out = nullptr;
    if (prime_bytes != 4 * jfsx_rsa::kLimbs) return JFSX_EINVAL;  // RSA-2048 (1024-bit primes)
    jfsx_rsa::Key k;
    const uint8_t empty = 0;
    if (!jfsx_rsa::key_setup(k, p, q, dp, dq, qinv, label_len ? label : &empty, label_len)) return JFSX_EINVAL;
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    jfsx_rsa_key *rk = new jfsx_rsa_key();
    rk->device = c->device;
    if (hipMalloc((void **)&rk->d_key, sizeof(k)) != hipSuccess) {
        delete rk;
        return JFSX_ENOMEM;
    }
    if (hipMemcpy(rk->d_key, &k, sizeof(k), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(rk->d_key);
        delete rk;
        return JFSX_EIO;
    }
    *out = rk;
    return 0;
}

int jfsx_rsa_key_free(jfsx_rsa_key *k) {
    if (!k) return JFSX_EINVAL;
    (void)hipSetDevice(k->device);
    if (k->d_key) (void)hipFree(k->d_key);
    delete k;
    return 0;
}

int jfsx_rsa_oaep_decrypt_batch(jfsx_ctx *c, const jfsx_rsa_key *k, int n, const uint8_t *ct, uint64_t ct_stride,
                                const uint32_t *ct_len, uint8_t *msg, uint64_t msg_stride, int32_t *msg_len) {
    if (!c || !k || n < 0 || (n && (!ct || !ct_len || !msg_len || (msg_stride && !msg)))) return JFSX_EINVAL;
    if (n == 0) return 0;
    if (k->device != c->device) return JFSX_EINVAL;
    constexpr size_t K = jfsx_rsa::kModBytes;
    const size_t o_ct = 0, o_mh = align256(K * n), o_em = o_mh + align256(2 * 4 * jfsx_rsa::kLimbs * (size_t)n),
                 o_len = o_em + align256(K * n), dbytes = o_len + align256(4 * (size_t)n);
    const size_t hbytes = align256(K * n) + align256(4 * (size_t)n);
    std::lock_guard<std::mutex> g(c->mu);
    CtxScope es_(c);
    HIP_OK(hipSetDevice(c->device));
    int rc;
    if ((rc = ensure_dev(c, &c->rsa_d, &c->rsa_dcap, dbytes))) return rc;
    if ((rc = ensure_host(&c->rsa_h, &c->rsa_hcap, hbytes))) return rc;
    // Go's decrypt rejects a ciphertext longer than the modulus; shorter ones
    // are big-endian integers (left-padded here)
    for (int i = 0; i < n; i++) {
        uint8_t *d = (uint8_t *)c->rsa_h + K * i;
        const uint32_t l = ct_len[i] <= K ? ct_len[i] : 0;
        memset(d, 0, K - l);
        if (l) memcpy(d + K - l, ct + ct_stride * i, l);
    }
    char *d = c->rsa_d;
    HIP_OK(hipMemcpyAsync(d + o_ct, c->rsa_h, K * n, hipMemcpyHostToDevice, c->stream));
    launch_begin();
    launch_rsa_unwrap(c->stream, k->d_key, n, (const uint8_t *)(d + o_ct), (uint32_t *)(d + o_mh),
                      (uint8_t *)(d + o_em), (int32_t *)(d + o_len));
    HIP_OK(hipGetLastError());
    char *hl = c->rsa_h + align256(K * n);
    HIP_OK(hipMemcpyAsync(c->rsa_h, d + o_em, K * n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipMemcpyAsync(hl, d + o_len, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; i++) {
        int32_t l = ((const int32_t *)hl)[i];
        if (ct_len[i] > K) l = -1;
        msg_len[i] = l;
        if (l > 0 && msg_stride) memcpy(msg + msg_stride * i, c->rsa_h + K * i, std::min<uint64_t>(l, msg_stride));
    }
    return 0;
}

}  // extern "C"

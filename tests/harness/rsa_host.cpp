// CPU build of juicefs_amd/csrc/jfsx_rsa.h (test infrastructure only): the
// RSA-OAEP unwrap arithmetic, checked by tests/test_rsa.py against libcrypto.
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <thread>
// the sequence of Montgomery products and window-table reads, hashed
static uint64_t g_trace = 1469598103934665603ull, g_ops = 0;
#define JFSX_RSA_TRACE(tag, v) \
    (g_trace = (g_trace ^ ((uint64_t)(tag) << 8 ^ (uint64_t)(v))) * 1099511628211ull, g_ops++)
#define JFSX_HD static inline
#include "../../juicefs_amd/csrc/jfsx_rsa.h"

extern "C" {
// returns message length (copied to msg) or -1; -2 on a bad key
int rsa_unwrap(const uint8_t *p, const uint8_t *q, const uint8_t *dp, const uint8_t *dq, const uint8_t *qinv,
               const uint8_t *label, int label_len, const uint8_t *ct, uint8_t *msg) {
    static jfsx_rsa::Key k;
    if (!jfsx_rsa::key_setup(k, p, q, dp, dq, qinv, label, label_len)) return -2;
    uint8_t em[jfsx_rsa::kModBytes];
    const int n = jfsx_rsa::decrypt(k, ct, em);
    if (n > 0) memcpy(msg, em, n);
    return n;
}
void sha256(const uint8_t *a, int la, uint8_t *out) { jfsx_rsa::sha256_2(a, la, a, 0, out); }

// x^e mod m (128-byte big-endian operands, m an odd 1024-bit number) on the
// unwrap's exponentiation (mod_exp28, the one the GPU kernel runs); returns
// the operation-trace hash, *ops the count
uint64_t rsa_exp_trace(const uint8_t *m_be, const uint8_t *e_be, const uint8_t *x_be, uint8_t *out_be,
                       uint64_t *ops) {
    using namespace jfsx_rsa;
    uint32_t m[kLimbs], e[kLimbs], x[kLimbs], r2[kLimbs], r[kLimbs];
    from_be(m_be, 4 * kLimbs, m, kLimbs);
    from_be(e_be, 4 * kLimbs, e, kLimbs);
    from_be(x_be, 4 * kLimbs, x, kLimbs);
    mont_r2(m, r2, 2 * 28 * kL28);
    g_trace = 1469598103934665603ull;
    g_ops = 0;
    mod_exp28(x, e, m, mont_inv32(m[0]), r2, r);
    to_be(r, kLimbs, out_be, 4 * kLimbs);
    *ops = g_ops;
    return g_trace;
}

// mod_exp28_pair's lane exchange on the CPU: the two lanes are two threads
// that meet at a barrier for every exchanged word (SIMT lock step)
struct PairShared {
    std::atomic<uint32_t> gen{0};
    std::atomic<int> cnt{0};
    uint32_t slot[2];
};
struct PairThreads {
    uint32_t hi;
    PairShared *sh;
    bool tracing() const { return hi == 0; }
    void barrier() const {
        const uint32_t g = sh->gen.load(std::memory_order_acquire);
        if (sh->cnt.fetch_add(1, std::memory_order_acq_rel) == 1) {
            sh->cnt.store(0, std::memory_order_relaxed);
            sh->gen.store(g + 1, std::memory_order_release);
        } else {
            for (int k = 0; sh->gen.load(std::memory_order_acquire) == g; k++)
                if (k > 64) std::this_thread::yield();
        }
    }
    uint32_t xchg(uint32_t v, uint32_t from) const {
        sh->slot[hi] = v;
        barrier();
        const uint32_t r = sh->slot[from];
        barrier();
        return r;
    }
    uint32_t lo(uint32_t v) const { return xchg(v, 0); }
    uint32_t up(uint32_t v) const { return xchg(v, 1); }
    uint32_t other(uint32_t v) const { return xchg(v, hi ^ 1u); }
};

// rsa_exp_trace on mod_exp28_pair (the GPU kernel's two-lane form); *same =
// 1 when both lanes returned the same result
uint64_t rsa_exp_pair_trace(const uint8_t *m_be, const uint8_t *e_be, const uint8_t *x_be, uint8_t *out_be,
                            uint64_t *ops, int *same) {
    using namespace jfsx_rsa;
    uint32_t m[kLimbs], e[kLimbs], x[kLimbs], r2[kLimbs], r[2][kLimbs];
    from_be(m_be, 4 * kLimbs, m, kLimbs);
    from_be(e_be, 4 * kLimbs, e, kLimbs);
    from_be(x_be, 4 * kLimbs, x, kLimbs);
    mont_r2(m, r2, 2 * 28 * kL28);
    g_trace = 1469598103934665603ull;
    g_ops = 0;
    PairShared sh;
    auto lane = [&](uint32_t hi) { mod_exp28_pair(PairThreads{hi, &sh}, x, e, m, mont_inv32(m[0]), r2, r[hi]); };
    std::thread t1(lane, 1u);
    lane(0u);
    t1.join();
    *same = memcmp(r[0], r[1], sizeof(r[0])) == 0;
    to_be(r[0], kLimbs, out_be, 4 * kLimbs);
    *ops = g_ops;
    return g_trace;
}

// EME-OAEP decode of a 256-byte encoded message (label hash of `label`)
int oaep(uint8_t *em, const uint8_t *label, int label_len) {
    uint8_t lh[32];
    jfsx_rsa::sha256_2(label, label_len, label, 0, lh);
    return jfsx_rsa::oaep_decode(em, jfsx_rsa::kModBytes, lh);
}
}

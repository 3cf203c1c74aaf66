// CPU build of juicefs_amd/csrc/jfsx_rsa.h (test infrastructure only): the
// RSA-OAEP unwrap arithmetic, checked by tests/test_rsa.py against libcrypto.
#include <stdint.h>
#include <string.h>
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

// EME-OAEP decode of a 256-byte encoded message (label hash of `label`)
int oaep(uint8_t *em, const uint8_t *label, int label_len) {
    uint8_t lh[32];
    jfsx_rsa::sha256_2(label, label_len, label, 0, lh);
    return jfsx_rsa::oaep_decode(em, jfsx_rsa::kModBytes, lh);
}
}

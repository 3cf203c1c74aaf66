// CPU build of juicefs_amd/csrc/jfsx_rsa.h (test infrastructure only): the
// RSA-OAEP unwrap arithmetic, checked by tests/test_rsa.py against libcrypto.
#include <stdint.h>
#include <string.h>
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
}

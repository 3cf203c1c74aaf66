// CPU build of juicefs_amd/csrc/jfsx_aes_bs.h (test infrastructure only):
// BS3 / PERM emulate v_bitop3_b32 / v_perm_b32 so tests/test_aes_bs.py can pin
// the bitsliced AES-CTR decomposition against the oracle without a GPU.
#include <stdint.h>

static inline uint32_t bs3_emu(uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
    uint32_t r = 0;
    for (int i = 0; i < 8; i++)
        if ((tt >> i) & 1u) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
}
static inline uint32_t perm_emu(uint32_t hi, uint32_t lo, uint32_t sel) {
    const uint64_t pool = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int n = 0; n < 4; n++) r |= (uint32_t)((pool >> (8 * ((sel >> (8 * n)) & 7))) & 0xffu) << (8 * n);
    return r;
}
#define JFSX_HD static inline
#define BS3(a, b, c, tt) bs3_emu((a), (b), (c), (tt))
#define PERM(hi, lo, sel) perm_emu((hi), (lo), (sel))
#define OPAQUE(x) (void)(x)
#include "../../juicefs_amd/csrc/jfsx_aes_bs.h"

extern "C" {
// 32 keystream blocks E_K(nonce || BE32(c0 + 64k)), k = 0..31, as out[k][4] (LE dwords)
void bs_ctr32(const uint32_t rk[60], const uint32_t nonce[3], uint32_t c0, uint32_t out[128]) {
    uint32_t u[15][4];
    jfsx_bs::round_masks(rk, u);
    const uint32_t nrk[3] = {nonce[0] ^ rk[0], nonce[1] ^ rk[1], nonce[2] ^ rk[2]};
    uint32_t sbn[12], r1c[4];
    for (int i = 0; i < 12; i++) sbn[i] = jfsx_bs::sbox_byte((nrk[i >> 2] >> (8 * (i & 3))) & 0xffu);
    for (int c = 0; c < 4; c++) r1c[c] = jfsx_bs::round1_const(sbn, u[1], c);
    uint32_t st[128];
    jfsx_bs::ctr32(st, nrk, rk[3], c0, [&](int r, int w) { return u[r][w]; }, r1c);
    for (int k = 0; k < 32; k++)
        for (int w = 0; w < 4; w++) out[4 * k + w] = st[32 * w + k];
}
void bs_sbox_byte(uint32_t x, uint32_t mask, uint32_t *out) {
    uint32_t U[8], o[8];
    for (int j = 0; j < 8; j++) U[j] = (x >> (7 - j)) & 1u ? ~0u : 0u;
    uint32_t m[8];
    for (int j = 0; j < 8; j++) m[j] = ((mask ^ 0x63u) >> (7 - j)) & 1u ? ~0u : 0u;
    JFSX_SBOX_BS(U[0], U[1], U[2], U[3], U[4], U[5], U[6], U[7], m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7],
                 o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]);
    uint32_t y = 0;
    for (int j = 0; j < 8; j++) y |= (o[j] & 1u) << (7 - j);
    *out = y;
}
void bs_transpose32(uint32_t A[32]) { jfsx_bs::transpose32(A); }
}

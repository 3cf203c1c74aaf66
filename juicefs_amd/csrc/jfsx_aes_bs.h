// jfsx_aes_bs.h -- bitsliced AES-256-CTR keystream: 32 counter blocks per lane.
//
// The T-table AES of gcm_main is bound by LDS bandwidth (16 ds_read_b32 per
// block-round at 32 lanes/clk/CU).  Here the cipher runs on the VALU instead
// (128 lane-ops/clk/CU on gfx950): a lane holds the AES state of 32 counter
// blocks bitsliced over 128 VGPRs, st[8*i + b] = bit b of state byte i across
// the 32 blocks (bit k of the register = block slot k).  A round is 16 S-box
// circuits (jfsx_sbox_bs.h, 99 v_bitop3 each), ShiftRows as register renaming
// and a bitsliced MixColumns; AddRoundKey costs nothing: the round key is moved
// in front of MixColumns (u_r = SR^-1(MC^-1(rk_r))) and merged, with the S-box
// constant 0x63, into the S-box output XORs as wave-uniform 0/~0 masks.
//
// Counter layout (matches the row decomposition of gcm_main): lane slot k
// encrypts counter c0 + 64*k, so after the final 32x32 bit transposes
// st[32*w + k] is little-endian dword w of the keystream for row k of a
// 32 KiB segment (rows of 64 lanes x 16 B).
//
// The includer defines JFSX_HD (function qualifiers), BS3(a, b, c, tt) (a
// three-input bitwise op with truth table tt = f(0xF0, 0xCC, 0xAA)) and
// PERM(hi, lo, sel) (v_perm_b32 byte select) and OPAQUE(x) (an optimisation
// barrier on a wave-uniform value: keeps the per-round masks from being
// hoisted out of the segment loop into SGPRs that then spill).  gcm_main maps them to the gfx950
// builtins; the CPU harness of tests/test_aes_bs.py to a plain-C emulation.
#pragma once
#include <stdint.h>

#include "jfsx_sbox_bs.h"

namespace jfsx_bs {

// AES round key u_r -> S-box output masks for round r (FIPS-197 5.1).  Computed
// once per key by gcm_keysetup; consumed as 4 little-endian dwords per round.
JFSX_HD uint32_t gf_xt(uint32_t b) { return ((b << 1) ^ ((b & 0x80u) ? 0x1bu : 0u)) & 0xffu; }
JFSX_HD uint32_t gf_mul(uint32_t a, uint32_t b) {
    uint32_t r = 0;
    for (int i = 0; i < 8; i++) {
        if ((b >> i) & 1u) r ^= a;
        a = gf_xt(a);
    }
    return r;
}

// rk: 60 little-endian dwords of the FIPS-197 byte schedule (byte i of round
// key r = byte (i & 3) of rk[4r + i/4]).  Dword w of the S-box output mask of
// round r = 1..14:
//   r < 14:  u_r = SR^-1(MC^-1(rk_r)) ^ 0x63..63
//   r = 14:  u_r = SR^-1(rk_14) ^ 0x63..63
// (SR(y)[4c + row] = y[4((c + row) & 3) + row], so u[4c' + row] = v[4((c' - row) & 3) + row].)
JFSX_HD uint32_t round_mask_word(const uint32_t *rk, int r, int w) {
    uint32_t out = 0;
    for (int row = 0; row < 4; row++) {
        const int c = (w - row) & 3;  // source column of v
        uint32_t k[4];
        for (int q = 0; q < 4; q++) k[q] = (rk[4 * r + c] >> (8 * q)) & 0xffu;
        uint32_t v;
        if (r < 14)
            v = gf_mul(k[row], 14) ^ gf_mul(k[(row + 1) & 3], 11) ^ gf_mul(k[(row + 2) & 3], 13) ^
                gf_mul(k[(row + 3) & 3], 9);
        else
            v = k[row];
        out |= ((v ^ 0x63u) & 0xffu) << (8 * row);
    }
    return out;
}
JFSX_HD void round_masks(const uint32_t *rk, uint32_t (*u)[4]) {
    for (int r = 1; r <= 14; r++)
        for (int w = 0; w < 4; w++) u[r][w] = round_mask_word(rk, r, w);
}

// AES S-box of one byte (FIPS-197 5.1.1: inverse x^254, then the affine map)
JFSX_HD uint32_t sbox_byte(uint32_t x) {
    uint32_t y = x, r = 1;
    for (int e = 254; e; e >>= 1) {  // r = x^254
        if (e & 1) r = gf_mul(r, y);
        y = gf_mul(y, y);
    }
    uint32_t s = r;
    for (int i = 1; i < 5; i++) s ^= ((r << i) | (r >> (8 - i))) & 0xffu;
    return (s ^ 0x63u) & 0xffu;
}

// CTR round 1 with 12 wave-uniform state bytes (the nonce): after SubBytes and
// ShiftRows each column holds three uniform bytes and one counter byte (row
// 3 - c, from state byte 15 - c).  r1c[c] = MixColumns of column c with that
// byte zeroed (row r in byte r), i.e. the uniform part of round 1's output.
// sbn[i] = S(nonce_i ^ rk0_i) for i = 0..11 (sbox_byte); u1 = round_mask_word(rk, 1, *).
JFSX_HD uint32_t round1_const(const uint32_t *sbn, const uint32_t u1[4], int c) {
    uint32_t a[4];
    for (int r = 0; r < 4; r++) {
        const int i = 4 * ((c + r) & 3) + r;  // state byte under (r, c) after ShiftRows
        a[r] = i >= 12 ? 0u : (sbn[i] ^ ((u1[i >> 2] >> (8 * (i & 3))) & 0xffu) ^ 0x63u);
    }
    uint32_t out = 0;
    for (int r = 0; r < 4; r++)
        out |= (gf_mul(a[r], 2) ^ gf_mul(a[(r + 1) & 3], 3) ^ a[(r + 2) & 3] ^ a[(r + 3) & 3]) << (8 * r);
    return out;
}

// 0 / ~0 from bit n of a (wave-uniform in the kernel: one s_bfe_i32)
JFSX_HD uint32_t bmask(uint32_t a, int n) { return (uint32_t)((int32_t)(a << (31 - n)) >> 31); }

// SubBytes + masks on all 16 bytes, in place.  JFSX_SBOX_PAIR interleaves the
// gates of two S-boxes so a wave always has an independent op to issue.
#ifndef JFSX_SBOX_PAIR
#define JFSX_SBOX_PAIR 1
#endif
#define JFSX_BM(uw, sh) bmask(uw, sh + 7), bmask(uw, sh + 6), bmask(uw, sh + 5), bmask(uw, sh + 4), \
                        bmask(uw, sh + 3), bmask(uw, sh + 2), bmask(uw, sh + 1), bmask(uw, sh + 0)
#define JFSX_EXPAND(m, ...) m(__VA_ARGS__)  // expand JFSX_BM before the argument count
JFSX_HD void sub_bytes(uint32_t *st, const uint32_t u[4]) {
#if JFSX_SBOX_PAIR
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
        uint32_t *x = st + 8 * i, *y = st + 8 * (i + 1);
        const uint32_t ux = u[i >> 2], uy = u[(i + 1) >> 2];
        const int shx = 8 * (i & 3), shy = 8 * ((i + 1) & 3);
        uint32_t o0, o1, o2, o3, o4, o5, o6, o7, q0, q1, q2, q3, q4, q5, q6, q7;
        JFSX_EXPAND(JFSX_SBOX_BS2, x[7], x[6], x[5], x[4], x[3], x[2], x[1], x[0], JFSX_BM(ux, shx), o0, o1, o2, o3, o4, o5, o6, o7,
                      y[7], y[6], y[5], y[4], y[3], y[2], y[1], y[0], JFSX_BM(uy, shy), q0, q1, q2, q3, q4, q5, q6, q7);
        x[7] = o0; x[6] = o1; x[5] = o2; x[4] = o3; x[3] = o4; x[2] = o5; x[1] = o6; x[0] = o7;
        y[7] = q0; y[6] = q1; y[5] = q2; y[4] = q3; y[3] = q4; y[2] = q5; y[1] = q6; y[0] = q7;
    }
#else
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t uw = u[i >> 2];
        const int sh = 8 * (i & 3);
        uint32_t *x = st + 8 * i;
        uint32_t o0, o1, o2, o3, o4, o5, o6, o7;
        JFSX_EXPAND(JFSX_SBOX_BS, x[7], x[6], x[5], x[4], x[3], x[2], x[1], x[0], JFSX_BM(uw, sh), o0, o1, o2, o3, o4, o5, o6, o7);
        x[7] = o0; x[6] = o1; x[5] = o2; x[4] = o3; x[3] = o4; x[2] = o5; x[1] = o6; x[0] = o7;
    }
#endif
}

#define JFSX_X3(a, b, c) BS3((a), (b), (c), 0x96)
#define JFSX_X2(a, b) BS3((a), (b), 0u, 0x3c)

// MixColumns of one bitsliced column a[row][bit] into o[8*row + bit], 76 ops:
// y_r = a_r ^ a_r+1;  out_r = xtime(y_r) ^ a_r+1 ^ y_r+2
// (= 2a_r ^ 3a_r+1 ^ a_r+2 ^ a_r+3; xtime feeds bit 7 back into bits 0, 1, 3, 4)
template <class A>
JFSX_HD void mix_column(A a, uint32_t *o) {
    uint32_t y[4][8];
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int b = 0; b < 8; b++) y[r][b] = JFSX_X2(a[r][b], a[(r + 1) & 3][b]);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const uint32_t *x1 = a[(r + 1) & 3];
        const uint32_t *y0 = y[r], *y2 = y[(r + 2) & 3];
        uint32_t *q = o + 8 * r;
        q[0] = JFSX_X3(y0[7], x1[0], y2[0]);
        q[1] = JFSX_X3(JFSX_X3(y0[0], y0[7], x1[1]), y2[1], 0u);
        q[2] = JFSX_X3(y0[1], x1[2], y2[2]);
        q[3] = JFSX_X3(JFSX_X3(y0[2], y0[7], x1[3]), y2[3], 0u);
        q[4] = JFSX_X3(JFSX_X3(y0[3], y0[7], x1[4]), y2[4], 0u);
        q[5] = JFSX_X3(y0[4], x1[5], y2[5]);
        q[6] = JFSX_X3(y0[5], x1[6], y2[6]);
        q[7] = JFSX_X3(y0[6], x1[7], y2[7]);
    }
}

// ShiftRows (as renaming) + MixColumns: st <- MC(SR(st))
JFSX_HD void shift_mix(uint32_t *st) {
    uint32_t out[128];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        // a_r = byte (r, c) after ShiftRows = byte 4((c + r) & 3) + r before it
        const uint32_t *a[4];
#pragma unroll
        for (int r = 0; r < 4; r++) a[r] = st + 8 * (4 * ((c + r) & 3) + r);
        mix_column(a, out + 8 * (4 * c));
    }
#pragma unroll
    for (int i = 0; i < 128; i++) st[i] = out[i];
}

// final ShiftRows (renaming only)
JFSX_HD void shift_rows(uint32_t *st) {
    uint32_t out[128];
#pragma unroll
    for (int c = 0; c < 4; c++)
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int b = 0; b < 8; b++) out[8 * (4 * c + r) + b] = st[8 * (4 * ((c + r) & 3) + r) + b];
#pragma unroll
    for (int i = 0; i < 128; i++) st[i] = out[i];
}

// swap bits a[j + s] <-> b[j] for the j selected by m (32x32 transpose step)
template <int S>
JFSX_HD void tswap(uint32_t &a, uint32_t &b, uint32_t m) {
    uint32_t na, nb;
    if (S == 16) {
        nb = PERM(a, b, 0x03020706u);  // {a.b2, a.b3, b.b2, b.b3}
        na = PERM(a, b, 0x01000504u);  // {a.b0, a.b1, b.b0, b.b1}
    } else if (S == 8) {
        nb = PERM(a, b, 0x03070105u);  // {a.b1, b.b1, a.b3, b.b3}
        na = PERM(a, b, 0x02060004u);  // {a.b0, b.b0, a.b2, b.b2}
    } else {
        nb = BS3(a >> S, b, m, 0xe4);        // m ? (a >> S) : b
        na = BS3(b << S, a, m << S, 0xe4);   // (m << S) ? (b << S) : a
    }
    a = na;
    b = nb;
}

// in-place 32x32 bit transpose of A[0..31]: bit k of A[j] <-> bit j of A[k]
JFSX_HD void transpose32(uint32_t *A) {
#pragma unroll
    for (int k = 0; k < 32; k++)
        if (!(k & 16)) tswap<16>(A[k], A[k + 16], 0x0000ffffu);
#pragma unroll
    for (int k = 0; k < 32; k++)
        if (!(k & 8)) tswap<8>(A[k], A[k + 8], 0x00ff00ffu);
#pragma unroll
    for (int k = 0; k < 32; k++)
        if (!(k & 4)) tswap<4>(A[k], A[k + 4], 0x0f0f0f0fu);
#pragma unroll
    for (int k = 0; k < 32; k++)
        if (!(k & 2)) tswap<2>(A[k], A[k + 2], 0x33333333u);
#pragma unroll
    for (int k = 0; k < 32; k++)
        if (!(k & 1)) tswap<1>(A[k], A[k + 1], 0x55555555u);
}

// Round-0 state: counter blocks nonce || BE32(c0 + 64k), k = 0..31, xor rk_0.
// nrk[0..2] = nonce ^ rk[0..2] (wave-uniform), rk3 = rk[3], c0 = lane's counter.
JFSX_HD void load_counters(uint32_t *st, const uint32_t nrk_in[3], uint32_t rk3, uint32_t c0) {
    uint32_t nrk[3] = {nrk_in[0], nrk_in[1], nrk_in[2]};
    OPAQUE(nrk[0]);
    OPAQUE(nrk[1]);
    OPAQUE(nrk[2]);
    OPAQUE(rk3);
#pragma unroll
    for (int i = 0; i < 12; i++)
#pragma unroll
        for (int b = 0; b < 8; b++) st[8 * i + b] = bmask(nrk[i >> 2], 8 * (i & 3) + b);
    // counter bit n (of c0 + 64k) lives in byte 15 - n/8, bit n % 8; the key
    // byte over it is byte (15 - n/8) & 3 of rk3
    const uint32_t v = c0 >> 6;
    uint32_t carry = 0;
#pragma unroll
    for (int n = 0; n < 32; n++) {
        uint32_t bit;
        if (n < 6) {
            bit = bmask(c0, n);
        } else {
            const int q = n - 6;
            const uint32_t pk = q == 0 ? 0xAAAAAAAAu : q == 1 ? 0xCCCCCCCCu : q == 2 ? 0xF0F0F0F0u
                              : q == 3 ? 0xFF00FF00u : q == 4 ? 0xFFFF0000u : 0u;
            const uint32_t vb = bmask(v, q);
            bit = JFSX_X3(pk, vb, carry);
            carry = BS3(pk, vb, carry, 0xe8);  // majority
        }
        const int byte = 15 - n / 8;
        const uint32_t kb = bmask(rk3, 8 * (byte & 3) + (n & 7));
        st[8 * byte + (n & 7)] = JFSX_X2(bit, kb);
    }
}

// Full AES-256 of the 32 counter blocks; um(r, w) = dword w of round r's masks
// (round_mask_word), r1c = round1_const() of columns 0..3.
// On return st[32*w + k] = keystream dword w (little-endian) of slot k.
template <class UM>
JFSX_HD void ctr32(uint32_t *st, const uint32_t nrk[3], uint32_t rk3, uint32_t c0, UM um, const uint32_t r1c_in[4]) {
    load_counters(st, nrk, rk3, c0);
    {
        // round 1: S-boxes of the four counter bytes only; the nonce bytes'
        // contribution to MixColumns is the per-key constant r1c
        uint32_t u3 = um(1, 3), r1c[4] = {r1c_in[0], r1c_in[1], r1c_in[2], r1c_in[3]};
        OPAQUE(u3);
        for (int c = 0; c < 4; c++) OPAQUE(r1c[c]);
        uint32_t v[4][8];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t *x = st + 8 * (12 + q);
            const int sh = 8 * q;
            JFSX_EXPAND(JFSX_SBOX_BS, x[7], x[6], x[5], x[4], x[3], x[2], x[1], x[0], JFSX_BM(u3, sh), v[q][7], v[q][6],
                        v[q][5], v[q][4], v[q][3], v[q][2], v[q][1], v[q][0]);
        }
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const int r = 3 - c;
            const uint32_t *vv = v[3 - c];  // state byte 15 - c
            uint32_t x2[8], x3[8];
            x2[0] = vv[7];
            x2[1] = JFSX_X2(vv[0], vv[7]);
            x2[2] = vv[1];
            x2[3] = JFSX_X2(vv[2], vv[7]);
            x2[4] = JFSX_X2(vv[3], vv[7]);
            x2[5] = vv[4];
            x2[6] = vv[5];
            x2[7] = vv[6];
#pragma unroll
            for (int b = 0; b < 8; b++) x3[b] = JFSX_X2(x2[b], vv[b]);
#pragma unroll
            for (int row = 0; row < 4; row++) {
                const uint32_t *t = row == r ? x2 : row == ((r + 3) & 3) ? x3 : vv;
#pragma unroll
                for (int b = 0; b < 8; b++) st[8 * (4 * c + row) + b] = JFSX_X2(t[b], bmask(r1c[c], 8 * row + b));
            }
        }
    }
#pragma unroll 1
    for (int r = 2; r < 14; r++) {
        uint32_t u[4] = {um(r, 0), um(r, 1), um(r, 2), um(r, 3)};
        sub_bytes(st, u);
        shift_mix(st);
    }
    {
        uint32_t u[4] = {um(14, 0), um(14, 1), um(14, 2), um(14, 3)};
        for (int w = 0; w < 4; w++) OPAQUE(u[w]);
        sub_bytes(st, u);
        shift_rows(st);
    }
#pragma unroll
    for (int w = 0; w < 4; w++) transpose32(st + 32 * w);
}

}  // namespace jfsx_bs

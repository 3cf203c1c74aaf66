// jfsx_dev.h -- device helpers shared by the transform kernels (gfx950).
#pragma once
#include "jfsx_internal.h"

namespace jfsx {

__device__ __forceinline__ uint32_t lds_u32(const char *lds, uint32_t byteaddr) {
    return *reinterpret_cast<const uint32_t *>(lds + byteaddr);
}
__device__ __forceinline__ uint4 lds_u4(const char *lds, uint32_t byteaddr) {
    return *reinterpret_cast<const uint4 *>(lds + byteaddr);
}

// 4 * byte k of x in one VALU op: v_lshlrev_b32 with an SDWA byte select on the
// shifted operand.  With the table base below 64 KiB the base folds into the
// ds_read offset, so a table lookup costs one VALU op instead of two or three.
#if JFSX_CRCSDWA
template <int K>
__device__ __forceinline__ uint32_t byte_x4(uint32_t x) {
    uint32_t r;
    if constexpr (K == 0)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(x));
    else if constexpr (K == 1)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(x));
    else if constexpr (K == 2)
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(x));
    else
        asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(x));
    return r;
}
#ifdef JFSX_ABLATE_CRCBANK
// timing experiment only (wrong CRCs): every lookup keeps its SDWA address op
// plus one v_and_or_b32, but lands in the lane's own bank (conflict-free)
__device__ __forceinline__ uint32_t abl_bank(uint32_t a) {
    uint32_t r;
    asm volatile("v_and_or_b32 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"((threadIdx.x & 31u) << 2));
    return r;
}
#define CRC_T(t, x, k) lds_u32(lds, abl_bank(byte_x4<(k)>(x)) + CB + 1024u * (t))
#else
#define CRC_T(t, x, k) lds_u32(lds, byte_x4<(k)>(x) + CB + 1024u * (t))
#endif
#else
#define CRC_T(t, x, k) lds_u32(lds, ((((x) >> (8 * (k))) & 0xffu) << 2) + CB + 1024u * (t))
#endif

// crc_raw(A, 16-byte piece) = crc_raw(0, piece ^ shift(A, 1008 B) in the first word)
// S = 16: shift by 1008 B first; S = 20: shift by 4032 B; S < 0: no shift
template <uint32_t CB, int S = 16>
__device__ __forceinline__ uint32_t crc_piece(const char *lds, uint32_t A, uint32_t p0, uint32_t p1, uint32_t p2,
                                              uint32_t p3) {
#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
    uint32_t s = S < 0 ? A : X3(CRC_T(S, A, 0), CRC_T(S + 1, A, 1), CRC_T(S + 2, A, 2)) ^ CRC_T(S + 3, A, 3);
    uint32_t q = p0 ^ s;
    return X3(X3(X3(CRC_T(0, q, 0), CRC_T(1, q, 1), CRC_T(2, q, 2)), X3(CRC_T(3, q, 3), CRC_T(4, p1, 0), CRC_T(5, p1, 1)),
                 X3(CRC_T(6, p1, 2), CRC_T(7, p1, 3), CRC_T(8, p2, 0))),
              X3(CRC_T(9, p2, 1), CRC_T(10, p2, 2), CRC_T(11, p2, 3)),
              X3(CRC_T(12, p3, 0), CRC_T(13, p3, 1), X3(CRC_T(14, p3, 2), CRC_T(15, p3, 3), 0u)));
#undef X3
}

// byte-serial tail: crc_raw(shift(A,1008), first n bytes of the piece)
// CRCMODE bit 2 (JFSX_CRC_CT): the segment CRCs cover the ciphertext side
// (object checksum, pkg/object/checksum.go:31-53) instead of the plaintext
// (cache-file checksum, disk_cache.go:1218-1231).
template <int CRCMODE>
__device__ __forceinline__ uint4 crc_src(uint4 c, uint4 p) {
    return (CRCMODE & 4) ? c : p;
}

template <uint32_t CB, int S = 16>
__device__ __noinline__ uint32_t crc_partial(const char *lds, uint32_t A, const uint32_t p[4], int n) {
    uint32_t c = S < 0 ? A : CRC_T(S, A, 0) ^ CRC_T(S + 1, A, 1) ^ CRC_T(S + 2, A, 2) ^ CRC_T(S + 3, A, 3);
    for (int i = 0; i < n; i++) {
        uint32_t byte = (p[i >> 2] >> (8 * (i & 3))) & 0xffu;
        c = lds_u32(lds, (((c ^ byte) & 0xffu) << 2) + CB + 1024u * 15) ^ (c >> 8);
    }
    return c;
}

// 16-byte global load / store through an address_space(1) pointer: global_*
// instead of flat_* (flat ops count in both vmcnt and lgkmcnt, so every LDS
// wait would also wait for the outstanding HBM traffic).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4u gv4u;
__device__ __forceinline__ uint4 gld16(const uint8_t *p) {
    const v4u v = *(const gv4u *)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
// the same with the non-temporal hint (a streaming read nothing reuses)
__device__ __forceinline__ uint4 gld16_nt(const uint8_t *p) {
    const v4u v = __builtin_nontemporal_load((const gv4u *)(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gst16(uint8_t *p, uint4 v) {
    v4u w = {v.x, v.y, v.z, v.w};
    *(gv4u *)(p) = w;
}
__device__ __forceinline__ void gst16_nt(uint8_t *p, uint4 v) {
    v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, (gv4u *)(p));
}
// the AEAD kernels' block streams (plaintext in, ciphertext out): JFSX_AEAD_NT
// bit 1 gives the loads, bit 2 the stores the non-temporal hint (A/B)
#ifndef JFSX_AEAD_NT
#define JFSX_AEAD_NT 0
#endif
__device__ __forceinline__ uint4 ald16(const uint8_t *p) { return (JFSX_AEAD_NT & 1) ? gld16_nt(p) : gld16(p); }
__device__ __forceinline__ void ast16(uint8_t *p, uint4 v) {
    if (JFSX_AEAD_NT & 2)
        gst16_nt(p, v);
    else
        gst16(p, v);
}

// guarded 16-byte load of [o, o+16) clipped at end (zero fill)
__device__ __forceinline__ uint4 load_piece(const uint8_t *src, uint64_t o, uint64_t end) {
    if (o + 16 <= end) return gld16(src + o);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint64_t i = o; i < end && i < o + 16; i++) w[(i - o) >> 2] |= (uint32_t)src[i] << (8 * ((i - o) & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void store_piece(uint8_t *dst, uint64_t o, uint64_t end, uint4 v) {
    if (o + 16 <= end) {
        gst16(dst + o, v);
        return;
    }
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    for (uint64_t i = o; i < end && i < o + 16; i++) dst[i] = (uint8_t)(w[(i - o) >> 2] >> (8 * ((i - o) & 3)));
}


__device__ __forceinline__ void crc_verify_block(const BlkDev &blk, BlkOut &o, uint32_t lane) {
    // compare computed (native) vs expected (BE bytes); first failing segment
    const uint64_t nseg = (blk.len + kSeg - 1) / kSeg;
    for (uint64_t base = 0; base < nseg; base += 64) {
        const uint64_t s = base + lane;
        bool bad = false;
        uint32_t got = 0, ex = 0;
        if (s < nseg) {
            got = blk.crc_calc[s];
            const uint8_t *e = blk.crc + 4 * s;
            ex = ((uint32_t)e[0] << 24) | ((uint32_t)e[1] << 16) | ((uint32_t)e[2] << 8) | e[3];
            bad = got != ex;
        }
        const uint64_t m = __ballot(bad);
        if (m) {
            const int first = __builtin_ctzll(m);
            const uint32_t g2 = __shfl(got, first, 64), e2 = __shfl(ex, first, 64);
            if (lane == 0) {
                o.bad_seg = (int32_t)(base + first);
                o.got = g2;
                o.expect = e2;
            }
            return;
        }
    }
}

}  // namespace jfsx

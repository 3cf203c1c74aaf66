// jfsx_zstd.hip -- Zstandard frame decompression on gfx950 (the load side of
// --compress zstd volumes): one wave per object, the decoder
// of jfsx_zstd.h run wave-uniformly.
//
// Replaces ZStandard.Decompress = zstd.Decompress(dst, src)
// (pkg/compress/compress.go:93-100; DataDog/zstd v1.5.0) as called by
// cachedStore.load (pkg/chunk/cached_store.go:680-745).
//   * The compressed input is read with scalar loads (uniform addresses:
//     the bit readers' 8-byte windows come from the scalar cache).
//   * Decoding tables live in LDS (jzd::Tables, 20 KiB); table writes come
//     from lane 0 and every lane reads them (same wave: LDS order holds).
//   * Huffman literals go to a per-object 128 KiB scratch buffer; literal,
//     raw and RLE runs and matches are copied by the 64 lanes; a match reads
//     output written before it once the wave's stores have completed
//     (s_waitcnt vmcnt(0)), overlapping matches as out[o+j] = out[o-off+j%off].
#include "jfsx_dev.h"
#include "jfsx_zstd.h"
#include "jfsx_zstd2.h"

namespace jfsx {

namespace {

typedef __attribute__((address_space(4))) const uint32_t ccu32;
typedef __attribute__((address_space(1))) const uint8_t gcu8z;
typedef __attribute__((address_space(1))) uint8_t gu8z;

struct DevEnv {
    const uint8_t *src;  // compressed object
    int32_t n;
    uint8_t *dst;        // output (frame positions are offsets from dst)
    uint8_t *lit;        // literal scratch (kZstdScratch bytes)
    uint32_t lane;
    uint32_t fenced;     // output below this is visible to the wave's loads
    uint32_t lw0, lwv;   // literal window: scratch bytes [lw0, lw0 + 256), lane L holds dword L
#ifdef JFSX_ZSTD_STAMP
    unsigned long long st[8], last;
    __device__ __forceinline__ void stamp(int k) {
        unsigned long long t;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        st[k] += t - last;
        last = t;
    }
#else
    __device__ __forceinline__ void stamp(int) {}
#endif

    // input dword d (bytes [4d - sh, 4d - sh + 4) of src, src = al + sh), zero
    // when it holds no input byte; scalar load (uniform address)
    __device__ __forceinline__ uint32_t dw(int32_t d) const {
        const uintptr_t al = (uintptr_t)src & ~(uintptr_t)3;
        const int32_t sh = (int32_t)((uintptr_t)src & 3);
        const int32_t b0 = 4 * d - sh;  // first src byte of the dword
        if (b0 + 3 < 0 || b0 >= n) return 0u;
        uint32_t v = ZD_U32(*(ccu32 *)(al + 4 * (int64_t)d));
        // bytes outside [0, n) read as zero
        if (b0 < 0) v &= 0xffffffffu << (8 * (uint32_t)(-b0));
        if (b0 + 4 > n) v &= 0xffffffffu >> (8 * (uint32_t)(b0 + 4 - n));
        return v;
    }
    __device__ __forceinline__ uint32_t in8(int32_t i) const {
        if (i < 0 || i >= n) return 0;
        const int32_t x = i + (int32_t)((uintptr_t)src & 3);
        return (dw(x >> 2) >> (8 * (uint32_t)(x & 3))) & 255u;
    }
    __device__ __forceinline__ uint64_t in64(int32_t i) const {
        const int32_t x = i + (int32_t)((uintptr_t)src & 3);
        const int32_t d = x >> 2;  // floor (x may be negative)
        const uint32_t s = (uint32_t)(x & 3);
        const uint64_t lo = (uint64_t)dw(d) | ((uint64_t)dw(d + 1) << 32);
        if (!s) return lo;
        const uint64_t hi = dw(d + 2);
        return (lo >> (8 * s)) | (hi << (64 - 8 * s));
    }
    // bytes [i, i + 8), all inside the input: three scalar dword loads
    __device__ __forceinline__ uint64_t in64u(int32_t i) const {
        const uintptr_t a = (uintptr_t)src + (uint32_t)i;
        const uintptr_t al = a & ~(uintptr_t)3;
        const uint32_t sh = 8 * (uint32_t)(a & 3);
        const uint64_t lo = (uint64_t)ZD_U32(*(ccu32 *)al) | ((uint64_t)ZD_U32(*(ccu32 *)(al + 4)) << 32);
        // the third dword holds an input byte only when a is unaligned
        const uint64_t hi = ZD_U32(*(ccu32 *)(al + (sh ? 8 : 4)));
        return (lo >> sh) | ((hi << 32) << (32 - sh));
    }
    __device__ __forceinline__ void lit_put(uint32_t i, uint32_t b) const {
        if (lane == 0) *(gu8z *)(lit + i) = (uint8_t)b;
    }
    // 4 × 4 literal bytes: w_j's bytes at o_j .. o_j + 3 (lanes 0-15, one store)
    __device__ __forceinline__ void lit_put4(uint32_t o0, uint32_t w0, uint32_t o1, uint32_t w1, uint32_t o2,
                                             uint32_t w2, uint32_t o3, uint32_t w3) const {
        if (lane < 16) {
            const uint32_t j = lane >> 2, i = lane & 3;
            const uint32_t o = j == 0 ? o0 : j == 1 ? o1 : j == 2 ? o2 : o3;
            const uint32_t w = j == 0 ? w0 : j == 1 ? w1 : j == 2 ? w2 : w3;
            *(gu8z *)(lit + o + i) = (uint8_t)(w >> (8 * i));
        }
    }
    __device__ __forceinline__ void lit_fill(uint32_t i, uint32_t b, uint32_t cnt) const {
        for (uint32_t j = lane; j < cnt; j += 64) *(gu8z *)(lit + i + j) = (uint8_t)b;
    }
    __device__ __forceinline__ void fence() const {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    __device__ __forceinline__ void lit_sync() {
        fence();
        lw0 = 0xffffffffu;  // the block's literals are new
    }
    __device__ __forceinline__ void huf_fill(uint16_t *p, uint16_t v, uint32_t cnt) const {
        for (uint32_t j = lane; j < cnt; j += 64) p[j] = v;
    }
    // log-12 Huffman tables (none from libzstd's encoder): global scratch
    __device__ __forceinline__ uint16_t *huf_g() const { return (uint16_t *)(lit + kZstdHufOff); }
    __device__ __forceinline__ void huf_sync() const { fence(); }
    __device__ __forceinline__ uint32_t huf_ld(uint32_t i) const {
        return ZD_U32(*(const __attribute__((address_space(1))) uint16_t *)(lit + kZstdHufOff + 2 * i));
    }
    __device__ __forceinline__ void out_sync() const { fence(); }
    __device__ __forceinline__ void out_from_in(uint32_t o, int32_t i, uint32_t cnt) const {
        for (uint32_t j = lane; j < cnt; j += 64) *(gu8z *)(dst + o + j) = (uint8_t)in8_v(i + (int32_t)j);
    }
    // per-lane input byte (vector load)
    __device__ __forceinline__ uint32_t in8_v(int32_t i) const { return *(gcu8z *)(src + i); }
    // literal runs of up to 252 bytes come from a 256-byte register window of
    // the literal buffer (one load per window, not one per sequence)
    __device__ __forceinline__ void out_from_lit(uint32_t o, uint32_t i, uint32_t cnt) {
        if (cnt == 0) return;
        if (cnt <= 252) {
            if (i < lw0 || i + cnt > lw0 + 256u) {
                lw0 = i & ~3u;
                lwv = *(const __attribute__((address_space(1))) uint32_t *)(lit + lw0 + 4 * lane);
            }
            const uint32_t r = i - lw0;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                if (64 * k >= cnt) break;
                const uint32_t j = lane + 64 * k, q = r + j;
                const uint32_t d = __shfl(lwv, (int)((q >> 2) & 63), 64);
                if (j < cnt) *(gu8z *)(dst + o + j) = (uint8_t)(d >> (8 * (q & 3)));
            }
            return;
        }
        for (uint32_t j = lane; j < cnt; j += 64) *(gu8z *)(dst + o + j) = *(gcu8z *)(lit + i + j);
    }
    __device__ __forceinline__ void out_fill(uint32_t o, uint32_t b, uint32_t cnt) const {
        for (uint32_t j = lane; j < cnt; j += 64) *(gu8z *)(dst + o + j) = (uint8_t)b;
    }
    __device__ __forceinline__ void out_match(uint32_t o, uint32_t off, uint32_t cnt) {
        // wait for the wave's stores only when the source reaches past the
        // last fence (the output before o is all written by then)
        if (o - off + (off < cnt ? off : cnt) > fenced) {
            fence();
            fenced = o;
        }
        const uint8_t *m = dst + o - off;
        if (off >= cnt) {
            for (uint32_t j = lane; j < cnt; j += 64) *(gu8z *)(dst + o + j) = *(gcu8z *)(m + j);
        } else {
            for (uint32_t j = lane; j < cnt; j += 64) *(gu8z *)(dst + o + j) = *(gcu8z *)(m + j % off);
        }
    }
    __device__ __forceinline__ uint64_t out64(uint32_t o) const {
        uint64_t v = 0;
        for (uint32_t k = 0; k < 8; k++) v |= (uint64_t)(*(gcu8z *)(dst + o + k)) << (8 * k);
        return v;
    }
    __device__ __forceinline__ uint32_t out32(uint32_t o) const {
        uint32_t v = 0;
        for (uint32_t k = 0; k < 4; k++) v |= (uint32_t)(*(gcu8z *)(dst + o + k)) << (8 * k);
        return v;
    }
    __device__ __forceinline__ uint32_t out8(uint32_t o) const { return *(gcu8z *)(dst + o); }
};

}  // namespace

#ifdef JFSX_ZSTD_STAMP
__device__ unsigned long long g_zstd_stamps[8];  // diagnostic build: cycles per decoder section
}  // namespace jfsx
extern "C" int jfsx_debug_zstd_stamps(unsigned long long *out, int reset) {
    // out[0..7]: cycles per section; out[8..11]: jzd2 counters (ZSTAT)
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(jfsx::g_zstd_stamps), 64) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out + 8, HIP_SYMBOL(jzd2::g_zstd_counts), 32) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(jfsx::g_zstd_stamps), z, 64) != hipSuccess) return -1;
        if (hipMemcpyToSymbol(HIP_SYMBOL(jzd2::g_zstd_counts), z, 32) != hipSuccess) return -1;
    }
    return 0;
}
namespace jfsx {
#endif

// One wave per object.  ZDev.len = compressed bytes, ZDev.cap = dst capacity;
// ZOut.out_len = decoded bytes, status JFSX_EFORMAT for a frame
// ZSTD_decompress rejects, JFSX_EDSTSIZE for one whose output does not fit in
// cap (ZSTD_decompress's dstSize_tooSmall).
__global__ __launch_bounds__(64) void zstd_decompress_k(const ZDev *__restrict__ blks, ZOut *__restrict__ outs,
                                                        uint8_t *__restrict__ scratch) {
    __shared__ jzd::Tables T;
    const ZDev b = blks[blockIdx.x];
    DevEnv e{b.src, (int32_t)b.len, b.dst, scratch + (size_t)blockIdx.x * kZstdScratch, threadIdx.x, 0, 0xffffffffu, 0};
#ifdef JFSX_ZSTD_STAMP
    for (int k = 0; k < 8; k++) e.st[k] = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(e.last)::"memory");
#endif
    const int64_t r = jzd::decompress(e, T, b.len, b.cap);
#ifdef JFSX_ZSTD_STAMP
    if (threadIdx.x == 0)
        for (int k = 0; k < 8; k++) atomicAdd(&g_zstd_stamps[k], e.st[k]);
#endif
    if (threadIdx.x == 0) {
        outs[blockIdx.x].out_len = r < 0 ? 0 : (uint64_t)r;
        outs[blockIdx.x].status = r >= 0 ? JFSX_OK : r == jzd::ZD_EDSTSIZE ? JFSX_EDSTSIZE : JFSX_EFORMAT;
    }
}

// Block-parallel decoding (jfsx_zstd2.h), persistent waves: wave w decodes
// objects w, w + W, ... in its own arena of kZstdArena bytes.  An object the
// fast path does not take is marked (ZOut.fallback = why) and decoded by
// zstd_fallback_k, the serial decoder in a second launch over the same waves
// and arenas (scratch at the start of the arena), which sets the exact
// status.  Two kernels keep the serial decoder's registers out of this one.
__global__ __launch_bounds__(64) void zstd_decompress_par_k(const ZDev *__restrict__ blks, ZOut *__restrict__ outs,
                                                            uint8_t *__restrict__ arenas, int n) {
    __shared__ jzd2::Shared S;
    uint8_t *arena = arenas + (size_t)blockIdx.x * jzd2::kArena;
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        const ZDev b = blks[i];
        DevEnv e{b.src, (int32_t)b.len, b.dst, arena, threadIdx.x, 0, 0xffffffffu, 0};
#ifdef JFSX_ZSTD_STAMP
        for (int k = 0; k < 8; k++) e.st[k] = 0;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(e.last)::"memory");
#endif
        const int32_t r = jzd2::decompress_par(e, S, arena, b.len, b.cap);
#ifdef JFSX_ZSTD_STAMP
        if (threadIdx.x == 0)
            for (int k = 0; k < 8; k++) atomicAdd(&g_zstd_stamps[k], e.st[k]);
#endif
        if (threadIdx.x == 0) {
            outs[i].out_len = r < 0 ? 0 : (uint64_t)r;
            outs[i].status = r < 0 ? JFSX_EFORMAT : JFSX_OK;
            outs[i].fallback = r <= jzd2::kFallback ? -r - 2 : 0;
        }
        jzd2::wave_fence();
    }
}

__global__ __launch_bounds__(64) void zstd_fallback_k(const ZDev *__restrict__ blks, ZOut *__restrict__ outs,
                                                      uint8_t *__restrict__ arenas, int n) {
    __shared__ jzd::Tables T;
    uint8_t *arena = arenas + (size_t)blockIdx.x * jzd2::kArena;
    for (int i = blockIdx.x; i < n; i += gridDim.x) {
        if (!jzd2::uni((uint32_t)outs[i].fallback)) continue;
        const ZDev b = blks[i];
        DevEnv e{b.src, (int32_t)b.len, b.dst, arena, threadIdx.x, 0, 0xffffffffu, 0};
        const int64_t r = jzd::decompress(e, T, b.len, b.cap);
        if (threadIdx.x == 0) {
            outs[i].out_len = r < 0 ? 0 : (uint64_t)r;
            outs[i].status = r >= 0 ? JFSX_OK : r == jzd::ZD_EDSTSIZE ? JFSX_EDSTSIZE : JFSX_EFORMAT;
        }
        jzd2::wave_fence();
    }
}

int zstd_par_waves(int n, int ncu) { return n < ncu * kZstdWavesPerCu ? n : ncu * kZstdWavesPerCu; }

void launch_zstd_decompress(hipStream_t s, int n, const ZDev *blks, ZOut *outs, uint8_t *scratch, int waves) {
    if (n <= 0) return;
    if (waves > 0) {
        hipLaunchKernelGGL(zstd_decompress_par_k, dim3(waves), dim3(64), 0, s, blks, outs, scratch, n);
        hipLaunchKernelGGL(zstd_fallback_k, dim3(waves), dim3(64), 0, s, blks, outs, scratch, n);
    } else
        hipLaunchKernelGGL(zstd_decompress_k, dim3(n), dim3(64), 0, s, blks, outs, scratch);
}

}  // namespace jfsx

// jfsx_crc.hip -- CRC32C per 32 KiB segment over ranges (gfx950), and the
// synthetic-input generator.
//
// crc32c_segments replaces the CRC loops of checksum() (pkg/chunk/disk_cache.go:
// 1218-1231) and of cacheFile.ReadAt (disk_cache.go:1315-1327) for cache hits,
// none-cipher volumes and the staging re-read (pkg/chunk/cached_store.go:961-971).
// One wave per 32 KiB segment, 64 lanes x 16 B per row, slice-by-16 tables in
// LDS; lane CRCs are shifted to the segment end (GF(2) multiply by x^(8d) mod P)
// and XOR-reduced across the wave.
#include "jfsx_dev.h"

namespace jfsx {

constexpr uint32_t kCrcWaves = 4;  // 256-thread workgroups, one segment per wave
constexpr uint32_t kLdsCrcOnly = 0;

__global__ __launch_bounds__(kCrcWaves * 64) void crc_segments_k(const Task *__restrict__ tasks,
                                                                const BlkDev *__restrict__ blks, DevTables tab) {
    __shared__ __attribute__((aligned(16))) char lds[20480];
    const Task task = tasks[blockIdx.x];
    const BlkDev blk = blks[task.blk];
    const uint32_t tid = threadIdx.x;
    {
        const uint4 *gc = reinterpret_cast<const uint4 *>(tab.crc);
        uint4 *lc = reinterpret_cast<uint4 *>(lds);
        for (uint32_t i = tid; i < 1280; i += kCrcWaves * 64) lc[i] = gc[i];
    }
    __syncthreads();
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t seg0 = task.c0 + (uint64_t)wave * kSeg;
    if (seg0 >= task.c1) return;
    const uint64_t seg1 = seg0 + kSeg < task.c1 ? seg0 + kSeg : task.c1;
    const uint8_t *src = blk.src;
    uint32_t A = 0, lend = 0;
    const uint64_t nrows = (seg1 - seg0 + 1023) / 1024;
    uint4 nxt = load_piece(src, seg0 + 16 * lane, seg1);
    for (uint64_t r = 0; r < nrows; r++) {
        const uint64_t o = seg0 + 1024 * r + 16 * lane;
        uint4 p = nxt;
        if (r + 1 < nrows) nxt = load_piece(src, o + 1024, seg1);
        if (o + 16 <= seg1) {
            A = crc_piece<kLdsCrcOnly>(lds, A, p.x, p.y, p.z, p.w);
            lend = (uint32_t)(o + 16 - seg0);
        } else if (o < seg1) {
            const uint32_t pw[4] = {p.x, p.y, p.z, p.w};
            A = crc_partial<kLdsCrcOnly>(lds, A, pw, (int)(seg1 - o));
            lend = (uint32_t)(seg1 - seg0);
        }
    }
    const uint32_t Lseg = (uint32_t)(seg1 - seg0);
    uint32_t v, K;
    if (Lseg == (uint32_t)kSeg) {
        v = crc_mulmod(tab.crcx[lane], A);
        K = tab.crcx[96];
    } else {
        v = crc_mulmod(crc_xpow8(Lseg - lend, tab.crcx + 64), A);
        K = crc_mulmod(crc_xpow8(Lseg, tab.crcx + 64), 0xffffffffu);
    }
    const uint32_t raw = wave_xor(v);
    if (lane == 0) {
        const uint32_t crc = ~(K ^ raw);
        const uint64_t si = seg0 / kSeg;
        if (blk.crc_calc)
            blk.crc_calc[si] = crc;
        else
            *reinterpret_cast<uint32_t *>(blk.crc + 4 * si) = __builtin_bswap32(crc);
    }
}

// zero-length ranges/blocks still produce one zero CRC (Go's checksum(): 4 bytes)
__global__ __launch_bounds__(64) void crc_finalize_k(const BlkDev *__restrict__ blks, int crc_mode,
                                                    BlkOut *__restrict__ out) {
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    const BlkDev blk = blks[b];
    BlkOut o;
    for (int q = 0; q < 4; q++) o.tag[q] = 0;
    o.status = JFSX_OK;
    o.bad_seg = -1;
    o.got = o.expect = 0;
    if (crc_mode == JFSX_CRC_GEN && blk.len == 0 && lane == 0) *reinterpret_cast<uint32_t *>(blk.crc) = 0;
    if (crc_mode == JFSX_CRC_VERIFY) {
        crc_verify_block(blk, o, lane);
        if (o.bad_seg >= 0) o.status = JFSX_ECRC;
    }
    if (lane == 0) out[b] = o;
}

// SplitMix64 stream: word k of block b = mix64(seed + G*((b << 40) + k + 1))
// (identical to oracle/jfs_oracle.c orc_gen_block)
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void gen_synthetic_k(uint8_t *__restrict__ dst, uint64_t len, uint64_t seed,
                                                      uint64_t block) {
    const uint64_t G = 0x9E3779B97F4A7C15ULL;
    const uint64_t nw2 = len / 16;
    const uint64_t base = seed + G * ((block << 40) + 1);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nw2;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = mix64(base + G * (2 * i)), b = mix64(base + G * (2 * i + 1));
        *reinterpret_cast<ulonglong2 *>(dst + 16 * i) = make_ulonglong2(a, b);
    }
    if (blockIdx.x == 0 && threadIdx.x < 16) {
        const uint64_t i = nw2 * 16 + threadIdx.x;
        if (i < len) {
            const uint64_t w = mix64(base + G * (i / 8));
            dst[i] = (uint8_t)(w >> (8 * (i % 8)));
        }
    }
}

void launch_crc_segments(hipStream_t s, int ntasks, const Task *tasks, const BlkDev *blks, DevTables t) {
    if (ntasks > 0) hipLaunchKernelGGL(crc_segments_k, dim3(ntasks), dim3(kCrcWaves * 64), 0, s, tasks, blks, t);
}

void launch_crc_finalize(hipStream_t s, int n, int crc_mode, const BlkDev *blks, BlkOut *out) {
    if (n > 0) hipLaunchKernelGGL(crc_finalize_k, dim3(n), dim3(64), 0, s, blks, crc_mode, out);
}

void launch_gen_synthetic(hipStream_t s, uint8_t *dst, uint64_t len, uint64_t seed, uint64_t block) {
    uint64_t nw2 = len / 16;
    uint64_t blocks = (nw2 + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(gen_synthetic_k, dim3((unsigned)blocks), dim3(256), 0, s, dst, len, seed, block);
}

}  // namespace jfsx

// AddressSanitizer run of the engine's Zstandard decoder (jfsx_zstd.h through
// the host harness zstd_host.cpp): frames with XXH64 content checksums whose
// lengths are not multiples of 8 decode into buffers that end exactly at the
// decoded size, so a read past the output (the checksum tail) is reported.
// Frames come from the system libzstd (dlopen'ed; test infrastructure only).
#include <dlfcn.h>
#include <stdio.h>

#include "zstd_host.cpp"

typedef void *(*cctx_new_t)(void);
typedef size_t (*cctx_free_t)(void *);
typedef size_t (*set_t)(void *, int, int);
typedef size_t (*comp2_t)(void *, void *, size_t, const void *, size_t);
typedef size_t (*bound_t)(size_t);
typedef unsigned (*iserr_t)(size_t);

int main() {
    void *z = dlopen("libzstd.so.1", RTLD_NOW);
    if (!z) {
        printf("libzstd.so.1 not loadable\n");
        return 2;
    }
    auto cnew = (cctx_new_t)dlsym(z, "ZSTD_createCCtx");
    auto cfree = (cctx_free_t)dlsym(z, "ZSTD_freeCCtx");
    auto cset = (set_t)dlsym(z, "ZSTD_CCtx_setParameter");
    auto comp2 = (comp2_t)dlsym(z, "ZSTD_compress2");
    auto bound = (bound_t)dlsym(z, "ZSTD_compressBound");
    auto iserr = (iserr_t)dlsym(z, "ZSTD_isError");
    uint64_t s = 0x243F6A8885A308D3ull;
    int fails = 0, cases = 0;
    const size_t sizes[] = {1, 3, 5, 7, 9, 13, 31, 33, 100, 1001, 4099, 65537, 131075, 300007};
    for (size_t n : sizes)
        for (int kind = 0; kind < 2; kind++) {
            std::vector<uint8_t> src(n);
            for (size_t i = 0; i < n; i++) {
                s = s * 6364136223846793005ull + 1442695040888963407ull;
                src[i] = kind ? (uint8_t)('a' + (s >> 60) % 6) : (uint8_t)(s >> 56);
            }
            void *cc = cnew();
            cset(cc, 100, 1);  // ZSTD_c_compressionLevel
            cset(cc, 201, 1);  // ZSTD_c_checksumFlag
            std::vector<uint8_t> frame(bound(n));
            const size_t fl = comp2(cc, frame.data(), frame.size(), src.data(), n);
            cfree(cc);
            if (iserr(fl)) return 3;
            // exact-size input and output allocations
            std::vector<uint8_t> in(frame.begin(), frame.begin() + fl);
            uint8_t *out = new uint8_t[n];
            const int64_t r = zstd_host_decompress(in.data(), (int64_t)fl, out, (int64_t)n);
            cases++;
            if (r != (int64_t)n || memcmp(out, src.data(), n) != 0) {
                printf("mismatch n=%zu kind=%d r=%lld\n", n, kind, (long long)r);
                fails++;
            }
            delete[] out;
        }
    printf("zstd asan run: %d cases, %d failures\n", cases, fails);
    if (fails == 0) printf("zstd sanitizer run ok\n");
    return fails ? 1 : 0;
}

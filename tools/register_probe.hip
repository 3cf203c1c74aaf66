// register_probe.hip -- per-call cost of pinning a caller's pageable buffer
// (hipHostRegister / hipHostUnregister) against bouncing it (a memcpy into
// engine-pinned memory), for the per-object host path: the
// wall time of each on one thread, and the H2D rate from each source.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/register_probe tools/register_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t n = 4 << 20;
    const int reps = 200;
    char *d = nullptr, *pin = nullptr;
    if (hipMalloc((void **)&d, n) || hipHostMalloc((void **)&pin, n, hipHostMallocPortable)) return 1;
    hipStream_t s;
    hipStreamCreate(&s);
    for (int size_mb = 1; size_mb <= 4; size_mb *= 4) {
        const size_t m = (size_t)size_mb << 20;
        double t_reg = 0, t_unreg = 0, t_h2d_reg = 0, t_cpy = 0, t_h2d_pin = 0;
        double t_call_reg = 0, t_call_pin = 0, t_call_d2h = 0, t_d2h_reg = 0;
        for (int r = 0; r < reps; r++) {
            char *h = (char *)malloc(m + 4096);
            char *p = h + 64;  // a heap slice: not page aligned
            memset(h, r, m + 4096);
            double t0 = now();
            if (hipHostRegister(p, m, hipHostRegisterDefault) != hipSuccess) {
                printf("hipHostRegister failed\n");
                return 1;
            }
            double t1 = now();
            hipMemcpyAsync(d, p, m, hipMemcpyHostToDevice, s);
            double t1b = now();
            hipStreamSynchronize(s);
            double t2 = now();
            if (r >= 10) t_call_reg += t1b - t1;
            hipHostUnregister(p);
            double t3 = now();
            memcpy(pin, p, m);
            double t4 = now();
            hipMemcpyAsync(d, pin, m, hipMemcpyHostToDevice, s);
            double t4b = now();
            hipStreamSynchronize(s);
            double t5 = now();
            if (r >= 10) t_call_pin += t4b - t4;
            // the D2H direction into registered memory
            hipHostRegister(p, m, hipHostRegisterDefault);
            double t6 = now();
            hipMemcpyAsync(p, d, m, hipMemcpyDeviceToHost, s);
            double t6b = now();
            hipStreamSynchronize(s);
            double t7 = now();
            hipHostUnregister(p);
            if (r >= 10) t_call_d2h += t6b - t6, t_d2h_reg += t7 - t6;
            if (r >= 10) {
                t_reg += t1 - t0, t_h2d_reg += t2 - t1, t_unreg += t3 - t2, t_cpy += t4 - t3, t_h2d_pin += t5 - t4;
            }
            free(h);
        }
        const int k = reps - 10;
        printf("{\"bytes\": %zu, \"register_us\": %.1f, \"unregister_us\": %.1f, \"h2d_registered_us\": %.1f, "
               "\"memcpy_to_pinned_us\": %.1f, \"h2d_pinned_us\": %.1f, \"async_call_registered_us\": %.1f, "
               "\"async_call_pinned_us\": %.1f, \"d2h_registered_us\": %.1f, \"d2h_async_call_registered_us\": %.1f}\n",
               m, 1e6 * t_reg / k, 1e6 * t_unreg / k, 1e6 * t_h2d_reg / k, 1e6 * t_cpy / k, 1e6 * t_h2d_pin / k,
               1e6 * t_call_reg / k, 1e6 * t_call_pin / k, 1e6 * t_d2h_reg / k, 1e6 * t_call_d2h / k);
    }
    return 0;
}

// Store drain under staggered wave arrival (the step kernel's shape): each 64-row wave waits
// `delay(block)` before its block store.  Shows whether the write drain rate depends on how many
// waves store concurrently, and what nontemporal stores change.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
constexpr int OBS = 297, ROWS = 64;

__device__ __forceinline__ void spin_us(uint32_t us) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)us * 100) __builtin_amdgcn_s_sleep(2);
}

template <bool NT>
__global__ __launch_bounds__(64) void k_stag(int32_t *out, int spread_us) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[ROWS * OBS];
    const int lane = threadIdx.x, t0 = blockIdx.x * ROWS;
    for (int i = 0; i < OBS; ++i) rows[lane * OBS + i] = (uint8_t)(i + lane);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    if (spread_us) spin_us((uint32_t)((blockIdx.x * 2654435761u) % (uint32_t)(spread_us + 1)));
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows);
    int32_t *dst = out + (size_t)t0 * OBS;
    const int full = ROWS * OBS / 4;
    int d = lane;
    for (; d + 64 * 4 < full; d += 64 * 5) {
        uint32_t w[5];
#pragma unroll
        for (int u = 0; u < 5; ++u) w[u] = src[d + 64 * u];
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            typedef int v4i __attribute__((ext_vector_type(4)));
            v4i v = {(int)(w[u] & 0xFF), (int)((w[u] >> 8) & 0xFF), (int)((w[u] >> 16) & 0xFF), (int)(w[u] >> 24)};
            v4i *p = reinterpret_cast<v4i *>(dst + 4 * (d + 64 * u));
            if (NT) __builtin_nontemporal_store(v, p); else *p = v;
        }
    }
    for (; d < full; d += 64) {
        const uint32_t w = src[d];
        *reinterpret_cast<int4 *>(dst + 4 * d) = make_int4(w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24);
    }
}

template <typename F>
float timeit(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    launch(); hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return 1000.f * ms / reps;
}

int main() {
    const int n = 65536;
    const size_t bytes = (size_t)n * OBS * 4;
    int32_t *out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    for (int spread : {0, 10, 20, 30}) {
        float p = timeit([&] { k_stag<false><<<n / 64, 64>>>(out, spread); }, 30);
        float q = timeit([&] { k_stag<true><<<n / 64, 64>>>(out, spread); }, 30);
        printf("spread %2d us: plain %7.2f us   nt %7.2f us   (drain-only est plain %6.2f, %6.0f GB/s)\n", spread, p, q,
               p - spread, bytes / 1e3 / (p - 0.5 * spread));
    }
    hipFree(out);
    return 0;
}

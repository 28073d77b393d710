// Why does the step kernel's observation store run at half the rate of microbench_store's
// unroll-5 loop?  Same loop, varying one difference at a time:
//   LDS footprint per wave (19 KB vs the engine's 40 KB), a state-load phase before the stores
//   (22 word planes per lane, like load_tab + load_pool), and timing (amortised over 50
//   back-to-back launches vs an event pair around every launch).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_store3.hip -o /tmp/mbs3 && /tmp/mbs3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("%s: %s\n", #x, hipGetErrorString(e));                          \
            return 1;                                                              \
        }                                                                          \
    } while (0)
constexpr int OBS = 297, ROWS = 64, PLANES = 22;

template <int LDS_BYTES, bool LOAD, bool FILL = true>
__global__ __launch_bounds__(64) void k_store(int32_t *out, const uint32_t *planes, int n) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    uint8_t *rows = lds;
    const int lane = threadIdx.x, t0 = blockIdx.x * ROWS, t = t0 + lane;
    uint32_t acc = (uint32_t)lane;
    if (LOAD) {
#pragma unroll
        for (int w = 0; w < PLANES; ++w) acc += planes[(size_t)w * n + t];
    }
    if (FILL)
        for (int i = 0; i < OBS; ++i) rows[lane * OBS + i] = (uint8_t)(i + acc);
    else
        rows[lane] = (uint8_t)acc;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows);
    int32_t *dst = out + (size_t)t0 * OBS;
    const int full = ROWS * OBS / 4;
    constexpr int U = 5;
    int d = lane;
    for (; d + 64 * (U - 1) < full; d += 64 * U) {
        uint32_t w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = src[d + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u)
            *reinterpret_cast<int4 *>(dst + 4 * (d + 64 * u)) =
                make_int4(w[u] & 0xFF, (w[u] >> 8) & 0xFF, (w[u] >> 16) & 0xFF, w[u] >> 24);
    }
    for (; d < full; d += 64) {
        const uint32_t w = src[d];
        *reinterpret_cast<int4 *>(dst + 4 * d) = make_int4(w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24);
    }
}

template <typename F>
float amortised(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return 1000.f * ms / reps;
}

template <typename F>
float per_launch(F launch, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipDeviceSynchronize();
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(a);
        launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        tot += ms;
    }
    return 1000.f * tot / reps;
}

int main() {
    const int n = 65536;
    const size_t bytes = (size_t)n * OBS * 4;
    int32_t *out;
    uint32_t *planes;
    CHECK(hipMalloc(&out, bytes + 4096));
    CHECK(hipMalloc(&planes, (size_t)PLANES * n * 4));
    CHECK(hipMemset(planes, 1, (size_t)PLANES * n * 4));
    const double mb = bytes / 1e6;
    const int reps = 50;
    auto rep = [&](const char *name, float a, float p) {
        printf("%-34s amortised %7.2f us (%6.0f GB/s)   per-launch events %7.2f us\n", name, a, mb * 1e3 / a, p);
    };
#define RUN(NAME, LDSB, LOAD, ...)                                                                 \
    {                                                                                              \
        auto l = [&] { k_store<LDSB, LOAD, ##__VA_ARGS__><<<n / 64, 64>>>(out, planes, n); };      \
        rep(NAME, amortised(l, reps), per_launch(l, reps));                                        \
    }
    RUN("lds 19 KB, no loads", 19072, false);
    RUN("lds 40 KB, no loads", 40064, false);
    RUN("lds 19 KB, 22-plane loads", 19072, true);
    RUN("lds 40 KB, 22-plane loads", 40064, true);
    RUN("lds 80 KB, 22-plane loads", 80064, true);
    RUN("lds 40 KB, no loads, no LDS fill", 40064, false, false);
    RUN("lds 40 KB, 22-plane loads, no fill", 40064, true, false);
    CHECK(hipFree(out));
    CHECK(hipFree(planes));
    return 0;
}

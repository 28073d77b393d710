// Cache-policy variants of the rollout store's write pattern (one wave per 64 tables, rows [K][T][297]
// int32, 5 GB per launch): plain / __builtin_nontemporal_store / buffer stores with aux cache bits
// (1 = sc0, 2 = nt, 16 = sc1).  A second set runs the same stores while a second wave per workgroup
// gathers from a 384 KB table (the token-return table's size) and reports how long those gathers
// took: the stores that keep their lines in L2 push the table out.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_store_policy.hip -o /tmp/mbp && /tmp/mbp
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int OBS = 297, ROWS = 64;
constexpr int ROW_V4 = ROWS * OBS / 4;  // 4752 16-byte vectors per 64-row block

// MODE: 0 plain, 1 builtin nontemporal, 2 buffer store with aux AUX
template <int MODE, int AUX>
__device__ __forceinline__ void st(v4i *blk, int d, v4i v) {
    if (MODE == 0) blk[d] = v;
    else if (MODE == 1) __builtin_nontemporal_store(v, blk + d);
    else {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(blk, (short)0, ROW_V4 * 16, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, d * 16, 0, AUX);
    }
}

// W = 1: store wave only; W = 2: wave 1 gathers from `tab` (n4 vectors) each step and records its time
template <int MODE, int AUX, int W>
__global__ __launch_bounds__(64 * W) void k_rows(v4i *out, int T, int K, const v4i *tab, int n4, unsigned long long *gt) {
    const int lane = threadIdx.x & 63;
    const size_t blk = (size_t)T * OBS / 4;
    if (threadIdx.x < 64) {
        for (int k = 0; k < K; ++k) {
            v4i *dst = out + (size_t)k * blk + (size_t)blockIdx.x * ROW_V4;
            int d = lane;
            for (; d + 64 * 4 < ROW_V4; d += 64 * 5) {
#pragma unroll
                for (int u = 0; u < 5; ++u) st<MODE, AUX>(dst, d + 64 * u, v4i{k, d, u, 0});
            }
            for (; d < ROW_V4; d += 64) st<MODE, AUX>(dst, d, v4i{k, d, 0, 0});
        }
    } else {
        uint32_t x = blockIdx.x * 64 + lane, acc = 0;
        const unsigned long long t0 = wall_clock64();
        for (int k = 0; k < 8 * K; ++k) {  // dependent random gathers, about one per 2 us of stores
            x = x * 1664525u + 1013904223u + acc;
            const v4i v = tab[x % (uint32_t)n4];
            acc += (uint32_t)v.x & 1u;
            __builtin_amdgcn_s_sleep(20);
        }
        const unsigned long long t1 = wall_clock64();
        if (lane == 0) gt[blockIdx.x] = t1 - t0;
        if (acc == 12345678u) out[0] = v4i{1, 2, 3, 4};
    }
}

template <typename F>
static float timeit(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const int T = 65536, K = 64;
    const size_t bytes = (size_t)K * T * OBS * 4;
    const int nb = T / ROWS;
    v4i *out, *tab;
    unsigned long long *gt;
    const int n4 = 393216 / 16;
    CHECK(hipMalloc(&out, bytes));
    CHECK(hipMalloc(&tab, (size_t)n4 * 16));
    CHECK(hipMemset(tab, 1, (size_t)n4 * 16));
    CHECK(hipMalloc(&gt, nb * sizeof(unsigned long long)));
    int wclk = 100000;
    hipDeviceGetAttribute(&wclk, hipDeviceAttributeWallClockRate, 0);  // kHz
    unsigned long long h[1024];
    auto rep = [&](const char *name, float ms, bool gathers) {
        printf("%-44s %9.1f us  %7.1f GB/s", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
        if (gathers) {
            hipMemcpy(h, gt, sizeof(h), hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < nb; ++i) s += (double)h[i];
            printf("   gather wave %8.1f us (mean)", s / nb / (wclk * 1e-3));
        }
        printf("\n");
    };
    printf("# store cache policies, rows [K][T] 1 wave/64 tables, %.2f GB per launch\n", bytes / 1e9);
#define V(MODE, AUX, NAME)                                                                                          \
    rep(NAME, timeit([&] { k_rows<MODE, AUX, 1><<<nb, 64>>>(out, T, K, tab, n4, gt); }, 5), false);                  \
    rep(NAME " + gathers", timeit([&] { k_rows<MODE, AUX, 2><<<nb, 128>>>(out, T, K, tab, n4, gt); }, 5), true);
    V(0, 0, "plain")
    V(1, 0, "builtin nontemporal")
    V(2, 0, "buffer aux 0")
    V(2, 1, "buffer sc0")
    V(2, 2, "buffer nt")
    V(2, 16, "buffer sc1")
    V(2, 17, "buffer sc0 sc1")
    V(2, 18, "buffer nt sc1")
    V(2, 19, "buffer sc0 nt sc1")
    CHECK(hipFree(out));
    CHECK(hipFree(tab));
    CHECK(hipFree(gt));
    return 0;
}

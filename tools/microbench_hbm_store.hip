// HBM write-bandwidth micro-benchmark for the rollout store: how fast can 1024-2048 waves write a
// [K][T][297] int32 block (5 GB at K=64, T=65536 — 20x the 256 MiB Infinity Cache) compared with a
// grid-stride stream of the same bytes?  Variants: plain / nontemporal stores, one wave per 64 rows
// (the rollout kernel's output wave) or grid-stride, 1 or 2 output waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_hbm_store.hip -o /tmp/mbh && /tmp/mbh
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int OBS = 297, ROWS = 64;
constexpr int ROW_V4 = ROWS * OBS / 4;  // 4752 16-byte vectors per 64-row block

template <bool NT>
__device__ __forceinline__ void st(v4i *p, v4i v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// grid-stride stream of n4 vectors
template <bool NT>
__global__ __launch_bounds__(256) void k_grid(v4i *out, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        st<NT>(out + i, v4i{(int)i, 1, 2, 3});
}

// rollout-store shape: one wave owns 64 tables; for k = 0..K-1 it writes its 64 rows of block k
// (76 KB contiguous), block k at k*T*297 ints.  `spin` adds VALU work between blocks (the rules).
template <bool NT>
__global__ __launch_bounds__(64) void k_rows(v4i *out, int T, int K, int spin) {
    const int lane = threadIdx.x;
    const size_t blk = (size_t)T * OBS / 4;
    v4i *base = out + (size_t)blockIdx.x * ROW_V4;
    uint32_t x = lane;
    for (int k = 0; k < K; ++k) {
        for (int s = 0; s < spin; ++s) x = x * 1664525u + 1013904223u;
        v4i *dst = base + (size_t)k * blk;
        int d = lane;
        for (; d + 64 * 7 < ROW_V4; d += 64 * 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) st<NT>(dst + d + 64 * u, v4i{(int)x, k, d, u});
        }
        for (; d < ROW_V4; d += 64) st<NT>(dst + d, v4i{(int)x, k, d, 0});
    }
}

// same, but a workgroup of W waves covers W*64 tables (more waves per SIMD when W*blocks > 1024)
template <bool NT>
__global__ __launch_bounds__(256) void k_rows_w(v4i *out, int T, int K) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t blk = (size_t)T * OBS / 4;
    v4i *base = out + ((size_t)blockIdx.x * (blockDim.x >> 6) + w) * ROW_V4;
    for (int k = 0; k < K; ++k) {
        v4i *dst = base + (size_t)k * blk;
        int d = lane;
        for (; d + 64 * 7 < ROW_V4; d += 64 * 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) st<NT>(dst + d + 64 * u, v4i{k, d, u, 0});
        }
        for (; d < ROW_V4; d += 64) st<NT>(dst + d, v4i{k, d, 0, 0});
    }
}

// step-major variant: a wave writes ALL of its tables' K rows contiguously (layout [T][K][297]),
// i.e. 64*K rows = 4.9 MB per wave in one sequential stream
template <bool NT>
__global__ __launch_bounds__(64) void k_rows_tmajor(v4i *out, int T, int K) {
    const int lane = threadIdx.x;
    v4i *base = out + (size_t)blockIdx.x * ROW_V4 * K;
    const int total = ROW_V4 * K;
    int d = lane;
    for (; d + 64 * 7 < total; d += 64 * 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) st<NT>(base + d + 64 * u, v4i{d, u, 0, 0});
    }
    for (; d < total; d += 64) st<NT>(base + d, v4i{d, 0, 0, 0});
}

// R rows per wave (R = 64: 1024 waves, 32: 2048 waves), W waves per workgroup, optional second
// stream of 45-byte rows (the masks) after each obs block
template <bool NT, int R, bool MASK>
__global__ __launch_bounds__(256) void k_rows_r(v4i *out, v4i *mask, int T, int K) {
    constexpr int RV4 = R * OBS / 4;
    constexpr int MV4 = R * 45 / 16;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const size_t wave = (size_t)blockIdx.x * (blockDim.x >> 6) + w;
    const size_t blk = (size_t)T * OBS / 4, mblk = (size_t)T * 45 / 16;
    for (int k = 0; k < K; ++k) {
        v4i *dst = out + (size_t)k * blk + wave * RV4;
        int d = lane;
        for (; d + 64 * 4 < RV4; d += 64 * 5) {
#pragma unroll
            for (int u = 0; u < 5; ++u) st<NT>(dst + d + 64 * u, v4i{k, d, u, 0});
        }
        for (; d < RV4; d += 64) st<NT>(dst + d, v4i{k, d, 0, 0});
        if (MASK) {
            v4i *m = mask + (size_t)k * mblk + wave * MV4;
            for (int c = lane; c < MV4; c += 64) st<NT>(m + c, v4i{k, c, 0, 0});
        }
    }
}

// XCD-aware placement of the same [K][T] rows: the dispatcher hands workgroup b to XCD b % 8, so
// wave b writes block slot (b % 8) * (nw / 8) + b / 8 — each XCD's waves then cover one contiguous
// eighth of every step's 78 MB block instead of every eighth 76 KB chunk
template <bool NT, int R>
__global__ __launch_bounds__(64) void k_rows_x(v4i *out, int T, int K) {
    constexpr int RV4 = R * OBS / 4;
    const int lane = threadIdx.x;
    const size_t nw = gridDim.x;
    const size_t wave = (blockIdx.x % 8) * (nw / 8) + blockIdx.x / 8;
    const size_t blk = (size_t)T * OBS / 4;
    for (int k = 0; k < K; ++k) {
        v4i *dst = out + (size_t)k * blk + wave * RV4;
        int d = lane;
        for (; d + 64 * 4 < RV4; d += 64 * 5) {
#pragma unroll
            for (int u = 0; u < 5; ++u) st<NT>(dst + d + 64 * u, v4i{k, d, u, 0});
        }
        for (; d < RV4; d += 64) st<NT>(dst + d, v4i{k, d, 0, 0});
    }
}

// read + write copy (the guide's 6.29 TB/s float4 copy)
__global__ __launch_bounds__(256) void k_copy(const v4i *in, v4i *out, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in[i];
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
    const size_t bytes = (size_t)K * T * OBS * 4;  // 4.98 GB
    const size_t n4 = bytes / 16;
    v4i *out, *in;
    CHECK(hipMalloc(&out, bytes));
    CHECK(hipMalloc(&in, bytes));
    CHECK(hipMemset(in, 1, bytes));
    const int nb = T / ROWS;  // 1024 waves
    auto rep = [&](const char *name, float ms, double nbytes) {
        printf("%-58s %9.1f us  %7.1f GB/s\n", name, ms * 1e3, nbytes / (ms * 1e-3) / 1e9);
    };
    printf("# HBM store micro-benchmark, MI355X, %.2f GB per launch (K=%d x T=%d x 297 int32)\n", bytes / 1e9, K, T);
    rep("grid-stride v4 stores, 2048x256", timeit([&] { k_grid<false><<<2048, 256>>>(out, n4); }, 5), bytes);
    rep("grid-stride v4 stores, 8192x256", timeit([&] { k_grid<false><<<8192, 256>>>(out, n4); }, 5), bytes);
    rep("grid-stride v4 NT stores, 2048x256", timeit([&] { k_grid<true><<<2048, 256>>>(out, n4); }, 5), bytes);
    rep("grid-stride v4 NT stores, 8192x256", timeit([&] { k_grid<true><<<8192, 256>>>(out, n4); }, 5), bytes);
    rep("rows [K][T] 1 wave/64 tables (1024 waves)", timeit([&] { k_rows<false><<<nb, 64>>>(out, T, K, 0); }, 5), bytes);
    rep("rows [K][T] 1 wave/64 tables NT", timeit([&] { k_rows<true><<<nb, 64>>>(out, T, K, 0); }, 5), bytes);
    rep("rows [K][T] + 200 VALU/step", timeit([&] { k_rows<false><<<nb, 64>>>(out, T, K, 200); }, 5), bytes);
    rep("rows [K][T] + 200 VALU/step NT", timeit([&] { k_rows<true><<<nb, 64>>>(out, T, K, 200); }, 5), bytes);
    rep("rows [K][T] 4 waves/WG (1024 waves, 256 WG)", timeit([&] { k_rows_w<false><<<nb / 4, 256>>>(out, T, K); }, 5), bytes);
    rep("rows [K][T] 4 waves/WG NT", timeit([&] { k_rows_w<true><<<nb / 4, 256>>>(out, T, K); }, 5), bytes);
    // 2 waves per SIMD: half the tables per wave-block pairing, 2048 waves of 32-row... emulate by T2 = 2T rows of half K
    rep("rows [T][K] table-major 1024 waves", timeit([&] { k_rows_tmajor<false><<<nb, 64>>>(out, T, K); }, 5), bytes);
    rep("rows [T][K] table-major NT", timeit([&] { k_rows_tmajor<true><<<nb, 64>>>(out, T, K); }, 5), bytes);
    v4i *mk;
    CHECK(hipMalloc(&mk, (size_t)K * T * 45));
    rep("rows_r R=64 1 wave/WG (1024 waves)", timeit([&] { k_rows_r<false, 64, false><<<nb, 64>>>(out, mk, T, K); }, 5), bytes);
    rep("rows_r R=32 1 wave/WG (2048 waves)", timeit([&] { k_rows_r<false, 32, false><<<2 * nb, 64>>>(out, mk, T, K); }, 5), bytes);
    rep("rows_r R=32 2 waves/WG (2048 waves)", timeit([&] { k_rows_r<false, 32, false><<<nb, 128>>>(out, mk, T, K); }, 5), bytes);
    rep("rows_r R=32 NT 1 wave/WG", timeit([&] { k_rows_r<true, 32, false><<<2 * nb, 64>>>(out, mk, T, K); }, 5), bytes);
    rep("rows_r R=16 1 wave/WG (4096 waves)", timeit([&] { k_rows_r<false, 16, false><<<4 * nb, 64>>>(out, mk, T, K); }, 5), bytes);
    rep("rows_x R=64 XCD-contiguous (1024 waves)", timeit([&] { k_rows_x<false, 64><<<nb, 64>>>(out, T, K); }, 5), bytes);
    rep("rows_x R=64 XCD-contiguous NT", timeit([&] { k_rows_x<true, 64><<<nb, 64>>>(out, T, K); }, 5), bytes);
    rep("rows_x R=32 XCD-contiguous (2048 waves)", timeit([&] { k_rows_x<false, 32><<<2 * nb, 64>>>(out, T, K); }, 5), bytes);
    rep("rows_r R=64 1 wave/WG again (same-box A/B)", timeit([&] { k_rows_r<false, 64, false><<<nb, 64>>>(out, mk, T, K); }, 5), bytes);
    rep("rows_x R=64 XCD-contiguous again", timeit([&] { k_rows_x<false, 64><<<nb, 64>>>(out, T, K); }, 5), bytes);
    const double mb = bytes + (double)K * T * 45;
    rep("rows_r R=64 + mask stream", timeit([&] { k_rows_r<false, 64, true><<<nb, 64>>>(out, mk, T, K); }, 5), mb);
    rep("rows_r R=64 + mask stream NT", timeit([&] { k_rows_r<true, 64, true><<<nb, 64>>>(out, mk, T, K); }, 5), mb);
    rep("rows_r R=32 + mask stream (2048 waves)", timeit([&] { k_rows_r<false, 32, true><<<2 * nb, 64>>>(out, mk, T, K); }, 5), mb);
    rep("rows_r R=32 + mask stream NT", timeit([&] { k_rows_r<true, 32, true><<<2 * nb, 64>>>(out, mk, T, K); }, 5), mb);
    CHECK(hipFree(mk));
    rep("copy v4 2048x256 (read+write bytes)", timeit([&] { k_copy<<<2048, 256>>>(in, out, n4); }, 5), 2.0 * bytes);
    // in-L3 reference: a 78 MB block rewritten
    const size_t small4 = (size_t)T * OBS / 4;
    rep("grid-stride v4 stores over 78 MB (L3-resident)", timeit([&] { k_grid<false><<<2048, 256>>>(out, small4); }, 20), small4 * 16.0);
    rep("rows K=1 (78 MB, L3-resident)", timeit([&] { k_rows<false><<<nb, 64>>>(out, T, 1, 0); }, 20), small4 * 16.0);
    CHECK(hipFree(out));
    CHECK(hipFree(in));
    return 0;
}

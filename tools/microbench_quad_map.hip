// Store-only rates of the headline's output pattern under different wave -> table-block maps, with
// the quad kernel's shape (four output waves per workgroup, 256 workgroups) beside one output wave
// per workgroup (1024 workgroups): the per-step [K][T][297] int32 rows (76 KB per 64-row block) and,
// with MASK, the [K][T][45] int8 masks, K = 128 steps (10 GB per launch, the headline's).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_quad_map.hip -o tools/mbq_map.bin && ./tools/mbq_map.bin [T] [rounds]
// T = 32768 (round 6): config 4's per-GPU share, 4 players x 32 768 tables under the
// six-wave dealer's shape (two output waves per workgroup on adjacent blocks, one workgroup per CU,
// 256 workgroups) — the same [K][T][297] rows and [K][T][45] masks (the observation row of every player
// count is 297 int32).
// Maps (wave w of workgroup b, nb workgroups, xmap(b) = (b % 8) * (nb / 8) + b / 8, XCD-contiguous):
//   0 identity        block = b * W + w
//   1 quad (current)  block = W * xmap(b) + w     (a workgroup's W blocks adjacent)
//   2 quarters        block = w * nb + xmap(b)    (wave w of every workgroup in the w-th quarter)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int OBS = 297, ROWS = 64, RV4 = ROWS * OBS / 4, MV4 = ROWS * 45 / 16;

template <bool NT>
__device__ __forceinline__ void st(v4i *p, v4i v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NT, int MAP, int W, bool MASK>
__global__ __launch_bounds__(64 * W) void k_map(v4i *out, v4i *mask, int T, int K) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t xb = (b & 7u) * (nb >> 3) + (b >> 3);
    const size_t blkid = MAP == 0 ? (size_t)b * W + w : MAP == 1 ? (size_t)W * xb + w : (size_t)w * nb + xb;
    const size_t blk = (size_t)T * OBS / 4, mblk = (size_t)T * 45 / 16;
    for (int k = 0; k < K; ++k) {
        v4i *dst = out + (size_t)k * blk + blkid * RV4;
        int d = lane;
        for (; d + 64 * 4 < RV4; d += 64 * 5) {
#pragma unroll
            for (int u = 0; u < 5; ++u) st<NT>(dst + d + 64 * u, v4i{k, d, u, 0});
        }
        for (; d < RV4; d += 64) st<NT>(dst + d, v4i{k, d, 0, 0});
        if (MASK) {
            v4i *m = mask + (size_t)k * mblk + blkid * MV4;
            for (int c = lane; c < MV4; c += 64) st<NT>(m + c, v4i{k, c, 0, 0});
        }
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

int main(int argc, char **argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 65536, K = 128;
    const int rounds = argc > 2 ? atoi(argv[2]) : 2;
    const size_t bytes = (size_t)K * T * OBS * 4, mbytes = (size_t)K * T * 45;
    v4i *out, *mask;
    CHECK(hipMalloc(&out, bytes));
    CHECK(hipMalloc(&mask, mbytes));
    const int waves = T / ROWS;  // 1024
    auto rep = [&](const char *name, float ms, double nbytes) {
        printf("%-52s %9.1f us  %7.1f GB/s\n", name, ms * 1e3, nbytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    printf("# [K][T] row stores + masks, K=%d T=%d: %.2f GB per launch\n", K, T, (bytes + mbytes) / 1e9);
    const double nb2 = (double)bytes + mbytes;
    if (T != 65536) {  // the C4 share's shape: 2 output waves per workgroup (six-wave dealer), 256 workgroups
        for (int round = 0; round < rounds; ++round) {
            rep("W=2 map 1 dealer2 (adjacent blocks) NT", timeit([&] { k_map<true, 1, 2, true><<<waves / 2, 128>>>(out, mask, T, K); }, 4), nb2);
            rep("W=1 map 1 XCD-contiguous NT", timeit([&] { k_map<true, 1, 1, true><<<waves, 64>>>(out, mask, T, K); }, 4), nb2);
            rep("W=2 map 1 dealer2 (adjacent blocks) plain", timeit([&] { k_map<false, 1, 2, true><<<waves / 2, 128>>>(out, mask, T, K); }, 4), nb2);
            rep("W=2 map 0 identity NT", timeit([&] { k_map<true, 0, 2, true><<<waves / 2, 128>>>(out, mask, T, K); }, 4), nb2);
        }
        CHECK(hipFree(out));
        CHECK(hipFree(mask));
        return 0;
    }
    for (int round = 0; round < rounds; ++round) {
        rep("W=1 map 0 identity NT", timeit([&] { k_map<true, 0, 1, true><<<waves, 64>>>(out, mask, T, K); }, 4), nb2);
        rep("W=1 map 1 XCD-contiguous NT", timeit([&] { k_map<true, 1, 1, true><<<waves, 64>>>(out, mask, T, K); }, 4), nb2);
        rep("W=4 map 1 quad (adjacent blocks) NT", timeit([&] { k_map<true, 1, 4, true><<<waves / 4, 256>>>(out, mask, T, K); }, 4), nb2);
        rep("W=4 map 2 quarters NT", timeit([&] { k_map<true, 2, 4, true><<<waves / 4, 256>>>(out, mask, T, K); }, 4), nb2);
        rep("W=4 map 0 identity NT", timeit([&] { k_map<true, 0, 4, true><<<waves / 4, 256>>>(out, mask, T, K); }, 4), nb2);
        rep("W=1 map 1 XCD-contiguous plain", timeit([&] { k_map<false, 1, 1, true><<<waves, 64>>>(out, mask, T, K); }, 4), nb2);
        rep("W=4 map 1 quad (adjacent blocks) plain", timeit([&] { k_map<false, 1, 4, true><<<waves / 4, 256>>>(out, mask, T, K); }, 4), nb2);
        rep("W=4 map 2 quarters plain", timeit([&] { k_map<false, 2, 4, true><<<waves / 4, 256>>>(out, mask, T, K); }, 4), nb2);
    }
    CHECK(hipFree(out));
    CHECK(hipFree(mask));
    return 0;
}

// Store-pattern micro-benchmark shaped like k_rollout's steady state: 1024 one-wave workgroups,
// each owning 64 tables, K steps per launch; per step a dependent VALU chain (the rules work,
// `spin` iterations) and then the 64 x 297 int32 observation block expanded from LDS bytes with
// 16-byte stores.  What varies is WHERE a wave's 64 rows live:
//   block   wave w owns tables [64w, 64w+64): one contiguous 76 KB region per wave (k_rollout now)
//   group4  wave w owns 16 groups of 4 tables, group g = tables 4(w + W*g) .. +3: at a given step
//           position all waves write neighbouring 4.6 KB pieces (a grid-stride-like write front)
//   group16 the same with groups of 16 tables (4 groups per wave)
// and whether the stores are plain or nontemporal.  Standalone:
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_store5.hip -o /tmp/mbs5 && /tmp/mbs5
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) {                                                        \
            printf("%s: %s\n", #x, hipGetErrorString(e));                             \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

constexpr int OBS = 297, ROWS = 64, WORDS = ROWS * OBS / 4;  // 4752 LDS dwords = 16-B stores per wave
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i expand4(uint32_t w) {
    v4i v = {(int)(w & 0xFFu), (int)((w >> 8) & 0xFFu), (int)((w >> 16) & 0xFFu), (int)(w >> 24)};
    return v;
}

// GROUP = tables per contiguous group (64 = the whole wave block)
template <int GROUP, bool NT, int RW = 64, bool STORE = true>
__global__ __launch_bounds__(64) void k_steps(v4i *out, int K, int spin, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[RW * OBS];
    const int lane = threadIdx.x, w = blockIdx.x, W = gridDim.x;
    constexpr int GW = (GROUP < RW ? GROUP : RW) * OBS / 4;  // 16-B stores per group
    constexpr int WORDS = RW * OBS / 4;
    uint32_t acc = lane * 2654435761u + w;
    for (int k = 0; k < K; ++k) {
        // "rules": a dependent integer chain, then the row bytes into LDS
        for (int i = 0; i < spin; ++i) acc = acc * 1664525u + 1013904223u;
        if (lane < RW)
            for (int i = 0; i < OBS; ++i) rows[lane * OBS + i] = (uint8_t)(acc + i);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        const uint32_t *src = reinterpret_cast<const uint32_t *>(rows);
        constexpr int U = 5;
        for (int d0 = 0; STORE && d0 < WORDS; d0 += 64 * U) {
            uint32_t x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int d = d0 + 64 * u + lane;
                x[u] = d < WORDS ? src[d] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int d = d0 + 64 * u + lane;
                if (d < WORDS) {
                    const int g = d / GW, e = d - g * GW;
                    const size_t idx = (size_t)(w + (size_t)W * g) * GW + e;
                    if (NT) __builtin_nontemporal_store(expand4(x[u]), out + idx);
                    else out[idx] = expand4(x[u]);
                }
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// Software-pipelined variant: two LDS row buffers; step k's compute is cut into NSEG segments and
// after each segment 1/NSEG of step k-1's block stores are issued from the other buffer, so the
// wave never issues its whole block in one burst (which stalls it for the drain) and its store
// stream keeps flowing while it computes.
template <int NSEG>
__global__ __launch_bounds__(64) void k_pipe(v4i *out, int K, int spin, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[2][ROWS * OBS];
    const int lane = threadIdx.x, w = blockIdx.x;
    uint32_t acc = lane * 2654435761u + w;
    constexpr int PER = (WORDS + NSEG * 64 - 1) / (NSEG * 64) * 64;  // LDS words per segment (multiple of 64)
    v4i *dst = out + (size_t)w * WORDS;
    for (int k = 0; k <= K; ++k) {
        const uint32_t *prev = reinterpret_cast<const uint32_t *>(rows[(k + 1) & 1]);
        for (int sgm = 0; sgm < NSEG; ++sgm) {
            if (k < K)
                for (int i = 0; i < spin / NSEG; ++i) acc = acc * 1664525u + 1013904223u;
            if (k > 0) {
                const int d0 = sgm * PER;
#pragma unroll 4
                for (int d = d0 + lane; d < d0 + PER && d < WORDS; d += 64) dst[d] = expand4(prev[d]);
            }
        }
        if (k < K)
            for (int i = 0; i < OBS; ++i) rows[k & 1][lane * OBS + i] = (uint8_t)(acc + i);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const int n = 65536, waves = n / ROWS, K = 64;
    const size_t bytes = (size_t)n * OBS * 4;
    v4i *out;
    uint32_t *sink;
    CHECK(hipMalloc(&out, bytes + 4096));
    CHECK(hipMalloc(&sink, 64));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char *name, auto kern, int spin, int nw = waves) {
        kern<<<nw, 64>>>(out, K, spin, sink);
        hipDeviceSynchronize();
        hipEventRecord(a);
        const int reps = 5;
        for (int r = 0; r < reps; ++r) kern<<<nw, 64>>>(out, K, spin, sink);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us_step = 1000.0 * ms / reps / K;
        printf("%-10s spin %5d  %7.2f us/step  %7.1f GB/s\n", name, spin, us_step, bytes / us_step / 1e3);
    };
    for (int spin : {0, 200, 400, 600, 1200}) {
        run("compute", k_steps<64, false, 64, false>, spin);
        run("block", k_steps<64, false>, spin);
        run("block32", k_steps<64, false, 32>, spin, 2 * waves);  // 32 tables per wave, 2 waves per SIMD
        run("pipe4", k_pipe<4>, spin);
    }
    return 0;
}

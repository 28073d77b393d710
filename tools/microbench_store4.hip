// Store address pattern vs HBM write rate.  Same per-wave work as the engine's obs block (64 rows
// x 297 int32 from LDS bytes, 16-byte stores, 5 LDS reads per 5 stores), but the wave's 64 rows
// are 64/G groups of G consecutive rows spread over the batch (group g at row g*(n*G/64) + w*G):
// G = 64 is the engine's contiguous ownership (1024 concurrent 76 KB streams); small G makes the
// concurrently written addresses of all waves closer together (a moving front).
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_store4.hip -o tools/microbench_store4.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int OBS = 297;
typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4i expand4(uint32_t w) {
    v4i v = {(int)(w & 0xFFu), (int)((w >> 8) & 0xFFu), (int)((w >> 16) & 0xFFu), (int)(w >> 24)};
    return v;
}

template <int G, bool NT>
__global__ __launch_bounds__(64) void k_groups(int32_t *out, int n) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[64 * OBS + 16];
    const int lane = threadIdx.x, w = blockIdx.x;
    rows[lane] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows);
    constexpr int NG = 64 / G, PER = G * OBS / 4;  // int4 chunks per group
    const int span = n / NG;                        // rows per group region
#pragma unroll 1
    for (int g = 0; g < NG; ++g) {
        v4i *dst = reinterpret_cast<v4i *>(out + ((size_t)g * span + (size_t)w * G) * OBS);
        const uint32_t *s = src + g * PER;
        int d = lane;
        for (; d + 64 * 4 < PER; d += 64 * 5) {
            uint32_t x[5];
#pragma unroll
            for (int u = 0; u < 5; ++u) x[u] = s[d + 64 * u];
#pragma unroll
            for (int u = 0; u < 5; ++u) {
                if (NT) __builtin_nontemporal_store(expand4(x[u]), &dst[d + 64 * u]);
                else dst[d + 64 * u] = expand4(x[u]);
            }
        }
        for (; d < PER; d += 64) dst[d] = expand4(s[d]);
    }
}

template <typename F>
float timeit(F launch, int reps = 30) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; ++r) launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return 1000.f * ms / reps;
}

int main() {
    const int n = 65536;
    const size_t bytes = (size_t)n * OBS * 4;
    int32_t *out;
    if (hipMalloc(&out, bytes + 4096) != hipSuccess) return 1;
    auto rep = [&](const char *name, float us) { printf("%-22s %7.2f us  %6.0f GB/s\n", name, us, bytes / 1e3 / us); };
    rep("G=64 (engine)", timeit([&] { k_groups<64, false><<<n / 64, 64>>>(out, n); }));
    rep("G=32", timeit([&] { k_groups<32, false><<<n / 64, 64>>>(out, n); }));
    rep("G=16", timeit([&] { k_groups<16, false><<<n / 64, 64>>>(out, n); }));
    rep("G=8", timeit([&] { k_groups<8, false><<<n / 64, 64>>>(out, n); }));
    rep("G=4", timeit([&] { k_groups<4, false><<<n / 64, 64>>>(out, n); }));
    rep("G=64 nt", timeit([&] { k_groups<64, true><<<n / 64, 64>>>(out, n); }));
    rep("G=16 nt", timeit([&] { k_groups<16, true><<<n / 64, 64>>>(out, n); }));
    return 0;
}

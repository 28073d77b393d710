// Store-path micro-benchmark for the step kernel's output shape: 65536 rows x 297 int32
// (obs) staged as bytes in LDS per 64-row wave, expanded to int32 and stored.  Variants show
// the floor and what each structural choice costs.  Standalone: hipcc -O3 --offload-arch=gfx950
//   tools/microbench_store.hip -o /tmp/mbs && /tmp/mbs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
constexpr int OBS = 297, ROWS = 64;

// baseline: pure streaming int4 stores of the same byte count (grid-stride)
__global__ void k_stream(int4 *out, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        out[i] = make_int4((int)i, 1, 2, 3);
}

// current engine shape: 1 wave per block, LDS bytes -> int4, one LDS read + wait per store
template <int UNROLL>
__global__ __launch_bounds__(64) void k_lds(int32_t *out, int n) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[ROWS * OBS];
    const int lane = threadIdx.x, t0 = blockIdx.x * ROWS;
    for (int i = 0; i < OBS; ++i) rows[lane * OBS + i] = (uint8_t)(i + lane);
    __syncthreads();
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows);
    int32_t *dst = out + (size_t)t0 * OBS;
    const int full = ROWS * OBS / 4;  // 4752
    if (UNROLL == 1) {
        for (int d = lane; d < full; d += 64) {
            const uint32_t w = src[d];
            *reinterpret_cast<int4 *>(dst + 4 * d) = make_int4(w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24);
        }
    } else {
        int d = lane;
        for (; d + 64 * (UNROLL - 1) < full; d += 64 * UNROLL) {
            uint32_t w[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) w[u] = src[d + 64 * u];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
                *reinterpret_cast<int4 *>(dst + 4 * (d + 64 * u)) =
                    make_int4(w[u] & 0xFF, (w[u] >> 8) & 0xFF, (w[u] >> 16) & 0xFF, w[u] >> 24);
        }
        for (; d < full; d += 64) {
            const uint32_t w = src[d];
            *reinterpret_cast<int4 *>(dst + 4 * d) = make_int4(w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24);
        }
    }
}

// wider: each lane expands 16 bytes (ds_read_b128) into 4 int4 stores; per instruction the
// wave still writes 1 KB contiguous (lane stride 16 B within each of the 4 store passes)
__global__ __launch_bounds__(64) void k_lds128(int32_t *out, int n) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[ROWS * OBS];
    const int lane = threadIdx.x, t0 = blockIdx.x * ROWS;
    for (int i = 0; i < OBS; ++i) rows[lane * OBS + i] = (uint8_t)(i + lane);
    __syncthreads();
    const uint4 *src = reinterpret_cast<const uint4 *>(rows);
    int32_t *dst = out + (size_t)t0 * OBS;
    const int full16 = ROWS * OBS / 16;  // 1188 x 16 B
    for (int q = lane; q < full16; q += 64) {
        const uint4 v = src[q];
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
            *reinterpret_cast<int4 *>(dst + 16 * q + 4 * u) =
                make_int4(w4[u] & 0xFF, (w4[u] >> 8) & 0xFF, (w4[u] >> 16) & 0xFF, w4[u] >> 24);
    }
}

// same as k_lds<4> but 4 waves per block (256 threads), each wave its own 64 rows
__global__ __launch_bounds__(256) void k_lds_wg4(int32_t *out, int n) {
    __shared__ __attribute__((aligned(16))) uint8_t rows_all[4 * ROWS * OBS];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t *rows = rows_all + w * ROWS * OBS;
    const int t0 = (blockIdx.x * 4 + w) * ROWS;
    for (int i = 0; i < OBS; ++i) rows[lane * OBS + i] = (uint8_t)(i + lane);
    __syncthreads();
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows);
    int32_t *dst = out + (size_t)t0 * OBS;
    const int full = ROWS * OBS / 4;
    int d = lane;
    for (; d + 64 * 3 < full; d += 256) {
        uint32_t x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = src[d + 64 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            *reinterpret_cast<int4 *>(dst + 4 * (d + 64 * u)) = make_int4(x[u] & 0xFF, (x[u] >> 8) & 0xFF, (x[u] >> 16) & 0xFF, x[u] >> 24);
    }
    for (; d < full; d += 64) {
        const uint32_t x = src[d];
        *reinterpret_cast<int4 *>(dst + 4 * d) = make_int4(x & 0xFF, (x >> 8) & 0xFF, (x >> 16) & 0xFF, x >> 24);
    }
}

// no LDS: every lane writes its own row directly, dword by dword (uncoalesced per instruction)
__global__ __launch_bounds__(64) void k_direct(int32_t *out, int n) {
    const int t = blockIdx.x * 64 + threadIdx.x;
    int32_t *row = out + (size_t)t * OBS;
    for (int i = 0; i < OBS; ++i) row[i] = i + t;
}

template <typename F>
float timeit(F launch, int reps) {
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

int main() {
    const int n = 65536;
    const size_t bytes = (size_t)n * OBS * 4;
    int32_t *out;
    CHECK(hipMalloc(&out, bytes + 4096));
    const int reps = 50;
    const double mb = bytes / 1e6;
    auto rep = [&](const char *name, float us) { printf("%-28s %8.2f us  %7.1f GB/s\n", name, us, mb * 1e3 / us); };
    rep("stream int4 grid 1024x256", timeit([&] { k_stream<<<1024, 256>>>((int4 *)out, bytes / 16); }, reps));
    rep("stream int4 grid 4096x256", timeit([&] { k_stream<<<4096, 256>>>((int4 *)out, bytes / 16); }, reps));
    rep("stream int4 grid 1024x64", timeit([&] { k_stream<<<1024, 64>>>((int4 *)out, bytes / 16); }, reps));
    rep("lds->int4 (engine now)", timeit([&] { k_lds<1><<<n / 64, 64>>>(out, n); }, reps));
    rep("lds->int4 unroll 5", timeit([&] { k_lds<5><<<n / 64, 64>>>(out, n); }, reps));
    rep("lds->int4 unroll 15", timeit([&] { k_lds<15><<<n / 64, 64>>>(out, n); }, reps));
    rep("lds b128 -> 4 x int4", timeit([&] { k_lds128<<<n / 64, 64>>>(out, n); }, reps));
    rep("lds unroll 4, 4 waves/WG", timeit([&] { k_lds_wg4<<<n / 256, 256>>>(out, n); }, reps));
    rep("direct per-lane rows", timeit([&] { k_direct<<<n / 64, 64>>>(out, n); }, reps));
    CHECK(hipFree(out));
    return 0;
}

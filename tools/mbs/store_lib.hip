// The microbench_store3 kernel (no loads, no LDS fill) as a C-ABI library, so the same store
// loop can run from Python on torch-allocated and on hipMalloc'd buffers (tools/mbs/buffers.py).
#include <hip/hip_runtime.h>
#include <stdint.h>
constexpr int OBS = 297, ROWS = 64;

__global__ __launch_bounds__(64) void k_store(int32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t rows[40064];
    const int lane = threadIdx.x, t0 = blockIdx.x * ROWS;
    rows[lane] = (uint8_t)lane;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows);
    int32_t *dst = out + (size_t)t0 * OBS;
    const int full = ROWS * OBS / 4;
    int d = lane;
    for (; d + 64 * 4 < full; d += 64 * 5) {
        uint32_t w[5];
#pragma unroll
        for (int u = 0; u < 5; ++u) w[u] = src[d + 64 * u];
#pragma unroll
        for (int u = 0; u < 5; ++u)
            *reinterpret_cast<int4 *>(dst + 4 * (d + 64 * u)) =
                make_int4(w[u] & 0xFF, (w[u] >> 8) & 0xFF, (w[u] >> 16) & 0xFF, w[u] >> 24);
    }
    for (; d < full; d += 64) {
        const uint32_t w = src[d];
        *reinterpret_cast<int4 *>(dst + 4 * d) = make_int4(w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24);
    }
}

extern "C" int mbs_store(void *out, int n, void *stream) {
    hipLaunchKernelGGL(k_store, dim3(n / 64), dim3(64), 0, (hipStream_t)stream, (int32_t *)out);
    return (int)hipGetLastError();
}
extern "C" void *mbs_malloc(size_t bytes) {
    void *p = nullptr;
    return hipMalloc(&p, bytes) == hipSuccess ? p : nullptr;
}

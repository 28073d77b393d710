// Does the rollout store's write pattern alone (rows [K][T][297] int32, one wave per 64 tables,
// 1024 waves, 5 GB) finish later on some XCCs?  Each wave stamps its start and end (s_memrealtime,
// 100 MHz); we print the mean end by blockIdx % 8 (= XCC) and by blockIdx / 128, as
// tools/wsstamps.py does for k_rollout_ws.  The swapped variants write each workgroup's rows into
// its neighbour's block (b ^ 1): if the slow XCCs follow the workgroup, not the addresses, the
// asymmetry is in the XCC's write path.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench_store_xcc.hip -o tools/mbs/mb_xcc && tools/mbs/mb_xcc
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef int v4i __attribute__((ext_vector_type(4)));
constexpr int OBS = 297, ROWS = 64;
constexpr int ROW_V4 = ROWS * OBS / 4;

template <bool NT>
__global__ __launch_bounds__(128) void k_rows(v4i *out, int T, int K, unsigned long long *st, int swap) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x < 64) {  // second wave idle, as the rules wave's slot (same placement as k_rollout_ws)
        const size_t blk = (size_t)T * OBS / 4;
        for (int k = 0; k < K; ++k) {
            v4i *dst = out + (size_t)k * blk + (size_t)(blockIdx.x ^ swap) * ROW_V4;
            int d = lane;
            for (; d + 64 * 4 < ROW_V4; d += 64 * 5) {
#pragma unroll
                for (int u = 0; u < 5; ++u) {
                    if (NT) __builtin_nontemporal_store(v4i{k, d, u, 0}, dst + d + 64 * u);
                    else dst[d + 64 * u] = v4i{k, d, u, 0};
                }
            }
            for (; d < ROW_V4; d += 64) {
                if (NT) __builtin_nontemporal_store(v4i{k, d, 0, 0}, dst + d);
                else dst[d] = v4i{k, d, 0, 0};
            }
        }
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            st[2 * blockIdx.x] = t0;
            st[2 * blockIdx.x + 1] = t1;
        }
    }
}

int main() {
    const int T = 65536, K = 64, nb = T / ROWS;
    const size_t bytes = (size_t)K * T * OBS * 4;
    v4i *out;
    unsigned long long *st, h[2 * 1024];
    CHECK(hipMalloc(&out, bytes));
    CHECK(hipMalloc(&st, sizeof(h)));
    for (int v = 0; v < 4; ++v) {
        const int nt = v & 1, swap = v >> 1;
        double endx[8] = {0}, endq[8] = {0};
        int cx[8] = {0}, cq[8] = {0};
        double mx = 0, sum = 0;
        const int reps = 5;
        for (int rep = 0; rep < reps + 1; ++rep) {
            if (nt) k_rows<true><<<nb, 128>>>(out, T, K, st, swap);
            else k_rows<false><<<nb, 128>>>(out, T, K, st, swap);
            CHECK(hipDeviceSynchronize());
            if (rep == 0) continue;
            CHECK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull;
            for (int b = 0; b < nb; ++b) t0 = h[2 * b] < t0 ? h[2 * b] : t0;
            double m = 0;
            for (int b = 0; b < nb; ++b) {
                const double e = (h[2 * b + 1] - t0) * 0.01;  // us
                endx[b % 8] += e, cx[b % 8]++;
                endq[b / 128] += e, cq[b / 128]++;
                sum += e;
                m = e > m ? e : m;
            }
            mx += m;
        }
        printf("%s stores%s: mean end %.1f us, mean max %.1f us\n  mean end by blockIdx %% 8:", nt ? "NT" : "plain",
               swap ? ", workgroup b writes block b^1" : "",
               sum / (reps * nb), mx / reps);
        for (int x = 0; x < 8; ++x) printf(" %.0f", endx[x] / cx[x]);
        printf("\n  mean end by blockIdx / 128:");
        for (int x = 0; x < 8; ++x) printf(" %.0f", endq[x] / cq[x]);
        printf("\n");
    }
    CHECK(hipFree(out));
    CHECK(hipFree(st));
    return 0;
}

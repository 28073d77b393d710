// Where does a pool deal's time go?  Per-lane CPython MT19937 init_by_array (serial chain),
// the deal's output stream, and the full Fisher-Yates deal with its LDS scratch, each on a
// full grid (1024 waves, one per SIMD) and on the refill's typical grid (273 waves).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 [-DSPL_SCRATCH_STRIDE=112] tools/microbench_deal.hip -o ...
#include "../splendor-gym_amd/csrc/spl_engine.hip"

using namespace spl;

__global__ __launch_bounds__(64) void k_init_only(uint32_t *out, uint32_t seed0) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    MTStream ms;
    ms.init(seed0 + t * 2654435761u);
    out[t] = ms.s1 ^ ms.r_a0 ^ ms.r_c0;
}

template <int NOUT>
__global__ __launch_bounds__(64) void k_init_outputs(uint32_t *out, uint32_t seed0) {
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    MTStream ms;
    ms.init(seed0 + t * 2654435761u);
    uint32_t x = 0;
    for (int j = 0; j < NOUT; ++j) x ^= ms.next(j);
    out[t] = x;
}

__global__ __launch_bounds__(64) void k_deal(uint8_t *recs, uint32_t *out, uint32_t seed0) {
    __shared__ uint8_t scr_all[64 * kScratchStride] __attribute__((aligned(16)));
    const uint32_t t = blockIdx.x * 64 + threadIdx.x;
    Deal d;
    const uint32_t f = deal_into(seed0 + t * 2654435761u, 2, recs + (size_t)t * 128, &scr_all[threadIdx.x * kScratchStride], d);
    out[t] = d.board[0] ^ d.nob0 ^ f;
}

template <typename F>
float timeit(F launch, int reps = 10) {
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
    uint32_t *out;
    uint8_t *recs;
    if (hipMalloc(&out, 65536 * 4) != hipSuccess || hipMalloc(&recs, 65536 * 128) != hipSuccess) return 1;
    for (int waves : {1024, 273, 64}) {
        printf("waves %4d: init %7.1f us  init+150 out %7.1f us  init+300 out %7.1f us  deal %7.1f us\n", waves,
               timeit([&] { k_init_only<<<waves, 64>>>(out, 12345u); }),
               timeit([&] { k_init_outputs<150><<<waves, 64>>>(out, 12345u); }),
               timeit([&] { k_init_outputs<300><<<waves, 64>>>(out, 12345u); }),
               timeit([&] { k_deal<<<waves, 64>>>(recs, out, 12345u); }));
    }
    return 0;
}

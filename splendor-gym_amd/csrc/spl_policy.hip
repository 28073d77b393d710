// spl_policy.hip — fused ActorCritic forward for batched self-play on MI355X (gfx950).
//
// Reference network (ppo_splendor.py:40-59): actor and critic are separate
// Linear(297,256)-Tanh-Linear(256,256)-Tanh-Linear(256,{45|1}) MLPs; get_action_and_value
// samples masked_categorical(actor(x), mask) (ppo_splendor.py:27-37) and returns log_prob,
// entropy and critic(x); opponents play the greedy masked argmax of a frozen actor
// (training_utils.py:263-276).  Here one launch evaluates that for every table:
//
//   * a workgroup = 8 waves = 256 tables (two waves per SIMD), one wave = 32 tables = the 32
//     columns of every v_mfma_f32_32x32x16_bf16 tile.  Activations are computed TRANSPOSED (hidden
//     unit on the accumulator row, table on the lane), so each layer's accumulator registers are
//     directly the next layer's B operand: no LDS round trip between layers (the k order inside a
//     16-step is permuted; the packed weights carry the matching column order).
//   * weights are packed once (k_pack) into 20 KB "chunks" — one 32-row output tile of one layer,
//     [k-step][lane][8 bf16] in fragment order plus the tile's bias in accumulator order — and
//     streamed through a 6-slot LDS ring with global_load_lds (5 chunks in flight), shared by the
//     workgroup's 8 waves; a 65 536-table batch is one workgroup per CU.
//   * observations (int32) load straight into registers as the layer-1 B fragments (bf16; every
//     obs value is a small integer, exact in bf16) and stay there through both networks' layer 1.
//   * the critic's one-unit output layer runs on VALU in fp32 as its layer-2 tiles come out;
//     tanh (v_exp + v_rcp) runs inside the next tile's MFMA stream; masking, log-softmax, entropy
//     and the Philox-driven inverse-CDF sample are fused after the last tile on register-resident
//     logits; the sampled action differs from torch's multinomial stream by design (same
//     distribution), logits match the fp32 module to bf16 accuracy.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/splendor_amd.h"
#include "../../include/splendor_policy.h"
#include "spl_rng.h"

int spl_fail(int code, const std::string &msg);  // spl_engine.hip: sets spl_last_error()

namespace splp {

using spl::philox4x32;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kObs = 297, kAct = 45, kHid = 256;
constexpr int kK1 = 19;  // layer-1 k-steps of 16: 297 inputs padded to 304
constexpr int kK2 = 16;  // layers 2 and 3: 256 inputs
constexpr int kChunk = 20480, kBiasOff = 19 * 1024;
constexpr int kActorChunks = 18, kCriticChunks = 17, kAllChunks = 35;
// Ablation switches for profiling builds only (tools/ablate_policy.sh); the product build defines none.
#ifndef SPL_ACT_ABL
#define SPL_ACT_ABL 0
#endif
constexpr int ABL_MFMA = 1, ABL_EPI = 2, ABL_XLOAD = 4, ABL_RING = 8;
#ifndef SPL_ACT_RELOAD_X
#define SPL_ACT_RELOAD_X 0  // 1: reload the observation after the critic (fewer registers live)
#endif

constexpr int kWaves = 8, kRowsPerWave = 32, kRowsPerBlock = kWaves * kRowsPerWave;  // 256 tables
constexpr int kSlots = 6;                         // weight ring: 5 chunks in flight
constexpr int kMaskWave = kRowsPerWave * kAct;    // 1 440 B
constexpr int kLogitRow = 65;                     // floats per staged logit row
constexpr int kLdsMask = kSlots * kChunk;         // 122 880 B of ring
constexpr int kLds = kLdsMask + kWaves * kMaskWave;  // 134 400 B
static_assert(kWaves * kRowsPerWave * kLogitRow * 4 <= kLdsMask, "logits reuse the weight ring");
static_assert(kLds <= 160 * 1024, "LDS");
// fp32 critic output layer after the chunks of a full image: w3 [256], b3, zero padding
constexpr int kCriticTail = 272 * 4;

// chunk order of an image: with a critic [critic L1 x8][critic L2 x8][critic L3 x1], then
// [actor L1 x8][actor L2 x8][actor L3 x2] — the order a forward pass consumes them; the actor part
// of a full image (its last 18 chunks) is an actor-only image.

// ------------------------------------------------------------------------------------------
// packing
// ------------------------------------------------------------------------------------------
struct PackNet {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    int out;
};

__device__ __forceinline__ uint16_t bf16_bits(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }

// one block per physical chunk
__global__ __launch_bounds__(256) void k_pack(PackNet actor, PackNet critic, int with_critic, uint8_t *dst) {
    const int ch = blockIdx.x;
    const int net = with_critic && ch < kCriticChunks ? 1 : 0;  // 0 actor, 1 critic
    const int local = ch - (with_critic && !net ? kCriticChunks : 0);
    const int layer = local < 8 ? 1 : local < 16 ? 2 : 3;
    const int tile = local - (layer - 1) * 8;
    const PackNet &P = net ? critic : actor;
    const float *W = layer == 1 ? P.w1 : layer == 2 ? P.w2 : P.w3;
    const float *B = layer == 1 ? P.b1 : layer == 2 ? P.b2 : P.b3;
    const int in = layer == 1 ? kObs : kHid, rows = layer == 3 ? P.out : kHid;
    const int ks = layer == 1 ? kK1 : kK2;
    uint8_t *out = dst + (size_t)ch * kChunk;
    for (int v = threadIdx.x; v < kChunk / 16; v += blockDim.x) {
        const int s = v >> 6, lane = v & 63, i = lane & 31, h = lane >> 5, row = 32 * tile + i;
        if (s == 19 && lane < 8) continue;  // bias, below
        uint16_t e[8];
        for (int j = 0; j < 8; ++j) {
            float x = 0.f;
            if (s < ks) {
                // layer 1: B is the observation, natural k = 16s + 8h + j.  Layers 2-3: B is the
                // previous tile's accumulator, whose element j of lane half h is input unit
                // 32*(s/2) + 16*(s%2) + 8*(j/4) + 4h + j%4.
                const int k = layer == 1 ? 16 * s + 8 * h + j
                                         : 32 * (s >> 1) + 16 * (s & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
                if (row < rows && k < in) x = W[(size_t)row * in + k];
            }
            e[j] = bf16_bits(x);
        }
        u32x4 w = {e[0] | (uint32_t)e[1] << 16, e[2] | (uint32_t)e[3] << 16, e[4] | (uint32_t)e[5] << 16,
                   e[6] | (uint32_t)e[7] << 16};
        *reinterpret_cast<u32x4 *>(out + (size_t)v * 16) = w;
    }
    if (net == 1 && layer == 3) {  // the critic's output layer also as fp32 (evaluated on VALU)
        float *tail = reinterpret_cast<float *>(dst + (size_t)kAllChunks * kChunk);
        for (int k = threadIdx.x; k < 272; k += blockDim.x) tail[k] = k < kHid ? W[k] : k == kHid ? B[0] : 0.f;
    }
    if (threadIdx.x < 32) {  // bias in accumulator order: [lane half][reg] -> row (reg&3)+8(reg>>2)+4h
        const int h = threadIdx.x >> 4, reg = threadIdx.x & 15;
        const int row = 32 * tile + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        reinterpret_cast<float *>(out + kBiasOff)[threadIdx.x] = row < rows ? B[row] : 0.f;
    }
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
struct ActArgs {
    const int32_t *obs;
    const int8_t *mask;
    int32_t *action;
    float *logprob, *entropy, *value, *logits;
    const float *critic_out;  // fp32 critic output layer (kCriticTail) of a full image
    uint64_t seed, ply;
    const uint64_t *ply_base;
    int64_t table0;
    int n;
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}

typedef __attribute__((address_space(3))) void lds_void;
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));  // dword-aligned 16-B load

// this wave's 1-KB blocks of one chunk, global -> LDS: wave w moves blocks w, w+8, w+16 (< 20), so
// waves 0-3 issue 3 loads per chunk and waves 4-7 issue 2
constexpr int kChunkBlocks = kChunk / 1024;  // 20
__device__ __forceinline__ void issue_chunk(const uint8_t *W, int chunk, uint8_t *slot, int wave, int lane) {
    if constexpr (SPL_ACT_ABL & ABL_RING) return;
    const uint8_t *src = W + (size_t)chunk * kChunk + lane * 16;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const int blk = wave + kWaves * i;
        if (blk < kChunkBlocks)
            __builtin_amdgcn_global_load_lds(src + blk * 1024, (lds_void *)(slot + blk * 1024), 16, 0, 0);
    }
}

// tanh(x) = 1 - 2 / (e^2x + 1) as v_exp_f32 + v_rcp_f32 (about 1 ulp each; +-inf saturate to +-1):
// __expf / __fdividef compiled to the full-precision division sequence (v_div_scale / fmas /
// fixup, ~14 instructions per value), which made the tanh epilogues cost more than the MFMAs
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.88539008177792681f);  // 2 / ln 2
    return __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(e + 1.f), 1.f);
}

__device__ __forceinline__ bf16x8 pack8(float a0, float a1, float a2, float a3, float a4, float a5, float a6,
                                        float a7) {
    const bf16x2 p0 = {(__bf16)a0, (__bf16)a1}, p1 = {(__bf16)a2, (__bf16)a3}, p2 = {(__bf16)a4, (__bf16)a5},
                 p3 = {(__bf16)a6, (__bf16)a7};
    const u32x4 w = {__builtin_bit_cast(uint32_t, p0), __builtin_bit_cast(uint32_t, p1),
                     __builtin_bit_cast(uint32_t, p2), __builtin_bit_cast(uint32_t, p3)};
    return __builtin_bit_cast(bf16x8, w);
}

// tanh of one accumulator tile -> the two B fragments (k-steps 2t, 2t+1) of the next layer
__device__ __forceinline__ void tanh_pack(const f32x16 &a, bf16x8 &lo, bf16x8 &hi) {
    float t[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) t[r] = tanh_fast(a[r]);
    lo = pack8(t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7]);
    hi = pack8(t[8], t[9], t[10], t[11], t[12], t[13], t[14], t[15]);
}

// one 32-row output tile: bias + sum over KS k-steps, B fragments in registers (the observation
// for layer 1, the previous layer's tanh for layers 2-3); weight fragments from the LDS ring slot,
// read one group of 4 k-steps ahead of the MFMAs that use them (the scheduling barriers keep the
// compiler from hoisting every read of the tile, and its registers, to the top)
template <int KS, int NB>
__device__ __forceinline__ f32x16 tile_mma(const uint8_t *slot, const bf16x8 (&B)[NB], int lane) {
    static_assert(KS <= NB, "B fragments");
    constexpr int G = 4, NG = (KS + G - 1) / G;
    const float *bias = reinterpret_cast<const float *>(slot + kBiasOff) + (lane >> 5) * 16;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = bias[r];
    const bf16x8 *A = reinterpret_cast<const bf16x8 *>(slot) + lane;
    bf16x8 af[2][G];
#pragma unroll
    for (int i = 0; i < G; ++i) af[0][i] = A[i * 64];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (g + 1 < NG) {
#pragma unroll
            for (int i = 0; i < G; ++i) {
                const int s = (g + 1) * G + i;
                if (s < KS) af[(g + 1) & 1][i] = A[s * 64];
            }
        }
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const int s = g * G + i;
            if (s < KS) {
                if constexpr (SPL_ACT_ABL & ABL_MFMA) acc[i] += (float)af[g & 1][i][0] + (float)B[s][1];
                else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[g & 1][i], B[s], acc, 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

// tile_mma that also evaluates tanh of the PREVIOUS tile's accumulator `pend` into tp[16],
// four values per group of four MFMAs: the transcendental work (v_exp + v_rcp per value) issues in
// the MFMA gaps instead of as a separate VALU phase after every tile
template <int KS, int NB>
__device__ __forceinline__ f32x16 tile_mma_tanh(const uint8_t *slot, const bf16x8 (&B)[NB], int lane,
                                                const f32x16 &pend, float (&tp)[16]) {
    static_assert(KS <= NB, "B fragments");
    constexpr int G = 4, NG = (KS + G - 1) / G;
    static_assert(NG >= 4, "16 tanh values over at least four groups");
    const float *bias = reinterpret_cast<const float *>(slot + kBiasOff) + (lane >> 5) * 16;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = bias[r];
    const bf16x8 *A = reinterpret_cast<const bf16x8 *>(slot) + lane;
    bf16x8 af[2][G];
#pragma unroll
    for (int i = 0; i < G; ++i) af[0][i] = A[i * 64];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (g + 1 < NG) {
#pragma unroll
            for (int i = 0; i < G; ++i) {
                const int s = (g + 1) * G + i;
                if (s < KS) af[(g + 1) & 1][i] = A[s * 64];
            }
        }
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const int s = g * G + i;
            if (s < KS) {
                if constexpr (SPL_ACT_ABL & ABL_MFMA) acc[i] += (float)af[g & 1][i][0] + (float)B[s][1];
                else acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[g & 1][i], B[s], acc, 0, 0, 0);
            }
            if (g < 4) tp[4 * g + i] = tanh_fast(pend[4 * g + i]);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

// one layer of 8 tiles whose tanh feeds the next layer as bf16 B fragments H[16]; each tile's tanh
// runs inside the next tile's MFMAs, the last one after the loop
template <int KS, int NB, typename Enter>
__device__ __forceinline__ void layer_tanh(Enter &enter, const bf16x8 (&B)[NB], bf16x8 (&H)[16], int lane) {
    f32x16 pend = tile_mma<KS>(enter(), B, lane);
#pragma unroll
    for (int t = 1; t < 8; ++t) {
        float tp[16];
        const f32x16 acc = tile_mma_tanh<KS>(enter(), B, lane, pend, tp);
        H[2 * t - 2] = pack8(tp[0], tp[1], tp[2], tp[3], tp[4], tp[5], tp[6], tp[7]);
        H[2 * t - 1] = pack8(tp[8], tp[9], tp[10], tp[11], tp[12], tp[13], tp[14], tp[15]);
        pend = acc;
    }
    tanh_pack(pend, H[14], H[15]);
}

// Workgroup = 8 waves = 256 tables (two waves per SIMD), one wave = 32 tables = the 32 columns of
// every v_mfma_f32_32x32x16_bf16 tile.  Activations are TRANSPOSED (hidden unit on the
// accumulator row, table on the lane), so each layer's accumulators are directly the next layer's
// B operand, and the observation's B fragments are loaded straight from HBM into registers
// (8 int32 of one row per lane and k-step -> bf16; every obs value is a small integer, exact in
// bf16).  Weights stream once per workgroup through a 6-slot LDS ring (20-KB chunks = one 32-row
// tile of a layer, global_load_lds, 5 in flight) shared by the 8 waves; a 65 536-table grid is
// one workgroup per CU, so each CU streams the 0.7-MB image once per launch.  The critic's output
// layer (one unit) runs on VALU in fp32 as its layer-2 tiles come out, so neither its layer-2
// activations nor an output tile are ever materialised.
template <bool kCritic, bool kSample>
__global__ __launch_bounds__(512) void k_act(const uint8_t *__restrict__ W, ActArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    constexpr int kTotal = kCritic ? kAllChunks - 1 : kActorChunks;  // the critic L3 chunk is skipped
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int64_t tbase = (int64_t)blockIdx.x * kRowsPerBlock + wave * kRowsPerWave;
    const int valid = (int)max<int64_t>(0, min<int64_t>(kRowsPerWave, (int64_t)a.n - tbase));
    uint8_t *ring = lds;
    uint8_t *ms = lds + kLdsMask + wave * kMaskWave;
    auto chunk_of = [](int c) { return kCritic && c >= 16 ? c + 1 : c; };

    // weight ring prologue: chunks 0 .. kSlots-2 in flight
#pragma unroll
    for (int c = 0; c < kSlots - 1; ++c) issue_chunk(W, chunk_of(c), ring + c * kChunk, wave, lane);

    // observation B fragments: lane (r, h), k-step s = obs[table r][16s + 8h .. +7] as bf16
    const int32_t *xrow = a.obs + (size_t)min<int64_t>(tbase + r, (int64_t)a.n - 1) * kObs;
    auto load_x = [&](bf16x8 (&X)[kK1]) {
        if constexpr (SPL_ACT_ABL & ABL_XLOAD) {
            for (int s = 0; s < kK1; ++s) X[s] = pack8(h, r, 0, 1, 2, 3, 4, 5);
            return;
        }
#pragma unroll
        for (int s = 0; s < kK1 - 1; ++s) {
            const u32x4u v0 = *reinterpret_cast<const u32x4u *>(xrow + 16 * s + 8 * h);
            const u32x4u v1 = *reinterpret_cast<const u32x4u *>(xrow + 16 * s + 8 * h + 4);
            X[s] = pack8((float)(int)v0.x, (float)(int)v0.y, (float)(int)v0.z, (float)(int)v0.w, (float)(int)v1.x,
                         (float)(int)v1.y, (float)(int)v1.z, (float)(int)v1.w);
        }
        // k-step 18: k = 288..295 (h = 0) or 296 and the zero padding (h = 1)
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = 16 * (kK1 - 1) + 8 * h + j;
            v[j] = k < kObs ? (float)xrow[min(k, kObs - 1)] : 0.f;
        }
        X[kK1 - 1] = pack8(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
    };
    bf16x8 X[kK1];
    load_x(X);
    // masks as bytes
    if (valid == kRowsPerWave) {
        constexpr int kMQ = kMaskWave / 4;  // 360 dwords
        const uint32_t *msrc = reinterpret_cast<const uint32_t *>(a.mask + tbase * kAct);
        for (int q = lane; q < kMQ; q += 64) reinterpret_cast<uint32_t *>(ms)[q] = msrc[q];
    } else {
        const int8_t *msrc = a.mask + tbase * kAct;
        for (int e = lane; e < valid * kAct; e += 64) ms[e] = (uint8_t)msrc[e];
    }

    int c = 0;
    auto enter = [&]() -> const uint8_t * {
        // this wave's part of chunk c landed (later chunks' loads may stay outstanding)
        if (wave < kChunkBlocks - 2 * kWaves) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // everyone's part landed; slot c-1 is free
        asm volatile("" ::: "memory");
        const int nxt = c + kSlots - 1 < kTotal ? c + kSlots - 1 : kTotal - 1;  // past the end: harmless reload
        issue_chunk(W, chunk_of(nxt), ring + ((c + kSlots - 1) % kSlots) * kChunk, wave, lane);
        const uint8_t *slot = ring + (c % kSlots) * kChunk;
        ++c;
        return slot;
    };
    static_assert((kSlots - 2) * 3 == 12 && (kSlots - 2) * 2 == 8, "vmcnt immediates");

    bf16x8 H1[16], H2[16];
    float value = 0.f;
    if constexpr (kCritic) {
        layer_tanh<kK1>(enter, X, H1, lane);
        // layer 2 tile t -> tanh -> its 32 units' share of the fp32 output unit, on the spot
#pragma unroll 1
        for (int t = 0; t < 8; ++t) {
            const f32x16 acc = tile_mma<kK2>(enter(), H1, lane);
            const float *w3 = a.critic_out + 32 * t + 4 * h;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 w = *reinterpret_cast<const float4 *>(w3 + 8 * q);
                value += w.x * tanh_fast(acc[4 * q]) + w.y * tanh_fast(acc[4 * q + 1]) +
                         w.z * tanh_fast(acc[4 * q + 2]) + w.w * tanh_fast(acc[4 * q + 3]);
            }
        }
        value += __shfl_xor(value, 32) + a.critic_out[kHid];  // the other lane half's rows, bias
#if SPL_ACT_RELOAD_X
        // the observation again (L2 / Infinity Cache) instead of holding its 76 registers through
        // the critic's layer 2 (the enter() barriers' memory clobbers keep this a real reload)
        load_x(X);
#endif
    }
    layer_tanh<kK1>(enter, X, H1, lane);
    layer_tanh<kK2>(enter, H1, H2, lane);
    const f32x16 L0 = tile_mma<kK2>(enter(), H2, lane);
    const f32x16 L1 = tile_mma<kK2>(enter(), H2, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing reloads
    __builtin_amdgcn_s_barrier();                      // every wave is done with the ring

    // logits -> LDS [table][action] (reusing the ring), then the per-table epilogue
    float *lg = reinterpret_cast<float *>(ring) + wave * kRowsPerWave * kLogitRow;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int a0 = (reg & 3) + 8 * (reg >> 2) + 4 * h;
        lg[r * kLogitRow + a0] = L0[reg];
        if (32 + a0 < kAct) lg[r * kLogitRow + 32 + a0] = L1[reg];
    }
    wave_lds_sync();
    if (a.logits) {
        float *dst = a.logits + tbase * kAct;
        for (int i = lane; i < valid * kAct; i += 64) dst[i] = lg[(i / kAct) * kLogitRow + i % kAct];
    }
    if ((SPL_ACT_ABL & ABL_EPI) && h == 0 && r < valid) {
        a.action[tbase + r] = (int)lg[r * kLogitRow];
        return;
    }
    if (h == 0 && r < valid) {
        // the table's 45 logits and legal bits into registers (fully unrolled: the LDS reads issue
        // together instead of one latency per loop iteration), then max / softmax / sample in place
        const int64_t t = tbase + r;
        const float *row = lg + r * kLogitRow;
        const uint8_t *mrow = ms + r * kAct;
        float lv[kAct];
        uint64_t legal = 0;
#pragma unroll
        for (int k = 0; k < kAct; ++k) {
            lv[k] = row[k];
            legal |= (uint64_t)(mrow[k] != 0) << k;
        }
        int act = 0;
        if constexpr (!kSample) {
            // logits.masked_fill(mask < 0.5, -inf).argmax(): first maximum; all-illegal -> 0
            float best = -__builtin_inff();
#pragma unroll
            for (int k = 0; k < kAct; ++k) {
                const bool better = ((legal >> k) & 1) && lv[k] > best;
                best = better ? lv[k] : best;
                act = better ? k : act;
            }
        } else {
            // masked_categorical: illegal -> -inf unless the row has no legal action
            const uint64_t allow = legal ? legal : (1ull << kAct) - 1;
            float mx = -__builtin_inff();
#pragma unroll
            for (int k = 0; k < kAct; ++k) mx = ((allow >> k) & 1) ? fmaxf(mx, lv[k]) : mx;
            float S = 0.f, T = 0.f;
#pragma unroll
            for (int k = 0; k < kAct; ++k) {
                const float d = lv[k] - mx, p = ((allow >> k) & 1) ? __expf(d) : 0.f;
                lv[k] = p;  // the unnormalised probability, for the inverse-CDF scan
                S += p;
                T += p * d;
            }
            const float logS = __logf(S);
            const uint64_t ply = a.ply + (a.ply_base ? *a.ply_base : 0ull);
            const uint4 rnd = philox4x32(make_uint4((uint32_t)(a.table0 + t), (uint32_t)((uint64_t)(a.table0 + t) >> 32),
                                                    (uint32_t)ply, (uint32_t)(ply >> 32)),
                                         make_uint2((uint32_t)a.seed, (uint32_t)(a.seed >> 32) ^ 0xA5C3E1F7u));
            const float target = (float)(rnd.x >> 8) * (1.f / 16777216.f) * S;
            float cum = 0.f;
            int last = 0;
            bool found = false;
#pragma unroll
            for (int k = 0; k < kAct; ++k) {
                const bool al = (allow >> k) & 1;
                cum += lv[k];
                last = al ? k : last;
                const bool hit = al && !found && cum > target;
                act = hit ? k : act;
                found = found || hit;
            }
            if (!found) act = last;
            if (a.logprob) a.logprob[t] = row[act] - mx - logS;
            if (a.entropy) a.entropy[t] = logS - T / S;
            if (kCritic) a.value[t] = value;
        }
        a.action[t] = act;
    }
}

}  // namespace splp

using namespace splp;

int64_t splp32_bytes(int with_critic, int fmt);  // spl_policy32.hip: the fp32 images (fmt 0 exact, 1 two fp16 planes)
int splp32_pack(const spl_mlp_t *actor, const spl_mlp_t *critic, void *packed, void *stream, int fmt);
int splp32_act(const uint8_t *img, bool has_critic, bool critic, bool sample, int32_t n, const spl_act_args_t *args,
               void *stream, int fmt, int groups = 0, int64_t image_stride = 0, const int32_t *group_of = nullptr,
               void *scratch = nullptr);
int64_t splp32_group_scratch(int32_t n, int32_t groups);

// the fp32 precisions (spl_policy32.hip): the image format index, or -1
static int fp32_fmt(int precision) {
    return precision == SPL_PREC_FP32 ? 0 : precision == SPL_PREC_FP32_F16X2 ? 1 : -1;
}

extern "C" {

int64_t spl_policy_bytes(int32_t with_critic, int32_t precision) {
    if (fp32_fmt(precision) >= 0) return splp32_bytes(with_critic ? 1 : 0, fp32_fmt(precision));
    if (precision != SPL_PREC_BF16) return SPL_E_ARG;
    return with_critic ? (int64_t)kAllChunks * kChunk + kCriticTail : (int64_t)kActorChunks * kChunk;
}

int spl_policy_pack(const spl_mlp_t *actor, const spl_mlp_t *critic, int32_t precision, void *packed, void *stream) {
    if (!actor || !actor->w1 || !actor->b1 || !actor->w2 || !actor->b2 || !actor->w3 || !actor->b3)
        return spl_fail(SPL_E_ARG, "actor weights missing");
    if (critic && (!critic->w1 || !critic->b1 || !critic->w2 || !critic->b2 || !critic->w3 || !critic->b3))
        return spl_fail(SPL_E_ARG, "critic weights incomplete");
    if (!packed || ((uintptr_t)packed & 255u)) return spl_fail(SPL_E_ARG, "packed image must be 256-byte aligned");
    if (fp32_fmt(precision) >= 0) return splp32_pack(actor, critic, packed, stream, fp32_fmt(precision));
    if (precision != SPL_PREC_BF16) return spl_fail(SPL_E_ARG, "unknown precision");
    const PackNet A{actor->w1, actor->b1, actor->w2, actor->b2, actor->w3, actor->b3, kAct};
    const PackNet C = critic ? PackNet{critic->w1, critic->b1, critic->w2, critic->b2, critic->w3, critic->b3, 1} : A;
    const int chunks = critic ? kAllChunks : kActorChunks;
    hipLaunchKernelGGL(k_pack, dim3(chunks), dim3(256), 0, (hipStream_t)stream, A, C, critic ? 1 : 0,
                       static_cast<uint8_t *>(packed));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return spl_fail(SPL_E_HIP, std::string("k_pack launch: ") + hipGetErrorString(e));
    return SPL_OK;
}

// the observation: int32 obs (16-byte aligned), or (fp32 images) the compact obs_u8 rows
static int check_obs(const spl_act_args_t *args, int precision) {
    if (args->obs_u8) {
        if (args->obs) return spl_fail(SPL_E_ARG, "obs and obs_u8 are exclusive");
        if (fp32_fmt(precision) < 0) return spl_fail(SPL_E_ARG, "obs_u8 is read by the fp32 kernels");
        if ((uintptr_t)args->obs_u8 & 3u) return spl_fail(SPL_E_ARG, "obs_u8 must be 4-byte aligned");
        return SPL_OK;
    }
    if (!args->obs || ((uintptr_t)args->obs & 15u)) return spl_fail(SPL_E_ARG, "obs must be 16-byte aligned");
    return SPL_OK;
}

int spl_policy_act(const void *packed, int64_t packed_bytes, int32_t n, const spl_act_args_t *args, void *stream) {
    if (!args) return spl_fail(SPL_E_ARG, "null args");
    if (!packed || ((uintptr_t)packed & 255u)) return spl_fail(SPL_E_ARG, "packed image must be 256-byte aligned");
    const int precision = (args->image >> 1) & 3;
    const bool has_critic = (args->image & SPL_IMG_CRITIC) != 0;
    if (fp32_fmt(precision) < 0 && precision != SPL_PREC_BF16) return spl_fail(SPL_E_ARG, "unknown precision");
    // the image is described by args->image, and its size must be exactly that image's: a full image
    // passed as actor-only (or the reverse) would evaluate the wrong chunks
    if (packed_bytes != spl_policy_bytes(has_critic ? 1 : 0, precision))
        return spl_fail(SPL_E_ARG, "packed_bytes does not match the image described by args->image");
    if (n <= 0) return spl_fail(SPL_E_ARG, "n must be positive");
    if (int r = check_obs(args, precision)) return r;
    if (args->mode == SPL_ACT_VALUE) {  // ActorCritic.get_value (ppo_splendor.py:51): the critic alone
        if (!has_critic || !args->value) return spl_fail(SPL_E_ARG, "VALUE needs an image with a critic and a value output");
        if (fp32_fmt(precision) < 0) return spl_fail(SPL_E_ARG, "VALUE is implemented for fp32 images");
        return splp32_act(static_cast<const uint8_t *>(packed), true, true, false, n, args, stream, fp32_fmt(precision));
    }
    if (!args->mask || ((uintptr_t)args->mask & 3u)) return spl_fail(SPL_E_ARG, "mask must be 4-byte aligned");
    if (!args->action) return spl_fail(SPL_E_ARG, "action output missing");
    if (args->mode != SPL_ACT_SAMPLE && args->mode != SPL_ACT_GREEDY) return spl_fail(SPL_E_ARG, "unknown mode");
    const bool sample = args->mode == SPL_ACT_SAMPLE;
    const bool critic = sample && args->value;
    if (critic && !has_critic) return spl_fail(SPL_E_ARG, "value requested from an actor-only image");
    const uint8_t *img = static_cast<const uint8_t *>(packed);
    if (fp32_fmt(precision) >= 0)
        return splp32_act(img, has_critic, critic, sample, n, args, stream, fp32_fmt(precision));
    const float *critic_out = has_critic ? reinterpret_cast<const float *>(img + (size_t)kAllChunks * kChunk) : nullptr;
    const ActArgs a{args->obs,   args->mask,       args->action,   args->logprob, args->entropy,
                    args->value, args->logits,     critic_out,     args->seed,    args->ply,
                    args->ply_base, args->table0, n};
    const dim3 grid((unsigned)((n + kRowsPerBlock - 1) / kRowsPerBlock)), block(kWaves * 64);
    const hipStream_t s = (hipStream_t)stream;
    const uint8_t *W = img;
    if (has_critic && !critic) W += (size_t)kCriticChunks * kChunk;  // the actor part of a full image
    if (critic)
        hipLaunchKernelGGL((k_act<true, true>), grid, block, 0, s, W, a);
    else if (sample)
        hipLaunchKernelGGL((k_act<false, true>), grid, block, 0, s, W, a);
    else
        hipLaunchKernelGGL((k_act<false, false>), grid, block, 0, s, W, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return spl_fail(SPL_E_HIP, std::string("k_act launch: ") + hipGetErrorString(e));
    return SPL_OK;
}

int64_t spl_policy_group_scratch_bytes(int32_t n, int32_t n_images) {
    if (n <= 0 || n_images <= 0) return SPL_E_ARG;
    return splp32_group_scratch(n, n_images);
}

int spl_policy_act_grouped(const void *images, int64_t image_bytes, int32_t n_images, const int32_t *group_of,
                           void *scratch, int32_t n, const spl_act_args_t *args, void *stream) {
    if (!args || !group_of || !scratch) return spl_fail(SPL_E_ARG, "null argument");
    if (!images || ((uintptr_t)images & 255u) || (image_bytes & 255))
        return spl_fail(SPL_E_ARG, "images must be 256-byte aligned, image_bytes a multiple of 256");
    if (n_images <= 0 || n_images > 64) return spl_fail(SPL_E_ARG, "n_images must be 1..64");
    if (((uintptr_t)scratch & 3u)) return spl_fail(SPL_E_ARG, "scratch must be 4-byte aligned");
    const int precision = (args->image >> 1) & 3;
    const bool has_critic = (args->image & SPL_IMG_CRITIC) != 0;
    if (fp32_fmt(precision) < 0) return spl_fail(SPL_E_ARG, "grouped evaluation is implemented for fp32 images");
    if (has_critic) return spl_fail(SPL_E_ARG, "grouped evaluation serves actor-only images");
    if (image_bytes < spl_policy_bytes(0, precision)) return spl_fail(SPL_E_ARG, "image_bytes smaller than an image");
    if (n <= 0) return spl_fail(SPL_E_ARG, "n must be positive");
    if (int r = check_obs(args, precision)) return r;
    if (!args->mask || !args->action) return spl_fail(SPL_E_ARG, "mask / action missing");
    if (args->mode != SPL_ACT_SAMPLE && args->mode != SPL_ACT_GREEDY) return spl_fail(SPL_E_ARG, "unknown mode");
    if (args->value) return spl_fail(SPL_E_ARG, "grouped evaluation has no critic");
    return splp32_act(static_cast<const uint8_t *>(images), false, false, args->mode == SPL_ACT_SAMPLE, n, args, stream,
                      fp32_fmt(precision), n_images, image_bytes, group_of, scratch);
}

}  // extern "C"

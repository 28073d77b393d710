// spl_policy.hip — fused ActorCritic forward for batched self-play on MI355X (gfx950).
//
// Reference network (ppo_splendor.py:40-59): actor and critic are separate
// Linear(297,256)-Tanh-Linear(256,256)-Tanh-Linear(256,{45|1}) MLPs; get_action_and_value
// samples masked_categorical(actor(x), mask) (ppo_splendor.py:27-37) and returns log_prob,
// entropy and critic(x); opponents play the greedy masked argmax of a frozen actor
// (training_utils.py:263-276).  Here one launch evaluates that for every table:
//
//   * a workgroup = 4 waves = 128 tables, one wave = 32 tables = the 32 columns of every
//     v_mfma_f32_32x32x16_bf16 tile.  Activations are computed TRANSPOSED (hidden unit on the
//     accumulator row, table on the lane), so each layer's accumulator registers are directly the
//     next layer's B operand: no LDS round trip between layers (the k order inside a 16-step is
//     permuted; the packed weights carry the matching column order).
//   * weights are packed once (k_pack) into 20 KB "chunks" — one 32-row output tile of one layer,
//     [k-step][lane][8 bf16] in fragment order plus the tile's bias in accumulator order — and
//     streamed through a 3-slot LDS ring with global_load_lds (2 chunks in flight), shared by the
//     workgroup's 4 waves.  The whole image (0.7 MB) stays L2-resident across workgroups.
//   * observations (int32) are staged per wave in LDS as bf16 (every obs value is a small
//     integer, exact in bf16); layer 1 reads its B fragments from there (one ds_read_b128 per
//     MFMA beside the weight fragment's), so only the hidden activations occupy registers.
//   * tanh, bias, masking, log-softmax, entropy and the Philox-driven inverse-CDF sample are
//     fused after the last tile; the sampled action differs from torch's multinomial stream by
//     design (same distribution), logits match the fp32 module to bf16 accuracy.
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
constexpr int kWaves = 4, kRowsPerWave = 32, kRowsPerBlock = kWaves * kRowsPerWave;
constexpr int kXRow = 312;                       // bf16 per staged observation row (bank-conflict pad)
constexpr int kXWave = kRowsPerWave * kXRow * 2;  // 19 968 B
constexpr int kMaskWave = kRowsPerWave * kAct;    // 1 440 B
constexpr int kLogitRow = 65;                     // floats per staged logit row
constexpr int kLdsX = 3 * kChunk;
constexpr int kLdsMask = kLdsX + kWaves * kXWave;
constexpr int kLds = kLdsMask + kWaves * kMaskWave;  // 147 072 B
static_assert(kRowsPerWave * kLogitRow * 4 <= kXWave, "logits reuse the observation image");
static_assert(kLds <= 160 * 1024, "LDS");

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

// this wave's fifth of one chunk, global -> LDS (lane-linear 16-byte pieces)
__device__ __forceinline__ void issue_chunk(const uint8_t *W, int chunk, uint8_t *slot, int wave, int lane) {
    const uint8_t *src = W + (size_t)chunk * kChunk + wave * 1024 + lane * 16;
    uint8_t *dst = slot + wave * 1024;
#pragma unroll
    for (int i = 0; i < kChunk / 4096; ++i)
        __builtin_amdgcn_global_load_lds(src + i * 4096, (lds_void *)(dst + i * 4096), 16, 0, 0);
}

__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __expf(2.f * x);
    return 1.f - __fdividef(2.f, e + 1.f);
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

// one 32-row output tile: bias + sum over KS k-steps; B fragments from registers (layers 2-3) or
// from the wave's staged observation row (layer 1, a 16-byte LDS read per k-step).  LDS fragment
// reads run one group of 4 k-steps ahead of the MFMAs that use them; the scheduling barriers keep
// the compiler from hoisting every read of the tile (and its registers) to the top.
template <int KS, bool kBFromLds, typename BF>
__device__ __forceinline__ f32x16 tile_mma(const uint8_t *slot, BF B, int lane) {
    constexpr int G = 4, NG = (KS + G - 1) / G;
    const float *bias = reinterpret_cast<const float *>(slot + kBiasOff) + (lane >> 5) * 16;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = bias[r];
    const bf16x8 *A = reinterpret_cast<const bf16x8 *>(slot) + lane;
    bf16x8 af[2][G], bf[2][G];
#pragma unroll
    for (int i = 0; i < G; ++i) {
        af[0][i] = A[i * 64];
        if constexpr (kBFromLds) bf[0][i] = B[i];
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (g + 1 < NG) {
#pragma unroll
            for (int i = 0; i < G; ++i) {
                const int s = (g + 1) * G + i;
                if (s < KS) {
                    af[(g + 1) & 1][i] = A[s * 64];
                    if constexpr (kBFromLds) bf[(g + 1) & 1][i] = B[s];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const int s = g * G + i;
            if (s < KS) {
                if constexpr (kBFromLds)
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[g & 1][i], bf[g & 1][i], acc, 0, 0, 0);
                else
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[g & 1][i], B[s], acc, 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    return acc;
}

template <bool kCritic, bool kSample>
__global__ __launch_bounds__(256, 1) void k_act(const uint8_t *__restrict__ W, ActArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLds];
    constexpr int kTotal = kCritic ? kAllChunks : kActorChunks;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    const int64_t tbase = (int64_t)blockIdx.x * kRowsPerBlock + wave * kRowsPerWave;
    const int valid = (int)max<int64_t>(0, min<int64_t>(kRowsPerWave, (int64_t)a.n - tbase));
    uint8_t *ring = lds;
    __bf16 *xs = reinterpret_cast<__bf16 *>(lds + kLdsX + wave * kXWave);
    uint8_t *ms = lds + kLdsMask + wave * kMaskWave;

    // weight ring prologue: chunks 0 and 1 in flight
    issue_chunk(W, 0, ring, wave, lane);
    issue_chunk(W, 1, ring + kChunk, wave, lane);

    // stage this wave's observations (contiguous rows) as bf16 and its masks as bytes
    if (valid == kRowsPerWave) {  // full wave: branch-free 16-byte loads, all issued up front
        constexpr int kQ = kRowsPerWave * kObs / 4, kIters = (kQ + 63) / 64;  // 2376 int4, 38 per lane
        constexpr int kMQ = kMaskWave / 4, kMIters = (kMQ + 63) / 64;          // 360 dwords, 6 per lane
        const int4 *src = reinterpret_cast<const int4 *>(a.obs + tbase * kObs);
        const uint32_t *msrc = reinterpret_cast<const uint32_t *>(a.mask + tbase * kAct);
        int4 v[kIters];
        uint32_t mv[kMIters];
#pragma unroll
        for (int it = 0; it < kIters; ++it) v[it] = src[min(it * 64 + lane, kQ - 1)];
#pragma unroll
        for (int it = 0; it < kMIters; ++it) mv[it] = msrc[min(it * 64 + lane, kMQ - 1)];
#pragma unroll
        for (int it = 0; it < kIters; ++it) {
            const int q = it * 64 + lane;
            if (q < kQ) {
                const int vals[4] = {v[it].x, v[it].y, v[it].z, v[it].w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int e = 4 * q + i, row = e / kObs, k = e - row * kObs;
                    xs[row * kXRow + k] = (__bf16)(float)vals[i];
                }
            }
        }
#pragma unroll
        for (int it = 0; it < kMIters; ++it) {
            const int q = it * 64 + lane;
            if (q < kMQ) reinterpret_cast<uint32_t *>(ms)[q] = mv[it];
        }
    } else {  // the grid's last, partial wave (or an idle one): element-wise, bounds-checked
        const int32_t *src = a.obs + tbase * kObs;
        for (int e = lane; e < valid * kObs; e += 64) {
            const int row = e / kObs, k = e - row * kObs;
            xs[row * kXRow + k] = (__bf16)(float)src[e];
        }
        const int8_t *msrc = a.mask + tbase * kAct;
        for (int e = lane; e < valid * kAct; e += 64) ms[e] = (uint8_t)msrc[e];
    }
    for (int idx = lane; idx < kRowsPerWave * 7; idx += 64)  // k = 297..303 of every row
        xs[(idx / 7) * kXRow + kObs + idx % 7] = (__bf16)0.f;
    wave_lds_sync();
    const bf16x8 *xrow = reinterpret_cast<const bf16x8 *>(reinterpret_cast<const uint8_t *>(xs) + r * kXRow * 2) + h;
    struct XFrag {
        const bf16x8 *p;
        __device__ bf16x8 operator[](int s) const { return p[2 * s]; }
    } X{xrow};

    int c = 0;
    auto enter = [&]() -> const uint8_t * {
        asm volatile("s_waitcnt vmcnt(5)" ::: "memory");  // this wave's part of chunk c landed
        __builtin_amdgcn_s_barrier();                      // everyone's part landed; slot c-1 free
        asm volatile("" ::: "memory");
        const int nxt = c + 2 < kTotal ? c + 2 : kTotal - 1;  // past the end: harmless reload
        issue_chunk(W, nxt, ring + ((c + 2) % 3) * kChunk, wave, lane);
        const uint8_t *slot = ring + (c % 3) * kChunk;
        ++c;
        return slot;
    };

    bf16x8 H1[16], H2[16];
    float value = 0.f;
    if constexpr (kCritic) {  // critic first: only its scalar output stays live across the actor
#pragma unroll
        for (int t = 0; t < 8; ++t) tanh_pack(tile_mma<kK1, true>(enter(), X, lane), H1[2 * t], H1[2 * t + 1]);
#pragma unroll
        for (int t = 0; t < 8; ++t) tanh_pack(tile_mma<kK2, false>(enter(), H1, lane), H2[2 * t], H2[2 * t + 1]);
        value = tile_mma<kK2, false>(enter(), H2, lane)[0];  // row 0 = the critic output (lanes h == 0)
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) tanh_pack(tile_mma<kK1, true>(enter(), X, lane), H1[2 * t], H1[2 * t + 1]);
#pragma unroll
    for (int t = 0; t < 8; ++t) tanh_pack(tile_mma<kK2, false>(enter(), H1, lane), H2[2 * t], H2[2 * t + 1]);
    const f32x16 L0 = tile_mma<kK2, false>(enter(), H2, lane);
    const f32x16 L1 = tile_mma<kK2, false>(enter(), H2, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing reloads

    // logits -> LDS [table][action] (reusing the observation image), then per-table epilogue
    float *lg = reinterpret_cast<float *>(xs);
    wave_lds_sync();
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
    if (h == 0 && r < valid) {
        const int64_t t = tbase + r;
        const float *row = lg + r * kLogitRow;
        uint64_t legal = 0;
        for (int k = 0; k < kAct; ++k) legal |= (uint64_t)(ms[r * kAct + k] != 0) << k;
        int act = 0;
        if constexpr (!kSample) {
            // logits.masked_fill(mask < 0.5, -inf).argmax(): first maximum; all-illegal -> 0
            float best = -__builtin_inff();
            for (int k = 0; k < kAct; ++k)
                if (((legal >> k) & 1) && row[k] > best) best = row[k], act = k;
        } else {
            // masked_categorical: illegal -> -inf unless the row has no legal action
            const uint64_t allow = legal ? legal : (1ull << kAct) - 1;
            float mx = -__builtin_inff();
            for (int k = 0; k < kAct; ++k)
                if ((allow >> k) & 1) mx = fmaxf(mx, row[k]);
            float S = 0.f, T = 0.f;
            for (int k = 0; k < kAct; ++k)
                if ((allow >> k) & 1) {
                    const float d = row[k] - mx, p = __expf(d);
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
            for (int k = 0; k < kAct; ++k)
                if ((allow >> k) & 1) {
                    cum += __expf(row[k] - mx);
                    last = k;
                    if (!found && cum > target) act = k, found = true;
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

extern "C" {

int64_t spl_policy_bytes(int32_t with_critic) { return (int64_t)(with_critic ? kAllChunks : kActorChunks) * kChunk; }

int spl_policy_pack(const spl_mlp_t *actor, const spl_mlp_t *critic, void *packed, void *stream) {
    if (!actor || !actor->w1 || !actor->b1 || !actor->w2 || !actor->b2 || !actor->w3 || !actor->b3)
        return spl_fail(SPL_E_ARG, "actor weights missing");
    if (critic && (!critic->w1 || !critic->b1 || !critic->w2 || !critic->b2 || !critic->w3 || !critic->b3))
        return spl_fail(SPL_E_ARG, "critic weights incomplete");
    if (!packed || ((uintptr_t)packed & 255u)) return spl_fail(SPL_E_ARG, "packed image must be 256-byte aligned");
    const PackNet A{actor->w1, actor->b1, actor->w2, actor->b2, actor->w3, actor->b3, kAct};
    const PackNet C = critic ? PackNet{critic->w1, critic->b1, critic->w2, critic->b2, critic->w3, critic->b3, 1} : A;
    const int chunks = critic ? kAllChunks : kActorChunks;
    hipLaunchKernelGGL(k_pack, dim3(chunks), dim3(256), 0, (hipStream_t)stream, A, C, critic ? 1 : 0,
                       static_cast<uint8_t *>(packed));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return spl_fail(SPL_E_HIP, std::string("k_pack launch: ") + hipGetErrorString(e));
    return SPL_OK;
}

int spl_policy_act(const void *packed, int64_t packed_bytes, int32_t n, const spl_act_args_t *args, void *stream) {
    if (!args) return spl_fail(SPL_E_ARG, "null args");
    if (!packed || ((uintptr_t)packed & 255u)) return spl_fail(SPL_E_ARG, "packed image must be 256-byte aligned");
    if (packed_bytes < spl_policy_bytes(0)) return spl_fail(SPL_E_ARG, "packed image too small");
    if (n <= 0) return spl_fail(SPL_E_ARG, "n must be positive");
    if (!args->obs || ((uintptr_t)args->obs & 15u)) return spl_fail(SPL_E_ARG, "obs must be 16-byte aligned");
    if (!args->mask || ((uintptr_t)args->mask & 3u)) return spl_fail(SPL_E_ARG, "mask must be 4-byte aligned");
    if (!args->action) return spl_fail(SPL_E_ARG, "action output missing");
    if (args->mode != SPL_ACT_SAMPLE && args->mode != SPL_ACT_GREEDY) return spl_fail(SPL_E_ARG, "unknown mode");
    const bool has_critic = packed_bytes >= spl_policy_bytes(1);  // critic chunks follow the actor's
    const bool sample = args->mode == SPL_ACT_SAMPLE;
    const bool critic = sample && args->value;
    if (critic && !has_critic) return spl_fail(SPL_E_ARG, "value requested from an actor-only image");
    const ActArgs a{args->obs, args->mask, args->action, args->logprob, args->entropy, args->value, args->logits,
                    args->seed, args->ply, args->ply_base, args->table0, n};
    const dim3 grid((unsigned)((n + kRowsPerBlock - 1) / kRowsPerBlock)), block(kWaves * 64);
    const hipStream_t s = (hipStream_t)stream;
    const uint8_t *W = static_cast<const uint8_t *>(packed);
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

}  // extern "C"

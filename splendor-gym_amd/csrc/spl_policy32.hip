// spl_policy32.hip — the fused ActorCritic forward at fp32 accuracy (the reference's precision) on MI355X.
//
// Same network and epilogue as spl_policy.hip's bf16 kernel (ppo_splendor.py:27-59: actor and
// critic Linear(297,256)-Tanh-Linear(256,256)-Tanh-Linear(256,{45|1}); masked_categorical sample,
// log_prob, entropy, critic value; or the greedy masked argmax of training_utils.py:263-276), with
// fp32 operands carried exactly into the 16-bit matrix cores (gfx950 has no xf32 MFMA, and its fp32
// MFMA runs at 1/16 of the fp16/bf16 rate).  Two operand formats, each its own kernels in this file:
//   * SPL_PREC_FP32 — EXACT fp32 operands (FmtBf16x3; round 3's split, the default since round 5,
//     VERDICT r04 item 2): every fp32 operand x is three bf16 planes x = x0 + x1 + x2 (x0 = bf16(x),
//     x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)): 24 significant bits, so the planes hold x EXACTLY (bf16
//     has fp32's exponent range: no scaling).  A hidden-layer product a*w is the six plane products of
//     order <= 2 (a2w0 + a1w1 + a0w2 + a1w0 + a0w1 + a0w0, smallest first) on v_mfma_f32_16x16x32_bf16,
//     each bf16 x bf16 product exact in fp32; the dropped a1w2 + a2w1 + a2w2 are <= 2^-24 of |aw| each,
//     below fp32's own rounding of the sum.  Layer 1's operand, the observation, is integers: exact in
//     ONE bf16 plane below 256 (every observation value the engine writes except a move count above
//     255); where a wave holds a larger value (< 2^16) its residual plane adds two products to that
//     k-step (ObsHi).  tanh in fp32 to <= ~2 ulp everywhere (tanh_acc).
//   * SPL_PREC_FP32_F16X2 — fp32 within 2^-22 (FmtF16x2; round 4): every fp32 operand is two fp16
//     planes x = x0 + x1 (22 significant bits; weights scaled per output row by a power of two so the
//     row's largest |w| lands in [512, 1024) and every plane stays a normal fp16, hidden activations
//     scaled by 2^10); three plane products (a1w0 + a0w1 + a0w0, the dropped a1w1 <= 2^-22 |aw|) on
//     v_mfma_f32_16x16x32_f16; the observation (< 2048, exact in fp16) takes two.  tanh from exp
//     (tanh_fold: absolute error ~1e-7, relative error grows near 0).  Fewer products, so faster; not an
//     exact representation, and labelled so (bench.py).
//   * a wave = 16 tables = the 16 columns of every 16x16x32 tile; a workgroup = 8 waves = 128 tables
//     (two waves per SIMD).  Activations are TRANSPOSED (hidden unit on the accumulator row, table
//     on the lane): accumulator register i of lane group g holds unit 16t + 4g + i of tile t, and
//     tiles 2s, 2s+1 are lane group g's B elements of k-step s of the next layer (element e = unit
//     16(2s + e/4) + 4g + e%4) — no LDS round trip between layers; the packed weights carry the
//     matching input-unit order.  tanh runs in fp32 before the split.
//   * the observation loads into registers as the 10 layer-1 B fragments and stays there through both
//     networks' layer 1; a hidden layer's output is kPlanes planes x 8 k-steps x 8 elements per lane.
//   * weights stream once per workgroup through an LDS ring of chunks (one chunk = one 16-row output
//     tile of one layer, [k-step][plane][lane][8 elements] + biases + row factors; 31 KB for three
//     bf16 planes in 4 slots, 21 KB for two fp16 planes in 5), global_load_lds, shared by the 8 waves.
//   * the critic's one-unit output layer is a per-lane fp32 FMA chain over its layer-2 tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

// SPL_P32_PIPE (default 1): each tile's epilogue is issued in stages inside the next tile's k-steps
// (PendTile below); 0: after its own tile's MFMA chain (round 4's order).  Same results either way.
#ifndef SPL_P32_PIPE
#define SPL_P32_PIPE 1
#endif
// SPL_P32_RINGV: the weight ring filled through registers (global load, then ds_write a tile later)
// instead of LDS-DMA (see stage_chunk)
#ifndef SPL_P32_RINGV
#define SPL_P32_RINGV 0
#endif
// SPL_P32_GROUP 2 (default): one ring barrier per two chunks (four slots: two in use, two loading);
// exact k_act32<true, true> 215.8 -> 206 us, alternating on one box (profiles/r05/pol_ring_ab_r05g.txt;
// without any barrier, a racing timing build, 195 us: the barriers cost ~20 us, half of it recovered)
#ifndef SPL_P32_GROUP
#define SPL_P32_GROUP 2
#endif
// SPL_P32_SPREAD (group-2 ring, pipelined epilogue): the ring's LDS-DMA pieces are issued one per
// k-step inside the tiles (see tick in act32_body) instead of eight back to back right behind the even
// barrier (a piece issued among MFMAs costs the wave ~60 cycles of issue, 100-185 in a burst of eight,
// MI355X_MICROARCH.md).  0: the burst.  Alternating on one box, exact k_act32<true, true>: burst
// 208.3 us -> one piece per two k-steps of every tile 201.5 (profiles/r05/pol_spread_ab_r05j.txt) ->
// branch-free pieces 197.1 (pol_nobr_ab_r05k.txt) -> + the paired plane split 198.1 vs 201.4
// (pol_pair_ab_r05l.txt) -> even tiles load the next pair, hidden chunks without their padding blocks
// 191.9 vs 198.3 (pol_ahead_ab_r05m.txt)
#ifndef SPL_P32_SPREAD
#define SPL_P32_SPREAD 1
#endif
// timing ablations (wrong results by design): 1 tanh = identity, 2 one weight chunk (no ring
// streaming: no LDS-DMA piece after the prologue, no per-tile barrier), 4 A fragments loaded once
// per tile (no per-group LDS reads), 16 the ring without its barriers (waves race the slots), 32 no
// per-table epilogue (no softmax / sample / argmax), 64 no observation loads (zero layer-1 operand),
// 512 no MFMA at all (an empty asm keeps each product's operands live; 8 replaces it by a VALU op);
// the tail kernel k_act32_narrow: 128 its launch and index lookups only, 256 no layers (zero logits)
#ifndef SPL_POL_ABL
#define SPL_POL_ABL 0
#endif

#include "../../include/splendor_amd.h"
#include "../../include/splendor_policy.h"
#include "spl_rng.h"

int spl_fail(int code, const std::string &msg);  // spl_engine.hip: sets spl_last_error()

namespace splp32 {

using spl::philox4x32;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// ---- the two operand formats ------------------------------------------------------------------
struct FmtBf16x3 {  // SPL_PREC_FP32: exact (24 significant bits in three bf16 planes)
    typedef __bf16 pel;
    typedef bf16x8 pelx8;
    typedef bf16x2 pelx2;
    static constexpr int kPlanes = 3;
    static constexpr int kActScaleExp = 0;  // bf16 has fp32's exponent range: no scaling anywhere
    static constexpr int kRowMaxExp = 0;
    static constexpr int kSlots = 4;        // ring slots of 31 KB (3 chunks in flight)
    static constexpr bool kExact = true;
};
struct FmtF16x2 {   // SPL_PREC_FP32_F16X2: 22 significant bits in two fp16 planes
    typedef _Float16 pel;
    typedef f16x8 pelx8;
    typedef f16x2 pelx2;
    static constexpr int kPlanes = 2;
    static constexpr int kActScaleExp = 10;  // hidden activations enter the next layer as tanh * 2^10
    static constexpr int kRowMaxExp = 10;    // a weight row's largest |w| is scaled into [2^9, 2^10)
    static constexpr int kSlots = SPL_P32_GROUP == 2 ? 4 : 5;  // ring slots of 21 KB (4 chunks in flight)
    static constexpr bool kExact = false;
};

constexpr float kTwoLog2e = 2.8853900817779268f;  // 2 log2(e): exp(2|x|) = exp2(2 log2(e) |x|)
constexpr int kObs = 297, kAct = 45, kHid = 256;
constexpr int kKs1 = 10;    // layer-1 k-steps of 32: 297 inputs padded to 320
constexpr int kKs2 = 8;     // layers 2 and 3: 256 inputs
constexpr int kFrag = 1024;                       // one plane of one k-step: [lane][8 elements]
constexpr int kTiles = kHid / 16;                 // 16 output tiles of 16 rows per hidden layer
constexpr int kActTiles = 3;                      // 48 rows >= 45 logits
constexpr int kActorChunks = 2 * kTiles + kActTiles, kCriticChunks = 2 * kTiles;  // 35, 32
constexpr int kAllChunks = kActorChunks + kCriticChunks;                          // 67
constexpr int kCriticTail = 272 * 4;  // fp32 critic output layer: w3 [256], b3, padding
constexpr int kWaves = 8, kRowsPerWave = 16, kRowsPerBlock = kWaves * kRowsPerWave;  // 128 tables
constexpr int kMaskWave = kRowsPerWave * kAct;  // 720 B
constexpr int kLogitRow = 49;                   // floats per staged logit row (odd: conflict-free)

// sizes that follow from the format
template <class F>
struct Geo {
    // a layer's chunk: its KS k-steps of weight blocks, then one block of 16 biases, 16 row factors and
    // 16 tanh factors (bias_off); chunks are kChunk apart in the image (the largest, layer 1's) and a
    // hidden layer's 6 (exact) / 4 (f16x2) trailing blocks are zero padding the ring does not load
    static constexpr int kBiasOff = kKs1 * F::kPlanes * kFrag;
    static constexpr int kChunk = kBiasOff + 1024;
    static constexpr int bias_off(int ks) { return ks * F::kPlanes * kFrag; }
    static constexpr int blocks(int ks) { return ks * F::kPlanes + 1; }
    static constexpr int kLdsMask = F::kSlots * kChunk;
    static constexpr int kLdsCritic = kLdsMask + kWaves * kMaskWave;  // the critic's fp32 output layer (1 KB)
    static constexpr int kLds = kLdsCritic + kCriticTail;
    static constexpr int kChunkBlocks = kChunk / 1024;                           // 31 / 21
    static constexpr int kBlocksPerWave = (kChunkBlocks + kWaves - 1) / kWaves;  // 4 / 3
    // a wave's loads of the chunks after chunk c that may stay in flight when it enters chunk c
    static constexpr int kWaitMost = (F::kSlots - 2) * kBlocksPerWave, kWaitLast = (F::kSlots - 2) * (kBlocksPerWave - 1);
    static_assert(kWaves * kRowsPerWave * kLogitRow * 4 <= kLdsMask, "logits reuse the weight ring");
    static_assert(kLds <= 160 * 1024, "LDS");
    static_assert(kWaitMost <= 63, "vmcnt range");
};

// chunk order of an image (the order a forward pass consumes them): with a critic
// [critic L1 x16][critic L2 x16], then [actor L1 x16][actor L2 x16][actor L3 x3]; the actor part of
// a full image (its last 35 chunks) is laid out exactly as an actor-only image.

struct PackNet {
    const float *w1, *b1, *w2, *b2, *w3, *b3;
    int out;
};

// input unit of lane group g, element e at k-step s: natural order in layer 1 (the observation),
// the accumulator order of the previous layer's tiles in layers 2-3 (tile 2s + e/4, register e%4)
__device__ __forceinline__ int unit_of(int layer, int s, int g, int e) {
    return layer == 1 ? 32 * s + 8 * g + e : 16 * (2 * s + (e >> 2)) + 4 * g + (e & 3);
}

// x = x0 + x1 (+ x2) in the plane format (round to nearest even; the residuals are exact in fp32)
template <class F>
__device__ __forceinline__ void split_planes(float x, typename F::pel (&q)[F::kPlanes]) {
    typedef typename F::pel pel;
    q[0] = (pel)x;
    const float r = x - (float)q[0];
    q[1] = (pel)r;
    if constexpr (F::kPlanes == 3) q[2] = (pel)(r - (float)q[1]);
}

// one block per physical chunk: [k-step s][plane p][lane][8 elements], lane l = (g = l >> 4, r = l & 15)
// holds W[row 16*tile + r][unit_of(layer, s, g, e)] * 2^e_row split into the planes; then the 16 rows'
// biases scaled as the products are (2^(e_row + layer's activation exponent)), the 16 exact factors
// 2^-(e_row + activation exponent) that bring a row's sum back, and the 16 tanh factors (tanh_fold)
template <class F>
__device__ __forceinline__ void pack_chunk(PackNet actor, PackNet critic, int with_critic, uint8_t *dst) {
    typedef typename F::pel pel;
    constexpr int kChunk = Geo<F>::kChunk;
    const int ch = blockIdx.x;
    const int net = with_critic && ch < kCriticChunks ? 1 : 0;  // 0 actor, 1 critic
    const int local = ch - (with_critic && !net ? kCriticChunks : 0);
    const int layer = local < kTiles ? 1 : local < 2 * kTiles ? 2 : 3;
    const int tile = local - (layer - 1) * kTiles;
    const PackNet &P = net ? critic : actor;
    const float *W = layer == 1 ? P.w1 : layer == 2 ? P.w2 : P.w3;
    const float *B = layer == 1 ? P.b1 : layer == 2 ? P.b2 : P.b3;
    const int in = layer == 1 ? kObs : kHid, rows = layer == 3 ? P.out : kHid;
    const int ks = layer == 1 ? kKs1 : kKs2, bias_at = Geo<F>::bias_off(ks);
    uint8_t *out = dst + (size_t)ch * kChunk;
    pel *o = reinterpret_cast<pel *>(out);
    // each row's scale exponent: its largest |w| into [2^(kRowMaxExp-1), 2^kRowMaxExp) (fp16 planes)
    __shared__ float part[16][17];
    __shared__ int rexp[16];
    {
        const int r = threadIdx.x >> 4, c = threadIdx.x & 15, row = 16 * tile + r;
        float m = 0.f;
        if (row < rows)
            for (int k = c; k < in; k += 16) m = fmaxf(m, fabsf(W[(size_t)row * in + k]));
        part[r][c] = m;
        __syncthreads();
        if (threadIdx.x < 16) {
            float mx = 0.f;
            for (int j = 0; j < 16; ++j) mx = fmaxf(mx, part[threadIdx.x][j]);
            int x = 0;
            (void)frexpf(mx, &x);  // mx = f * 2^x, f in [0.5, 1)
            rexp[threadIdx.x] = (F::kRowMaxExp == 0 || mx == 0.f) ? 0 : max(-40, min(60, F::kRowMaxExp - x));
        }
        __syncthreads();
    }
    for (int v = threadIdx.x; v < ks * 64 * 8; v += blockDim.x) {
        const int e = v & 7, lane = (v >> 3) & 63, s = v >> 9;
        const int r = lane & 15, g = lane >> 4, row = 16 * tile + r, k = unit_of(layer, s, g, e);
        const float w = (row < rows && k < in) ? ldexpf(W[(size_t)row * in + k], rexp[r]) : 0.f;
        pel q[F::kPlanes];
        split_planes<F>(w, q);
        const size_t base = ((size_t)(s * F::kPlanes) * 64 + lane) * 8 + e;
#pragma unroll
        for (int p = 0; p < F::kPlanes; ++p) o[base + (size_t)p * 64 * 8] = q[p];
    }
    float *bias = reinterpret_cast<float *>(out + bias_at);
    const int act_exp = layer == 1 ? 0 : F::kActScaleExp;  // layer 1 reads the observation unscaled
    if (threadIdx.x < 16) {  // scaled biases in row order, the row factors, the tanh factors, zero padding
        const int row = 16 * tile + threadIdx.x, ex = rexp[threadIdx.x] + act_exp;
        bias[threadIdx.x] = row < rows ? ldexpf(B[row], ex) : 0.f;
        bias[16 + threadIdx.x] = ldexpf(1.f, -ex);
        // 2 log2(e) * the row factor (exact: a power of two): tanh's exp2 argument straight from the
        // unscaled sum (tanh_fold)
        bias[32 + threadIdx.x] = ldexpf(kTwoLog2e, -ex);
    }
    for (int v = bias_at + 192 + 4 * threadIdx.x; v < kChunk; v += 4 * blockDim.x)
        *reinterpret_cast<uint32_t *>(out + v) = 0u;
    if (net == 1 && layer == 2 && tile == 0) {  // the critic's output layer as fp32 (evaluated on VALU)
        float *tail = reinterpret_cast<float *>(dst + (size_t)kAllChunks * kChunk);
        for (int k = threadIdx.x; k < 272; k += blockDim.x) tail[k] = k < kHid ? P.w3[k] : k == kHid ? P.b3[0] : 0.f;
    }
}
__global__ __launch_bounds__(256) void k_pack32(PackNet actor, PackNet critic, int with_critic, uint8_t *dst) {
    pack_chunk<FmtBf16x3>(actor, critic, with_critic, dst);
}
__global__ __launch_bounds__(256) void k_pack32h(PackNet actor, PackNet critic, int with_critic, uint8_t *dst) {
    pack_chunk<FmtF16x2>(actor, critic, with_critic, dst);
}

struct ActArgs {
    const int32_t *obs;
    const uint8_t *obs_u8;  // compact rows instead of obs (spl_step_args_t.obs_u8), or NULL
    const int8_t *mask;
    int32_t *action;
    float *logprob, *entropy, *value, *logits;
    const float *critic_out;
    uint64_t seed, ply;
    const uint64_t *ply_base;
    int64_t table0;
    int n;
    // grouped evaluation (spl_policy_act_grouped): tables sorted by network (order[n]), per group
    // g its first workgroup gtab[g] (g <= G) and its first position in order gtab[G + 1 + g]
    const int32_t *order;
    const int32_t *gtab;
    int groups;
    int64_t image_stride;
    // grouped launches: counts[G] | cursor[G] of the grouping scratch, zeroed by workgroup 0 for the
    // next call's k_group_count (k_group_place has consumed them)
    int32_t *group_reset;
};

// tanh in fp32 without branches, to a few ulp everywhere (the exact format's): |x| < 0.625:
// x + x^3 P(x^2), a degree-4 fit in x^2 (<= 0.9 ulp in fp32 Horner, checked over [0, 0.625]);
// otherwise 1 - 2 / (exp(2|x|) + 1) on v_exp_f32 / v_rcp_f32 (~1.5 ulp with correctly rounded exp2
// and rcp, a few ulp on the hardware's).  Both halves are evaluated and selected, so a tile's 64
// lanes never diverge.  (The exp form alone cancels near 0: its error is absolute, ~1e-7, so the
// relative error grows as |x| shrinks — ADVICE r04; the fp16-plane format keeps it, labelled.)
__device__ __forceinline__ float tanh_acc(float x) {
#if SPL_POL_ABL & 1
    return x;
#else
    const float ax = __builtin_fabsf(x);
    const float z = ax * ax;
    float p = -0.005718891508877277f;
    p = __builtin_fmaf(p, z, 0.02065306343138218f);
    p = __builtin_fmaf(p, z, -0.053744640201330185f);
    p = __builtin_fmaf(p, z, 0.13331513106822968f);
    p = __builtin_fmaf(p, z, -0.3333328664302826f);
    const float small = __builtin_fmaf(ax * z, p, ax);
    const float e = __builtin_amdgcn_exp2f(ax * kTwoLog2e);  // exp(2|x|)
    const float big = __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
    return __builtin_copysignf(ax < 0.625f ? small : big, x);
#endif
}

// the fp16-plane format's tanh, with the tile's row factor and the next layer's activation scale
// folded in: 2^S tanh(x u) for c = 2 log2(e) u, as 2^S (1 - 2 / (exp(2|x u|) + 1)) (u and 2^S powers of
// two; |x| c and |x u| 2 log2(e) are the same real product, rounded once): six VALU ops, two of them
// transcendental; absolute error ~1e-7
template <int S>
__device__ __forceinline__ float tanh_fold(float x, float c) {
#if SPL_POL_ABL & 1
    return x * (float)(1 << S);
#else
    const float e = __builtin_amdgcn_exp2f(__builtin_fabsf(x) * c);
    return __builtin_copysignf(__builtin_fmaf(-(float)(2 << S), __builtin_amdgcn_rcpf(e + 1.0f), (float)(1 << S)), x);
#endif
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
}

typedef __attribute__((address_space(3))) void lds_void;

// the image as a buffer resource: the chunk and block offsets go in the scalar offset, the lane's
// 16 bytes in a constant VGPR, so an LDS-DMA issue costs no VALU (the 64-bit per-lane address of
// global_load_lds took a v_lshl_add_u64 per load)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t image_rsrc(const uint8_t *W) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(W), (short)0, 0x7FFFFFF0, 0x00020000);
}
// wave w's share of a chunk: 1-KB blocks w, w + 8, w + 16, ... (64 lanes x 16 B each)
template <class F>
__device__ __forceinline__ void issue_chunk(__amdgpu_buffer_rsrc_t rs, int chunk, uint8_t *slot, int wave, int lane) {
    constexpr int kChunk = Geo<F>::kChunk, kBlocks = Geo<F>::kChunkBlocks;
#pragma unroll
    for (int i = 0; i < Geo<F>::kBlocksPerWave; ++i) {
        const int blk = wave + kWaves * i;
        if (blk < kBlocks)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void *)(slot + blk * 1024), 16, lane * 16,
                                                     chunk * kChunk + blk * 1024, 0, 0);
    }
}

// the VGPR-staged ring (SPL_P32_RINGV): wave w's 1-KB blocks of a chunk as 16-byte buffer loads into
// registers, then ds_write_b128 into the slot a tile later (an LDS-DMA piece holds the issuing wave's
// instruction issue ~60-185 cycles, MI355X_MICROARCH.md; a load plus a 16-byte LDS store, ~20)
template <class F>
__device__ __forceinline__ void stage_chunk(__amdgpu_buffer_rsrc_t rs, int chunk, u32x4 (&stg)[Geo<F>::kBlocksPerWave],
                                            int wave, int lane) {
#pragma unroll
    for (int i = 0; i < Geo<F>::kBlocksPerWave; ++i) {
        const int blk = wave + kWaves * i;
        if (blk < Geo<F>::kChunkBlocks)
            stg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, chunk * Geo<F>::kChunk + blk * 1024, 0));
    }
}
template <class F>
__device__ __forceinline__ void write_chunk(const u32x4 (&stg)[Geo<F>::kBlocksPerWave], uint8_t *slot, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < Geo<F>::kBlocksPerWave; ++i) {
        const int blk = wave + kWaves * i;
        if (blk < Geo<F>::kChunkBlocks) *reinterpret_cast<u32x4 *>(slot + blk * 1024 + lane * 16) = stg[i];
    }
}

// s_waitcnt immediate for vmcnt(n) alone (gfx9: vmcnt[3:0] in bits 3:0, vmcnt[5:4] in 15:14)
constexpr int vmcnt_imm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70; }

template <class F>
__device__ __forceinline__ f32x4 mma(const typename F::pelx8 &a, const typename F::pelx8 &b, const f32x4 &c) {
#if SPL_POL_ABL & 8
    return c + (float)a[0] * (float)b[1];
#elif SPL_POL_ABL & 512  // no MFMA and no stand-in instruction: the operands stay live, the sum is the bias
    f32x4 d = c;
    asm volatile("" : "+v"(d) : "v"(a), "v"(b));
    return d;
#else
    if constexpr (F::kExact) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
#endif
}

// The observation's residual plane for the exact format (observation values >= 256 are not exact in
// one bf16 plane): `mask` bit s is set when any table of the wave has such a value in k-step s
// (wave-uniform), and that k-step then adds the two products (w1 + w0) x the residual, rebuilt from
// the row (a rare path: the engine writes values >= 256 only for move counts above 255)
struct ObsHi {
    uint32_t mask;
    const int32_t *row32;
    const uint8_t *row8;
};

// one observation value k of a row (int32 row, or a compact row: byte k, move_count's high byte at 297)
__device__ __forceinline__ int obs_value(const int32_t *row32, const uint8_t *row8, int k) {
    if (k >= kObs) return 0;
    if (row32) return row32[k];
    int v = row8[k];
    if (k == 295) v += 256 * (int)row8[297];
    return v;
}

// the residual plane x - bf16(x) of k-step s, lane group g (exact for |x| < 2^16)
__device__ __forceinline__ bf16x8 obs_residual(const ObsHi &h, int s, int g) {
    bf16x8 q;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const float x = (float)obs_value(h.row32, h.row8, 32 * s + 8 * g + e);
        q[e] = (__bf16)(x - (float)(__bf16)x);
    }
    return q;
}

// one 16-row output tile: bias + sum over KS k-steps of 32 inputs, returned at the true scale (the
// row factors undo the planes' scaling).  B: NB planes of the layer's input (1: the observation,
// exact in one plane but for ObsHi's residual; kPlanes: a split hidden layer), in registers.  A: the
// tile's weight planes per k-step from `src` (the LDS ring slot, or the image in global memory for the
// narrow kernel), D k-steps ahead of the MFMAs that use them.
// kFold: the sum is returned as the products left it (scaled by the row factor's inverse) and
// `fold` gets the tile's tanh factors (tanh_fold) instead.
// `stage(s)` runs after k-step s's MFMAs, inside the same scheduling segment (SPL_P32_PIPE: the previous
// tile's epilogue, one stage per k-step, so its VALU work issues between this tile's MFMAs).
struct NoStage {
    __device__ __forceinline__ void operator()(int) const {}
};
template <class F, int KS, int NB, int D, bool kFold = false, class Stage = NoStage>
__device__ __forceinline__ f32x4 tile_mma(const uint8_t *src, const typename F::pelx8 (&B)[NB][KS], int lane,
                                          f32x4 *fold = nullptr, const ObsHi *hi = nullptr, Stage &&stage = Stage()) {
    typedef typename F::pelx8 pelx8;
    constexpr int kPlanes = F::kPlanes;
    static_assert(NB == 1 || NB == kPlanes, "planes");
    const float *bias = reinterpret_cast<const float *>(src + Geo<F>::bias_off(KS)) + 4 * (lane >> 4);
    f32x4 acc = {bias[0], bias[1], bias[2], bias[3]};
    const f32x4 unscale = {bias[16], bias[17], bias[18], bias[19]};
    if constexpr (kFold) *fold = f32x4{bias[32], bias[33], bias[34], bias[35]};
    const pelx8 *A = reinterpret_cast<const pelx8 *>(src) + lane;  // k-step s, plane p at A[(kPlanes s + p) * 64]
    if constexpr (NB == 1 && F::kExact) {
        // the observation's residual plane (rare, wave-uniform): x1 w1 + x1 w0 of each flagged k-step
        // first (the smaller terms), then the main products below
        if (hi && hi->mask) {
            for (uint32_t m = hi->mask; m; m &= m - 1) {
                const int s = __builtin_ctz(m);
                const bf16x8 x1 = obs_residual(*hi, s, lane >> 4);
                acc = mma<F>(A[(kPlanes * s + 1) * 64], x1, acc);
                acc = mma<F>(A[(kPlanes * s + 0) * 64], x1, acc);
            }
        }
    }
    constexpr int NR = D + 1;
    pelx8 af[NR][kPlanes];
#pragma unroll
    for (int q = 0; q < D && q < KS; ++q)
#pragma unroll
        for (int p = 0; p < kPlanes; ++p) af[q][p] = A[(kPlanes * q + p) * 64];
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        if (!(SPL_POL_ABL & 4) && s + D < KS) {
#pragma unroll
            for (int p = 0; p < kPlanes; ++p) af[(s + D) % NR][p] = A[(kPlanes * (s + D) + p) * 64];
        }
        const pelx8 *a = af[(SPL_POL_ABL & 4) ? s % D : s % NR];
        if constexpr (NB == 1) {  // exact B: (a2 b +) a1 b + a0 b
#pragma unroll
            for (int p = kPlanes - 1; p >= 0; --p) acc = mma<F>(a[p], B[0][s], acc);
        } else if constexpr (kPlanes == 2) {  // the three products of order <= 1, smallest first
            acc = mma<F>(a[1], B[0][s], acc);
            acc = mma<F>(a[0], B[1][s], acc);
            acc = mma<F>(a[0], B[0][s], acc);
        } else {  // the six products of order <= 2, smallest first
            acc = mma<F>(a[2], B[0][s], acc);
            acc = mma<F>(a[1], B[1][s], acc);
            acc = mma<F>(a[0], B[2][s], acc);
            acc = mma<F>(a[1], B[0][s], acc);
            acc = mma<F>(a[0], B[1][s], acc);
            acc = mma<F>(a[0], B[0][s], acc);
        }
        stage(s);
        if (NB > 1 || (s & 1) == 1) __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (F::kRowMaxExp != 0 && !kFold) acc *= unscale;  // exact: powers of two
    return acc;
}

// planes of a pelx8 as dwords: element e in dword e / 2 (even e in the low half)
template <class F>
__device__ __forceinline__ uint32_t pk2(typename F::pel lo, typename F::pel hi) {
    const typename F::pelx2 v = {lo, hi};
    return __builtin_bit_cast(uint32_t, v);
}

// the four fp32 outputs h[0..3] of tile t (units 16t + 4g + i), scaled by 2^kActScaleExp (exact) ->
// elements 4(t & 1) .. +3 of k-step t / 2 of the next layer's B planes
template <class F, bool kScaled = false>  // kScaled: h already carries 2^kActScaleExp (tanh_fold)
__device__ __forceinline__ void put_split(typename F::pelx8 (&H)[F::kPlanes][kKs2], int t, const float (&h)[4]) {
    typedef typename F::pel pel;
    typedef typename F::pelx8 pelx8;
    pel x[4][F::kPlanes];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        split_planes<F>((F::kActScaleExp && !kScaled) ? h[i] * (float)(1 << F::kActScaleExp) : h[i], x[i]);
#pragma unroll
    for (int p = 0; p < F::kPlanes; ++p) {
        u32x4 w = __builtin_bit_cast(u32x4, H[p][t >> 1]);
        w[2 * (t & 1)] = pk2<F>(x[0][p], x[1][p]);
        w[2 * (t & 1) + 1] = pk2<F>(x[2][p], x[3][p]);
        H[p][t >> 1] = __builtin_bit_cast(pelx8, w);
    }
}

// ---- the staged epilogue (SPL_P32_PIPE) ------------------------------------------------------------
// A tile's epilogue (tanh of its four pre-activations per lane, the split of the results into the next
// layer's B planes, or the critic's value FMAs) is issued in stages inside the NEXT tile's k-step loop:
// stage s after k-step s's MFMAs, so that its VALU work fills the MFMA pipe's issue gaps instead of
// following the tile's MFMA chain (where both waves of a SIMD would do VALU at once while the matrix
// core idles).  Same instructions, same results: a stage only reorders independent work.
// stages 0-3: tanh of value s; 4-5: the split of values (0, 1) / (2, 3) into the planes of tile t
template <class F>
struct PendTile {
    f32x4 acc, c;  // pre-activations as the products left them; tanh factors (fp16-plane format)
    float h[4];
};
template <class F>
__device__ __forceinline__ float pend_tanh(const PendTile<F> &q, int i) {
    if constexpr (F::kExact) return tanh_acc(q.acc[i]);
    else return tanh_fold<F::kActScaleExp>(q.acc[i], q.c[i]);
}
// split_planes of two values at once, each plane as the packed dword of the pair: one paired
// conversion per plane (v_cvt_pk_bf16_f32 rounds both to nearest even) and the residuals from the
// packed halves (the bf16 -> fp32 widening is a shift or a mask), 11 VALU ops per pair in the exact
// format instead of 15 for two single splits plus their packing
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <class F>
__device__ __forceinline__ void split_pair(float a, float b, uint32_t (&d)[F::kPlanes]) {
    typedef typename F::pelx2 pelx2;
#pragma unroll
    for (int p = 0; p < F::kPlanes; ++p) {
        const pelx2 q = __builtin_convertvector((f32x2){a, b}, pelx2);
        d[p] = __builtin_bit_cast(uint32_t, q);
        if (p + 1 < F::kPlanes) {  // exact in fp32; two scalar subtractions, not one v_pk_add_f32 (which
            a -= (float)q[0];       // costs a wave ~13 more issue cycles beside MFMAs, MI355X_MICROARCH.md)
            b -= (float)q[1];
        }
    }
}
// values (2 pair, 2 pair + 1) of tile t -> dword 2 (t & 1) + pair of k-step t / 2 of every plane
template <class F>
__device__ __forceinline__ void put_pair(typename F::pelx8 (&H)[F::kPlanes][kKs2], int t, int pair, float ha, float hb) {
    typedef typename F::pelx8 pelx8;
    uint32_t d[F::kPlanes];
    split_pair<F>(ha, hb, d);  // h carries 2^kActScaleExp already (tanh_fold) or needs none (exact)
#pragma unroll
    for (int p = 0; p < F::kPlanes; ++p) {
        u32x4 w = __builtin_bit_cast(u32x4, H[p][t >> 1]);
        w[2 * (t & 1) + pair] = d[p];
        H[p][t >> 1] = __builtin_bit_cast(pelx8, w);
    }
}
// Each stage's results are pinned where the stage stands (an empty asm that reads and rewrites them):
// left alone, the compiler sinks every tile's epilogue of a layer to the first use of its results — all
// 16 of them into the NEXT layer's first tile, one ~1 000-instruction VALU block during which the matrix
// cores idle (the round-4 kernel's schedule too, seen in its ISA: 16 MFMA-only tiles, then 385 VALU +
// 128 transcendental ops at the start of the next layer).
template <class F>
__device__ __forceinline__ void pin(typename F::pelx8 &x) {
    asm volatile("" : "+v"(x));
}
__device__ __forceinline__ void pin(float &x) { asm volatile("" : "+v"(x)); }
template <class F>
__device__ __forceinline__ void split_stage(typename F::pelx8 (&H)[F::kPlanes][kKs2], int t, PendTile<F> &q, int s) {
    if (s < 4) {
        q.h[s] = pend_tanh<F>(q, s);
        pin(q.h[s]);
    } else if (s == 4 || s == 5) {
        put_pair<F>(H, t, s - 4, q.h[2 * (s - 4)], q.h[2 * (s - 4) + 1]);
#pragma unroll
        for (int p = 0; p < F::kPlanes; ++p) pin<F>(H[p][t >> 1]);
    }
}
// the critic's output unit: value += w[s] tanh(pre-activation s), w = the tile's output weights of this
// lane group's units (16 t + 4 g ..; staged in LDS once per workgroup: loaded per tile from global
// memory the compiler hoisted all 16 tiles' loads and spilled)
template <class F>
__device__ __forceinline__ void value_stage(PendTile<F> &q, const float *w, float &value, int s) {
    if (s < 4) {
        float y;
        if constexpr (F::kExact) y = tanh_acc(q.acc[s]);
        else y = tanh_fold<0>(q.acc[s], q.c[s]);  // the critic's layer-2 units unscaled
        value = __builtin_fmaf(w[s], y, value);
        pin(value);
    }
}

// a tile's four pre-activations -> tanh (the format's), scaled for the next layer
template <class F, int KS, int NB, int D, typename Enter>
__device__ __forceinline__ void tile_tanh(Enter &enter, const typename F::pelx8 (&B)[NB][KS], int lane, float (&h)[4],
                                          const ObsHi *hi) {
    if constexpr (F::kExact) {
        const f32x4 acc = tile_mma<F, KS, NB, D>(enter(), B, lane, nullptr, hi);
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = tanh_acc(acc[i]);
    } else {
        f32x4 c;
        const f32x4 acc = tile_mma<F, KS, NB, D, true>(enter(), B, lane, &c);
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = tanh_fold<F::kActScaleExp>(acc[i], c[i]);
    }
}

// a hidden layer: 16 tiles, each tile's tanh split into the next layer's B planes
template <class F, int KS, int NB, int D, typename Enter>
__device__ __forceinline__ void layer_tanh(Enter &enter, const typename F::pelx8 (&B)[NB][KS],
                                           typename F::pelx8 (&H)[F::kPlanes][kKs2], int lane, const ObsHi *hi) {
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {
        float h[4];
        tile_tanh<F, KS, NB, D>(enter, B, lane, h, hi);
        put_split<F, true>(H, t, h);
    }
}

// the observation's B fragments: lane (r, g), k-step s, element e = obs[table r][32s + 8g + e] from an
// int32 row, or from a compact row (spl_step_args_t.obs_u8: 300 bytes, move_count >> 8 at byte 297:
// 8 bytes per k-step as two dword loads, k = 296 alone, k >= 297 zero).  The exact format also returns
// which k-steps hold a value the bf16 plane does not represent exactly (ObsHi.mask, wave-uniform).
template <class F>
__device__ __forceinline__ uint32_t load_obs(const int32_t *row32, const uint8_t *row8, int g,
                                             typename F::pelx8 (&X)[1][kKs1]) {
    typedef typename F::pel pel;
    typedef typename F::pelx8 pelx8;
    uint32_t hi = 0u;
#pragma unroll
    for (int s = 0; s < kKs1; ++s) {
        const int k0 = 32 * s + 8 * g;
        int v[8];
        if (row32) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int k = k0 + e;
                v[e] = k < kObs ? row32[k < kObs ? k : 0] : 0;
            }
        } else {
            const uint32_t *w = reinterpret_cast<const uint32_t *>(row8);
            uint32_t lo = 0u, hw = 0u;
            if (k0 + 7 < kObs) {
                lo = w[k0 >> 2];
                hw = w[(k0 >> 2) + 1];
            } else if (k0 < kObs) {  // k0 = 296 (s = 9, g = 1): byte 296 only
                lo = w[k0 >> 2] & 0xFFu;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = (int)((lo >> (8 * e)) & 0xFFu);
                v[4 + e] = (int)((hw >> (8 * e)) & 0xFFu);
            }
            if (k0 == 288) v[7] += 256 * (int)((w[74] >> 8) & 0xFFu);  // k = 295: move_count
        }
        bool big = false;
        if constexpr (F::kExact) {
#pragma unroll
            for (int e = 0; e < 8; ++e) big = big || (v[e] >= 256 || v[e] <= -256);
        }
        const u32x4 q = {pk2<F>((pel)(float)v[0], (pel)(float)v[1]), pk2<F>((pel)(float)v[2], (pel)(float)v[3]),
                         pk2<F>((pel)(float)v[4], (pel)(float)v[5]), pk2<F>((pel)(float)v[6], (pel)(float)v[7])};
        X[0][s] = __builtin_bit_cast(pelx8, q);
        if constexpr (F::kExact) hi |= __any(big) ? 1u << s : 0u;
    }
    return hi;
}

// A-plane prefetch depth (k-steps) in the ring kernel.  The scheduler places a k-step's LDS reads
// anywhere inside the previous k-step's segment (often after half its MFMAs), so one k-step ahead left
// ~3 MFMAs of distance to cover the LDS latency in the hidden layers
#ifndef SPL_P32_AHEAD2
#define SPL_P32_AHEAD2 2
#endif
constexpr int kAheadL1 = 2, kAheadHid = SPL_P32_AHEAD2;

// The per-table epilogue over one table's 45 logits (`row`) and mask bytes: greedy masked argmax
// (training_utils.py:263-276) or masked_categorical's sample, log-prob and entropy, plus the critic
// value (ppo_splendor.py:40-59).  Called by every lane of the wave: the four lanes r, r+16, r+32,
// r+48 (lane group g) share table r's row, lane group g taking actions 12g .. 12g+11, and combine
// through shuffles (one lane per table had left three quarters of the wave idle through 45 accurate
// expf and the sampling scan: ~7 % of the exact sample+critic kernel, timing ablation bit 32).
// Results: the greedy action is the same first maximum; the softmax sums are taken per lane group
// and then added ((S0 + S1) + (S2 + S3)), and the sampling scan of group g starts from the sum of the
// groups before it, so a draw can land on the other side of a boundary only where the two summation
// orders round differently.  Only lanes of group 0 with `ok` (a row of this wave) write.
template <bool kCritic, bool kSample>
__device__ __forceinline__ void act_epilogue4(const ActArgs &a, const float *row, const uint8_t *mrow, int64_t t,
                                              float value, int g, bool ok) {
    constexpr int kPer = 12;  // actions per lane group (45 = 12 + 12 + 12 + 9)
    const int k0 = kPer * g, r = threadIdx.x & 15;
    float lv[kPer];
    uint32_t legal = 0u, inr = 0u;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
        const int k = k0 + j;
        const bool in = k < kAct;
        lv[j] = in ? row[in ? k : 0] : 0.f;
        legal |= (uint32_t)(in && mrow[in ? k : 0] != 0) << j;
        inr |= (uint32_t)in << j;
    }
    int act;
    if constexpr (!kSample) {
        // logits.masked_fill(mask < 0.5, -inf).argmax(): first maximum; all-illegal -> 0
        float best = -__builtin_inff();
        int bk = kAct;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const bool better = ((legal >> j) & 1) && lv[j] > best;
            best = better ? lv[j] : best;
            bk = better ? k0 + j : bk;
        }
#pragma unroll
        for (int off = 16; off <= 32; off <<= 1) {  // larger value, then the smaller action
            const float ob = __shfl_xor(best, off);
            const int ok_ = __shfl_xor(bk, off);
            const bool take = ob > best || (ob == best && ok_ < bk);
            best = take ? ob : best;
            bk = take ? ok_ : bk;
        }
        act = bk < kAct ? bk : 0;
    } else {
        // masked_categorical: illegal -> -inf unless the row has no legal action; fp32 softmax
        int any = legal != 0u;
        any |= __shfl_xor(any, 16);
        any |= __shfl_xor(any, 32);
        const uint32_t allow = any ? legal : inr;
        float mx = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < kPer; ++j) mx = ((allow >> j) & 1) ? fmaxf(mx, lv[j]) : mx;
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        float Sg = 0.f, Tg = 0.f;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const float d = lv[j] - mx, p = ((allow >> j) & 1) ? expf(d) : 0.f;
            lv[j] = p;
            Sg += p;
            Tg += p * d;
        }
        float S = Sg + __shfl_xor(Sg, 16), T = Tg + __shfl_xor(Tg, 16);  // (S0 + S1), (S2 + S3)
        S += __shfl_xor(S, 32);
        T += __shfl_xor(T, 32);
        const float logS = logf(S);
        const uint64_t ply = a.ply + (a.ply_base ? *a.ply_base : 0ull);
        const uint4 rnd = philox4x32(make_uint4((uint32_t)(a.table0 + t), (uint32_t)((uint64_t)(a.table0 + t) >> 32),
                                                (uint32_t)ply, (uint32_t)(ply >> 32)),
                                     make_uint2((uint32_t)a.seed, (uint32_t)(a.seed >> 32) ^ 0xA5C3E1F7u));
        const float target = (float)(rnd.x >> 8) * (1.f / 16777216.f) * S;
        // the scan of group g starts from the groups before it, in order
        const float s0 = __shfl(Sg, r), s1 = __shfl(Sg, r + 16), s2 = __shfl(Sg, r + 32);
        float cum = g == 0 ? 0.f : g == 1 ? s0 : g == 2 ? s0 + s1 : (s0 + s1) + s2;
        int hk = kAct, last = -1;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            const bool al = (allow >> j) & 1;
            cum += lv[j];
            last = al ? k0 + j : last;
            hk = (al && hk == kAct && cum > target) ? k0 + j : hk;
        }
#pragma unroll
        for (int off = 16; off <= 32; off <<= 1) {  // the first hit over the groups; the last allowed action
            hk = min(hk, __shfl_xor(hk, off));
            last = max(last, __shfl_xor(last, off));
        }
        act = hk < kAct ? hk : (last >= 0 ? last : 0);
        if (g == 0 && ok) {
            if (a.logprob) a.logprob[t] = row[act] - mx - logS;
            if (a.entropy) a.entropy[t] = logS - T / S;
            if (kCritic) a.value[t] = value;
        }
    }
    if (g == 0 && ok) a.action[t] = act;
}

// <false, false> greedy actor, <false, true> sampling actor, <true, true> critic + sampling actor
// (get_action_and_value), <true, false> critic only (ActorCritic.get_value, ppo_splendor.py:51)
template <class F, bool kCritic, bool kSample>
__device__ __forceinline__ void act32_body(const uint8_t *__restrict__ W, ActArgs a) {
    typedef typename F::pelx8 pelx8;
    typedef Geo<F> G;
    constexpr int kSlots = F::kSlots, kChunk = G::kChunk;
    __shared__ __attribute__((aligned(16))) uint8_t lds[G::kLds];
    constexpr bool kActor = kSample || !kCritic;
    constexpr int kTotal = kCritic ? (kActor ? kAllChunks : kCriticChunks) : kActorChunks;
    // the wave index made wave-uniform for the compiler (SGPR), so the ring's LDS slot addresses stay
    // scalar (M0 of the LDS-DMA loads) instead of readfirstlane'd VGPR arithmetic per load
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, r = lane & 15,
              g = lane >> 4;
    // rows [rbase, rend) of this workgroup: tables rbase.. directly, or positions of the grouped
    // order (one network per workgroup: the group whose workgroup range holds blockIdx.x)
    int64_t rbase = (int64_t)blockIdx.x * kRowsPerBlock, rend = a.n;
    if (a.group_reset && blockIdx.x == 0 && threadIdx.x < 2 * a.groups) a.group_reset[threadIdx.x] = 0;
    if (a.order) {
        const int b = (int)blockIdx.x;
        if (b >= a.gtab[a.groups]) return;  // past the last group's workgroups (every wave leaves)
        int grp = 0;
        for (int i = 1; i < a.groups; ++i) grp = a.gtab[i] <= b ? i : grp;
        W += (size_t)grp * a.image_stride;
        const int64_t first = a.gtab[a.groups + 1 + grp];
        rbase = first + (int64_t)(b - a.gtab[grp]) * kRowsPerBlock;
        rend = a.gtab[a.groups + 2 + grp];
    }
    const int64_t tbase = rbase + wave * kRowsPerWave;
    const int valid = (int)max<int64_t>(0, min<int64_t>(kRowsPerWave, rend - tbase));
    // table of row i of this wave (i < valid)
    auto table_of = [&](int i) -> int64_t { return a.order ? (int64_t)a.order[tbase + i] : tbase + i; };
    uint8_t *ring = lds;
    uint8_t *ms = lds + G::kLdsMask + wave * kMaskWave;
    const __amdgpu_buffer_rsrc_t wrs = image_rsrc(W);

#if SPL_P32_GROUP == 2
    static_assert(kSlots == 4, "two chunks per barrier: four slots");
    issue_chunk<F>(wrs, 0, ring, wave, lane);
    issue_chunk<F>(wrs, 1, ring + kChunk, wave, lane);
#elif SPL_P32_RINGV
    // VGPR-staged ring (SPL_P32_RINGV): chunks 0 .. S-3 by LDS-DMA, chunk S-2 into this wave's staging
    // registers; enter(c) writes the staged chunk c+S-2 into its slot and loads chunk c+S-1
    u32x4 stg[G::kBlocksPerWave];
#pragma unroll
    for (int c = 0; c < kSlots - 2; ++c) issue_chunk<F>(wrs, c, ring + c * kChunk, wave, lane);
    stage_chunk<F>(wrs, kSlots - 2 < kTotal ? kSlots - 2 : kTotal - 1, stg, wave, lane);
#else
#pragma unroll
    for (int c = 0; c < kSlots - 1; ++c) issue_chunk<F>(wrs, c, ring + c * kChunk, wave, lane);
#endif

    // grouped rows: the wave's table ids, one load (lane i < valid holds row i's), then shuffles
    const int32_t tid_own = (a.order && lane < valid) ? a.order[tbase + lane] : 0;
    // observation B fragments (load_obs)
    const int64_t xt = valid > 0 ? (a.order ? (int64_t)__shfl(tid_own, r < valid ? r : 0) : tbase + (r < valid ? r : 0)) : 0;
    pelx8 X[1][kKs1];
    ObsHi hi{0u, a.obs_u8 ? nullptr : a.obs + (size_t)xt * kObs, a.obs_u8 ? a.obs_u8 + (size_t)xt * 300 : nullptr};
#if SPL_POL_ABL & 64  // timing ablation: no observation loads (zero operand planes)
#pragma unroll
    for (int s = 0; s < kKs1; ++s) X[0][s] = pelx8{};
    hi.mask = 0u;
#else
    hi.mask = load_obs<F>(hi.row32, hi.row8, g, X);
#endif
    if constexpr (!kActor) {
        // get_value: no mask
    } else if (a.order) {
        // gathered rows: every mask byte of the wave's rows in one batch of independent loads (a
        // loop reading order[] per byte was two dependent round trips per iteration, ~12 of them)
        constexpr int kMI = (kMaskWave + 63) / 64;  // 12
        uint32_t mv[kMI];
#pragma unroll
        for (int i = 0; i < kMI; ++i) {
            const int e = lane + 64 * i, row = e / kAct;
            const int32_t tt = __shfl(tid_own, row < kRowsPerWave ? row : 0);
            mv[i] = e < valid * kAct ? (uint32_t)(uint8_t)a.mask[(int64_t)tt * kAct + e % kAct] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kMI; ++i) {
            const int e = lane + 64 * i;
            if (e < valid * kAct) ms[e] = (uint8_t)mv[i];
        }
    } else if (valid == kRowsPerWave) {
        constexpr int kMQ = kMaskWave / 4;  // 180 dwords
        const uint32_t *msrc = reinterpret_cast<const uint32_t *>(a.mask + tbase * kAct);
        for (int q = lane; q < kMQ; q += 64) reinterpret_cast<uint32_t *>(ms)[q] = msrc[q];
    } else {
        const int8_t *msrc = a.mask + tbase * kAct;
        for (int e = lane; e < valid * kAct; e += 64) ms[e] = (uint8_t)msrc[e];
    }

    int c = 0;
#if SPL_P32_SPREAD
    static_assert(SPL_P32_GROUP == 2 && SPL_P32_PIPE, "spread pieces ride the pipelined k-steps of the group-2 ring");
    // even tile c loads the next pair, chunks c+2 and c+3 (their slots held c-2 and c-1, free since the
    // barrier of c), which the barrier of c+2 waits for: a tile or more after the last piece is issued.
    // Pieces 0 .. kLast-1 of each chunk (blocks wave + 8 i, which every wave and layer has) one per
    // k-step from k-step 0, branch-free (a branch would end the scheduling region between a k-step's
    // MFMAs and the epilogue stage that should interleave with them; a chunk past the image's last
    // re-loads that last chunk into its free slot); the last piece after the tile's last k-step, where
    // a branch splits nothing, by the waves whose block the chunk's layer has (layer 1: all but the
    // last; a hidden layer: its bias block, wave 0).  Odd tiles load nothing.
    int dnext = 0;
    auto tick = [&](int s, int ks, int odd) {  // after k-step s of a tile of ks k-steps (s, ks, odd known at compile time)
        constexpr int kLast = G::kBlocksPerWave - 1;
        constexpr bool kNoStream = (SPL_POL_ABL & 2) != 0;  // ablation 2: no streaming at all
        if (odd || kNoStream) return;
        if (s < 2 * kLast) {
            const int j = s / kLast, blk = wave + kWaves * (s % kLast), ch = min(dnext + j, kTotal - 1);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void *)(ring + ((dnext + j) % kSlots) * kChunk + blk * 1024),
                                                     16, lane * 16, ch * kChunk + blk * 1024, 0, 0);
        }
        if (s == ks - 1) {
            const int blk = wave + kWaves * kLast;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int ch = dnext + j;
                const bool l1 = (kCritic && ch >= kCriticChunks ? ch - kCriticChunks : ch) < kTiles;
                if (ch < kTotal && blk < (l1 ? G::blocks(kKs1) : G::blocks(kKs2)))
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(wrs, (lds_void *)(ring + (ch % kSlots) * kChunk + blk * 1024), 16,
                                                             lane * 16, ch * kChunk + blk * 1024, 0, 0);
            }
        }
    };
#else
    auto tick = [&](int, int, int) {};
#endif
    auto enter = [&]() -> const uint8_t * {
#if SPL_POL_ABL & 2
        if (c++ == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        return ring;
#endif
#if SPL_P32_GROUP == 2
        // two chunks per barrier: on even c, wait for this wave's pieces of chunks c, c+1 (issued two tiles
        // ago), barrier (everyone's landed; everyone is done with c-2, c-1), then issue c+2, c+3 into their
        // slots; odd c just moves on to the next slot
        if ((c & 1) == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (!(SPL_POL_ABL & 16)) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
#if !SPL_P32_SPREAD
#pragma unroll
            for (int j = 2; j < 4; ++j)
                if (c + j < kTotal) issue_chunk<F>(wrs, c + j, ring + ((c + j) % kSlots) * kChunk, wave, lane);
#endif
        }
#elif SPL_P32_RINGV
        // the staged chunk c+S-2 (loaded one tile ago) -> its slot, which held chunk c-2 (every wave was
        // done with it at the previous barrier); then, behind this barrier, chunk c is complete (written
        // S-2 tiles ago, or by the prologue's LDS-DMA) and every wave is done with chunk c-1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (c + kSlots - 2 < kTotal) write_chunk<F>(stg, ring + ((c + kSlots - 2) % kSlots) * kChunk, wave, lane);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's part of it is in LDS
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (c + kSlots - 1 < kTotal) stage_chunk<F>(wrs, c + kSlots - 1, stg, wave, lane);
#else
        // this wave's part of chunk c landed (later chunks' loads may stay outstanding)
        if (wave < G::kChunkBlocks - (G::kBlocksPerWave - 1) * kWaves) __builtin_amdgcn_s_waitcnt(vmcnt_imm(G::kWaitMost));
        else __builtin_amdgcn_s_waitcnt(vmcnt_imm(G::kWaitLast));
        if (!(SPL_POL_ABL & 16)) __builtin_amdgcn_s_barrier();  // everyone's part landed; slot c-1 is free
        asm volatile("" ::: "memory");
        const int nxt = c + kSlots - 1 < kTotal ? c + kSlots - 1 : kTotal - 1;  // past the end: harmless reload
        issue_chunk<F>(wrs, nxt, ring + ((c + kSlots - 1) % kSlots) * kChunk, wave, lane);
#endif
        const uint8_t *slot = ring + (c % kSlots) * kChunk;
#if SPL_P32_SPREAD
        dnext = c + 2;
#endif
        ++c;
        return slot;
    };

    pelx8 H1[F::kPlanes][kKs2];
    float value = 0.f;
#if SPL_P32_PIPE
    // each tile's epilogue runs in stages inside the next tile's k-steps (PendTile; the last tile of a
    // layer inside the next layer's first tile, before that tile's k-step 7 reads the planes it writes)
    constexpr bool kFoldP = !F::kExact;
    PendTile<F> q;
    const float *crit = reinterpret_cast<const float *>(lds + G::kLdsCritic);  // the critic's output layer
    if constexpr (kCritic) {
        float *cw = reinterpret_cast<float *>(lds + G::kLdsCritic);
        for (int k = threadIdx.x; k < kCriticTail / 4; k += kWaves * 64) cw[k] = a.critic_out[k];
        // visible to every wave after the first ring barrier (enter)
#pragma unroll
        for (int t = 0; t < kTiles; ++t) {  // critic layer 1 -> H1
            f32x4 cf;
            const f32x4 acc = tile_mma<F, kKs1, 1, kAheadL1, kFoldP>(enter(), X, lane, &cf, &hi, [&](int s) {
                tick(s, kKs1, t & 1);
                if (t > 0) split_stage<F>(H1, t - 1, q, s);
            });
            q.acc = acc;
            q.c = cf;
        }
        {  // critic layer 2 -> its tiles' shares of the output unit; tile 0 finishes layer 1's last tile
            f32x4 cf;
            const f32x4 acc = tile_mma<F, kKs2, F::kPlanes, kAheadHid, kFoldP>(enter(), H1, lane, &cf, nullptr, [&](int s) {
                tick(s, kKs2, 0);
                split_stage<F>(H1, kTiles - 1, q, s);
            });
            q.acc = acc;
            q.c = cf;
        }
        auto crit_l2 = [&](int t, int odd) {
            f32x4 cf;
            const f32x4 acc = tile_mma<F, kKs2, F::kPlanes, kAheadHid, kFoldP>(enter(), H1, lane, &cf, nullptr, [&](int s) {
                tick(s, kKs2, odd);
                value_stage<F>(q, crit + 16 * (t - 1) + 4 * g, value, s);
            });
            q.acc = acc;
            q.c = cf;
        };
        crit_l2(1, 1);
#pragma unroll 1
        for (int t = 2; t < kTiles; t += 2) {  // one loop body of an even and an odd tile (as round 4's
            crit_l2(t, 0);                     // critic layer 2: no register array is indexed by t here)
            crit_l2(t + 1, 1);
        }
    }
    if constexpr (!kActor) {
#pragma unroll
        for (int s = 0; s < 4; ++s) value_stage<F>(q, crit + 16 * (kTiles - 1) + 4 * g, value, s);  // the last tile's share
        value += __shfl_xor(value, 16);  // the other lane groups' units, then the bias
        value += __shfl_xor(value, 32);
        value += crit[kHid];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing reloads land while the LDS is ours
        if (g == 0 && r < valid) a.value[table_of(r)] = value;
        return;
    }
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {  // actor layer 1 -> H1 (the critic's layer 2 has read H1 by now)
        f32x4 cf;
        const f32x4 acc = tile_mma<F, kKs1, 1, kAheadL1, kFoldP>(enter(), X, lane, &cf, &hi, [&](int s) {
            tick(s, kKs1, t & 1);
            if (t > 0) split_stage<F>(H1, t - 1, q, s);
            else if (kCritic) value_stage<F>(q, crit + 16 * (kTiles - 1) + 4 * g, value, s);
        });
        q.acc = acc;
        q.c = cf;
    }
    if constexpr (kCritic) {
        value += __shfl_xor(value, 16);
        value += __shfl_xor(value, 32);
        value += crit[kHid];
    }
    pelx8 H2[F::kPlanes][kKs2];
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {  // actor layer 2 -> H2
        f32x4 cf;
        const f32x4 acc = tile_mma<F, kKs2, F::kPlanes, kAheadHid, kFoldP>(enter(), H1, lane, &cf, nullptr, [&](int s) {
            tick(s, kKs2, t & 1);
            if (t == 0) split_stage<F>(H1, kTiles - 1, q, s);
            else split_stage<F>(H2, t - 1, q, s);
        });
        q.acc = acc;
        q.c = cf;
    }
    f32x4 L[kActTiles];
#pragma unroll
    for (int t = 0; t < kActTiles; ++t)  // the logits (true scale)
        L[t] = tile_mma<F, kKs2, F::kPlanes, kAheadHid>(enter(), H2, lane, nullptr, nullptr, [&](int s) {
            tick(s, kKs2, t & 1);
            if (t == 0) split_stage<F>(H2, kTiles - 1, q, s);
        });
#else
    if constexpr (kCritic) {
        layer_tanh<F, kKs1, 1, kAheadL1>(enter, X, H1, lane, &hi);
        // layer 2 tile t -> tanh -> its units' share of the fp32 output unit, on the spot
#pragma unroll 1
        for (int t = 0; t < kTiles; ++t) {
            const float4 w = *reinterpret_cast<const float4 *>(a.critic_out + 16 * t + 4 * g);
            float h[4];
            if constexpr (F::kExact) {
                const f32x4 acc = tile_mma<F, kKs2, F::kPlanes, kAheadHid>(enter(), H1, lane);
#pragma unroll
                for (int i = 0; i < 4; ++i) h[i] = tanh_acc(acc[i]);
            } else {
                f32x4 cf;
                const f32x4 acc = tile_mma<F, kKs2, F::kPlanes, kAheadHid, true>(enter(), H1, lane, &cf);
#pragma unroll
                for (int i = 0; i < 4; ++i) h[i] = tanh_fold<0>(acc[i], cf[i]);
            }
            value = __builtin_fmaf(w.x, h[0], value);
            value = __builtin_fmaf(w.y, h[1], value);
            value = __builtin_fmaf(w.z, h[2], value);
            value = __builtin_fmaf(w.w, h[3], value);
        }
        value += __shfl_xor(value, 16);  // the other lane groups' units, then the bias
        value += __shfl_xor(value, 32);
        value += a.critic_out[kHid];
    }
    if constexpr (!kActor) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing reloads land while the LDS is ours
        if (g == 0 && r < valid) a.value[table_of(r)] = value;
        return;
    }
    layer_tanh<F, kKs1, 1, kAheadL1>(enter, X, H1, lane, &hi);
    pelx8 H2[F::kPlanes][kKs2];
    layer_tanh<F, kKs2, F::kPlanes, kAheadHid>(enter, H1, H2, lane, nullptr);
    f32x4 L[kActTiles];
#pragma unroll
    for (int t = 0; t < kActTiles; ++t) L[t] = tile_mma<F, kKs2, F::kPlanes, kAheadHid>(enter(), H2, lane);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing reloads
    __builtin_amdgcn_s_barrier();                      // every wave is done with the ring

    // logits -> LDS [table][action] (reusing the ring), then the per-table epilogue
    float *lg = reinterpret_cast<float *>(ring) + wave * kRowsPerWave * kLogitRow;
#pragma unroll
    for (int t = 0; t < kActTiles; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int act = 16 * t + 4 * g + i;
            if (act < kAct) lg[r * kLogitRow + act] = L[t][i];
        }
    wave_lds_sync();
    if (a.logits) {
        for (int i = lane; i < valid * kAct; i += 64)
            a.logits[table_of(i / kAct) * kAct + i % kAct] = lg[(i / kAct) * kLogitRow + i % kAct];
    }
    if (SPL_POL_ABL & 32) {  // timing ablation: no per-table epilogue (action 0, value only)
        if (g == 0 && r < valid) {
            a.action[table_of(r)] = 0;
            if (kCritic) a.value[table_of(r)] = value;
        }
        return;
    }
    act_epilogue4<kCritic, kSample>(a, lg + r * kLogitRow, ms + r * kAct, r < valid ? table_of(r) : 0, value, g, r < valid);
}

// the exact format's kernels keep round 3-4's names (k_act32<critic, sample>), the fp16-plane ones are k_act32h
template <bool kCritic, bool kSample>
__global__ __launch_bounds__(kWaves * 64) void k_act32(const uint8_t *__restrict__ W, ActArgs a) {
    act32_body<FmtBf16x3, kCritic, kSample>(W, a);
}
template <bool kCritic, bool kSample>
__global__ __launch_bounds__(kWaves * 64) void k_act32h(const uint8_t *__restrict__ W, ActArgs a) {
    act32_body<FmtF16x2, kCritic, kSample>(W, a);
}

// ---- narrow workgroups: the tails of the grouped evaluation ----------------------------------
// 65 536 tables fill exactly two rounds of one 128-table workgroup per CU, so the partial last
// workgroup of every network (the group's tail) used to spill into a third round that took a whole
// round's time (each wave's MFMA chain is latency-bound, however few tables it carries).  A group's
// full 128-table workgroups stay in k_act32; its tail runs here in wave-tiles of 16 tables, ONE
// wave-tile per 8-wave workgroup, the 16 output tiles of each hidden layer split over the waves
// (wave w: tiles w, w + 8), the weights read straight from the image (L2-resident, shared by every
// workgroup of the network; tile_mma with the A planes kAheadGlobal k-steps ahead), and each
// layer's outputs exchanged through LDS.  A tail wave-tile takes a small fraction of a full
// workgroup's time (5 tile chains per wave instead of 35).
// (8 k-steps ahead measured the same 21.7-22.0 us per call in config 5: the three layers' ~16 us are the
// ~1 MB of one network's weights that every tail workgroup pulls through its CU, not the load latency;
// profiles/r05/narrow_tail_r05zx_zy.txt)
constexpr int kAheadGlobal = 3;

constexpr int kNarrowWaves = 8;  // two hidden-layer tiles per wave (2 waves per SIMD: room for the A fragments)

// one hidden layer split over the waves (wave w: tiles w and w + 8), then every wave gathers all
// 16 tiles' tanh outputs (its next layer's B fragments) from LDS
template <class F, int KS, int NB>
__device__ __forceinline__ void narrow_layer(const uint8_t *W, int chunk0, const typename F::pelx8 (&B)[NB][KS],
                                             typename F::pelx8 (&H)[F::kPlanes][kKs2], float *xbuf, int wave, int lane,
                                             const ObsHi *hi) {
#pragma unroll
    for (int h = 0; h < kTiles / kNarrowWaves; ++h) {
        const int t = wave + kNarrowWaves * h;
        const f32x4 acc = tile_mma<F, KS, NB, kAheadGlobal>(W + (size_t)(chunk0 + t) * Geo<F>::kChunk, B, lane, nullptr, hi);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float y;
            if constexpr (F::kExact) y = tanh_acc(acc[i]);
            else y = tanh_fold<0>(acc[i], kTwoLog2e);  // acc is at the true scale here (no fold)
            xbuf[(4 * t + i) * 64 + lane] = y;
        }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < kTiles; ++t) {
        float h[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) h[i] = xbuf[(4 * t + i) * 64 + lane];
        put_split<F>(H, t, h);
    }
    __syncthreads();  // xbuf is written again by the next layer
}

template <class F, bool kSample>
__device__ __forceinline__ void act32_narrow_body(const uint8_t *__restrict__ Wbase, ActArgs a) {
    typedef typename F::pelx8 pelx8;
    __shared__ __attribute__((aligned(16))) float xbuf[kTiles * 4 * 64];  // 16 KB: one layer's outputs
    __shared__ float lg[kRowsPerWave * kLogitRow];
    __shared__ uint8_t ms[kMaskWave];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, r = lane & 15, g = lane >> 4;
    const int b = (int)blockIdx.x, G = a.groups;
    // this workgroup's (network, tile of its tail) from the XCD-aware map k_group_place wrote (round 6):
    // every tile of one network's tail runs on ONE XCD (blocks b and b + 8 share one), so the network's
    // image is pulled into that XCD's L2 once and its other tiles hit there; -1: no tile (leave)
    const int e = a.order[(size_t)a.n + b];
    if (e < 0) return;
    const int grp = e >> 8, tile = e & 255;
    const uint8_t *W = Wbase + (size_t)grp * a.image_stride;
    const int64_t gfirst = a.gtab[G + 1 + grp], gend = a.gtab[G + 2 + grp];
    const int64_t tbase = gfirst + (gend - gfirst) / kRowsPerBlock * kRowsPerBlock + (int64_t)tile * kRowsPerWave;
    const int valid = (int)max<int64_t>(0, min<int64_t>(kRowsPerWave, gend - tbase));
    const int32_t tid_own = lane < valid ? a.order[tbase + lane] : 0;
    const int64_t xt = valid > 0 ? (int64_t)__shfl(tid_own, r < valid ? r : 0) : 0;
#if SPL_POL_ABL & 128  // timing ablation: the narrow kernel's launch and index lookups only
    if (tid_own == -12345) a.action[0] = (int32_t)xt;
    return;
#endif
    pelx8 X[1][kKs1];
    ObsHi hi{0u, a.obs_u8 ? nullptr : a.obs + (size_t)xt * kObs, a.obs_u8 ? a.obs_u8 + (size_t)xt * 300 : nullptr};
    hi.mask = load_obs<F>(hi.row32, hi.row8, g, X);
    if (wave == 0) {  // the wave-tile's mask bytes (gathered rows), for the epilogue
        constexpr int kMI = (kMaskWave + 63) / 64;
        uint32_t mv[kMI];
#pragma unroll
        for (int i = 0; i < kMI; ++i) {
            const int e = lane + 64 * i, row = e / kAct;
            const int32_t tt = __shfl(tid_own, row < kRowsPerWave ? row : 0);
            mv[i] = e < valid * kAct ? (uint32_t)(uint8_t)a.mask[(int64_t)tt * kAct + e % kAct] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kMI; ++i) {
            const int e = lane + 64 * i;
            if (e < valid * kAct) ms[e] = (uint8_t)mv[i];
        }
    }
    pelx8 H1[F::kPlanes][kKs2], H2[F::kPlanes][kKs2];
#if SPL_POL_ABL & 256  // timing ablation: no layers (zero logits), the loads and the epilogue only
    if (wave < kActTiles) {
        for (int i = 0; i < 4; ++i) {
            const int act = 16 * wave + 4 * g + i;
            if (act < kAct) lg[r * kLogitRow + act] = (float)X[0][0][i] * 0.f;
        }
    }
    (void)H1;
    (void)H2;
    (void)W;
    if (false) {
#else
    {
#endif
    narrow_layer<F>(W, 0, X, H1, xbuf, wave, lane, &hi);
    narrow_layer<F>(W, kTiles, H1, H2, xbuf, wave, lane, nullptr);
    if (wave < kActTiles) {  // logits: waves 0..2 take one 16-row tile each
        const f32x4 L = tile_mma<F, kKs2, F::kPlanes, kAheadGlobal>(W + (size_t)(2 * kTiles + wave) * Geo<F>::kChunk, H2, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int act = 16 * wave + 4 * g + i;
            if (act < kAct) lg[r * kLogitRow + act] = L[i];
        }
    }
    }
    __syncthreads();
    if (wave == 0 && a.logits) {
        for (int i = lane; i < valid * kAct; i += 64)
            a.logits[(int64_t)a.order[tbase + i / kAct] * kAct + i % kAct] = lg[(i / kAct) * kLogitRow + i % kAct];
    }
    if (wave == 0) {
        const int64_t tab = (int64_t)__shfl(tid_own, r);
        act_epilogue4<false, kSample>(a, lg + r * kLogitRow, ms + r * kAct, tab, 0.f, g, r < valid);
    }
}
template <bool kSample>
__global__ __launch_bounds__(kNarrowWaves * 64) void k_act32_narrow(const uint8_t *__restrict__ W, ActArgs a) {
    act32_narrow_body<FmtBf16x3, kSample>(W, a);
}
template <bool kSample>
__global__ __launch_bounds__(kNarrowWaves * 64) void k_act32h_narrow(const uint8_t *__restrict__ W, ActArgs a) {
    act32_narrow_body<FmtF16x2, kSample>(W, a);
}

}  // namespace splp32

using namespace splp32;

// ---- host side: fmt 0 = exact three bf16 planes (SPL_PREC_FP32), 1 = two fp16 planes (SPL_PREC_FP32_F16X2)
int64_t splp32_bytes(int with_critic, int fmt) {
    const int64_t chunk = fmt ? Geo<FmtF16x2>::kChunk : Geo<FmtBf16x3>::kChunk;
    return with_critic ? (int64_t)kAllChunks * chunk + kCriticTail : (int64_t)kActorChunks * chunk;
}

int splp32_pack(const spl_mlp_t *actor, const spl_mlp_t *critic, void *packed, void *stream, int fmt) {
    const PackNet A{actor->w1, actor->b1, actor->w2, actor->b2, actor->w3, actor->b3, kAct};
    const PackNet C = critic ? PackNet{critic->w1, critic->b1, critic->w2, critic->b2, critic->w3, critic->b3, 1} : A;
    if (fmt)
        hipLaunchKernelGGL(k_pack32h, dim3(critic ? kAllChunks : kActorChunks), dim3(256), 0, (hipStream_t)stream, A, C,
                           critic ? 1 : 0, static_cast<uint8_t *>(packed));
    else
        hipLaunchKernelGGL(k_pack32, dim3(critic ? kAllChunks : kActorChunks), dim3(256), 0, (hipStream_t)stream, A, C,
                           critic ? 1 : 0, static_cast<uint8_t *>(packed));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return spl_fail(SPL_E_HIP, std::string("k_pack32 launch: ") + hipGetErrorString(e));
    return SPL_OK;
}

// ---- grouping: counting sort of tables by network ------------------------------------------
// scratch (int32): counts[G] | cursor[G] | gtab[2G + 2] (workgroup starts G+1, order starts G+1) | order[n]
__global__ __launch_bounds__(256) void k_group_count(int n, int G, const int32_t *group_of, int32_t *counts) {
    __shared__ int32_t h[64];
    if (threadIdx.x < 64) h[threadIdx.x] = 0;
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int g = group_of[i];
        if (g >= 0 && g < G) atomicAdd(&h[g], 1);
    }
    __syncthreads();
    if (threadIdx.x < G && h[threadIdx.x]) atomicAdd(&counts[threadIdx.x], h[threadIdx.x]);
}

// Tables into their group's range of `order` (order within a group is irrelevant), the group scan
// included: every workgroup derives the groups' starts from the final counts itself (G <= 64, one
// pass by one thread) instead of a separate one-thread scan launch (a launch of its own cost ~4.6 us
// in the config-5 dual step's trace).  Ranks are taken in LDS and each workgroup reserves its span of
// every group with ONE global atomic on cursor[g] (relative to the group's start): one global atomic
// per table on a dozen hot addresses serialises in L2 (about 0.3 ms for 65 536 tables over 13
// groups).  Workgroup 0 writes the launch tables: gtab[g] the group's first full (128-table)
// workgroup of k_act32, gtab[G + 1 + g] its first position in `order`, ntab[g] its first narrow
// (16-table tail) workgroup of k_act32_narrow.  The grouped k_act32 launch that follows zeroes
// counts and cursors for the next call's k_group_count (ActArgs.group_reset: no memset launch, and
// no last-workgroup ticket here — 256 serialised atomics on one word cost this kernel ~7 us).
// narrow workgroups launched per grouped call: 8 XCDs x (tiles of at most ceil(G / 8) networks, 8 each)
static_assert(kRowsPerBlock / kRowsPerWave == 8, "a tail holds at most 8 sixteen-table tiles");
__host__ __device__ constexpr int narrow_grid(int G) { return 64 * ((G + 7) / 8); }
__global__ __launch_bounds__(256) void k_group_place(int n, int G, const int32_t *group_of, const int32_t *counts,
                                                     int32_t *cursor, int32_t *gtab, int32_t *order) {
    __shared__ int32_t cnt[64], base[64], start[64], tot[64];
    if (threadIdx.x < 64) cnt[threadIdx.x] = 0;
    int32_t *const nmap = order + n;  // narrow block -> (network << 8 | tail tile), -1 none
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < narrow_grid(G); i += 256) nmap[i] = -1;
    if (threadIdx.x < G) tot[threadIdx.x] = counts[threadIdx.x];  // one batch of loads, not G dependent trips
    __syncthreads();
    if (threadIdx.x == 0) {
        int pos = 0;
        for (int g = 0; g < G; ++g) {
            start[g] = pos;
            pos += tot[g];
        }
        if (blockIdx.x == 0) {
            int32_t *ntab = gtab + 2 * G + 2;
            int wg = 0, nw = 0;
            for (int g = 0; g < G; ++g) {
                const int c = tot[g];
                gtab[g] = wg;
                ntab[g] = nw;
                gtab[G + 1 + g] = start[g];
                wg += c / kRowsPerBlock;
                nw += (c % kRowsPerBlock + kRowsPerWave - 1) / kRowsPerWave;
            }
            gtab[G] = wg;
            ntab[G] = nw;
            gtab[2 * G + 1] = pos;
        }
    }
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x < 8) {
        // the tails' tiles, XCD-aware, one thread per XCD x: network g's tiles on XCD g % 8 (blocks
        // 8 s + g % 8, consecutive s); written after every thread's -1 above (two barriers since)
        const int x = threadIdx.x;
        int fill = 0;
        for (int g = x; g < G; g += 8) {
            const int tiles = (tot[g] % kRowsPerBlock + kRowsPerWave - 1) / kRowsPerWave;
            for (int i = 0; i < tiles; ++i) nmap[8 * (fill + i) + x] = g << 8 | i;
            fill += tiles;
        }
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int g = i < n ? group_of[i] : -1;
    const bool in = g >= 0 && g < G;
    const int rank = in ? atomicAdd(&cnt[g], 1) : 0;
    __syncthreads();
    if (threadIdx.x < G && cnt[threadIdx.x]) base[threadIdx.x] = start[threadIdx.x] + atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]);
    __syncthreads();
    if (in) order[base[g] + rank] = i;
}

constexpr int kMaxGroups = 64;

// counts[G] | cursor[G] | gtab[2G + 2] | ntab[G + 1] | order[n] | nmap[narrow_grid(G)]
int64_t splp32_group_scratch(int32_t n, int32_t groups) {
    return 4 * ((int64_t)5 * groups + 3 + n + narrow_grid(groups));
}

template <template <bool, bool> class K>
struct ActKernels {  // the four instantiations of one format's kernel template
    static void launch(const uint8_t *W, bool critic, bool sample, dim3 grid, dim3 block, hipStream_t s,
                       const ActArgs &a) {
        if (critic && sample) hipLaunchKernelGGL((K<true, true>::fn), grid, block, 0, s, W, a);
        else if (critic) hipLaunchKernelGGL((K<true, false>::fn), grid, block, 0, s, W, a);  // get_value
        else if (sample) hipLaunchKernelGGL((K<false, true>::fn), grid, block, 0, s, W, a);
        else hipLaunchKernelGGL((K<false, false>::fn), grid, block, 0, s, W, a);
    }
};
template <bool C, bool S>
struct ExactK {
    static constexpr auto fn = k_act32<C, S>;
};
template <bool C, bool S>
struct HalfK {
    static constexpr auto fn = k_act32h<C, S>;
};

// image: a packed fp32 image of format `fmt` (full when has_critic); critic: evaluate the critic
// (SAMPLE with value)
int splp32_act(const uint8_t *img, bool has_critic, bool critic, bool sample, int32_t n, const spl_act_args_t *args,
               void *stream, int fmt, int groups = 0, int64_t image_stride = 0, const int32_t *group_of = nullptr,
               void *scratch = nullptr) {
    const int64_t chunk = fmt ? Geo<FmtF16x2>::kChunk : Geo<FmtBf16x3>::kChunk;
    const float *critic_out = has_critic ? reinterpret_cast<const float *>(img + (size_t)kAllChunks * chunk) : nullptr;
    ActArgs a{args->obs,    args->obs_u8, args->mask,     args->action, args->logprob, args->entropy, args->value,
              args->logits, critic_out,   args->seed,     args->ply,    args->ply_base, args->table0, n,
              nullptr,      nullptr,      0,              0};
    dim3 grid((unsigned)((n + kRowsPerBlock - 1) / kRowsPerBlock)), block(kWaves * 64);
    if (groups > 0) {  // sort the tables by network, then one workgroup per 128 tables of one group
        if (groups > kMaxGroups) return spl_fail(SPL_E_ARG, "at most 64 networks per grouped call");
        if (critic) return spl_fail(SPL_E_ARG, "grouped evaluation serves actor-only images");
        // scratch: counts[G] | cursor[G] | gtab[2G + 2] | ntab[G + 1] | order[n]
        int32_t *counts = static_cast<int32_t *>(scratch), *cursor = counts + groups, *gtab = cursor + groups;
        int32_t *order = gtab + 2 * groups + 2 + groups + 1;
        const hipStream_t s = (hipStream_t)stream;
        const dim3 g256((unsigned)((n + 255) / 256));
        hipLaunchKernelGGL(k_group_count, g256, dim3(256), 0, s, n, groups, group_of, counts);
        hipLaunchKernelGGL(k_group_place, g256, dim3(256), 0, s, n, groups, group_of, counts, cursor, gtab, order);
        a.group_reset = counts;  // counts[G] | cursor[G], zeroed by the k_act32 launch below
        a.order = order;
        a.gtab = gtab;
        a.groups = groups;
        a.image_stride = image_stride;
        // full workgroups only (at most n / 128 of them); the tails go to k_act32_narrow below
    }
    const hipStream_t s = (hipStream_t)stream;
    const uint8_t *W = img;
    if (has_critic && !critic) W += (size_t)kCriticChunks * chunk;  // the actor part of a full image
    if (fmt) ActKernels<HalfK>::launch(W, critic, sample, grid, block, s, a);
    else ActKernels<ExactK>::launch(W, critic, sample, grid, block, s, a);
    if (groups > 0) {  // the groups' tails: at most 8 wave-tiles of 16 tables per group
        const dim3 ngrid((unsigned)narrow_grid(groups)), nblock(kNarrowWaves * 64);
        if (fmt && sample) hipLaunchKernelGGL(k_act32h_narrow<true>, ngrid, nblock, 0, s, W, a);
        else if (fmt) hipLaunchKernelGGL(k_act32h_narrow<false>, ngrid, nblock, 0, s, W, a);
        else if (sample) hipLaunchKernelGGL(k_act32_narrow<true>, ngrid, nblock, 0, s, W, a);
        else hipLaunchKernelGGL(k_act32_narrow<false>, ngrid, nblock, 0, s, W, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return spl_fail(SPL_E_HIP, std::string("k_act32 launch: ") + hipGetErrorString(e));
    return SPL_OK;
}

// spl_engine.hip — MI355X (gfx950) Splendor rollout engine: kernels + C-ABI.
//
// One wavefront lane = one table; a workgroup is ONE wave (64 tables) so small batches still
// spread over all 256 CUs.  State lives in HBM as 32-bit word planes (spl_layout.h) and is
// held in VGPRs for the whole step; branchy rules are predicated per lane (no MFMA: this is
// small-integer work).  Observations are staged in LDS as bytes (every value <= 255 except
// move_count, patched separately) and leave the CU as coalesced 16-byte int32x4 stores; masks
// leave as packed bytes built from per-lane 45-bit words in LDS.
//
// Reference semantics restated here (paths relative to the reference root):
//   engine/rules.py:40-93 legal_moves, :101-122 _pay_for_card, :125-129 _refill_slot,
//   :132-147 _grant_noble_if_applicable, :150-193 auto_return_tokens/_enforce_token_limit,
//   :196-287 apply_action, :290-312 compute_winner/is_terminal; engine/state.py:61-71
//   can_afford, :181-211 initial_state; engine/encode.py:124-187 encode_observation;
//   envs/splendor_env.py:41-115 reset/step/get_final_rewards.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/splendor_amd.h"
#include "spl_layout.h"
#include "spl_rng.h"

namespace spl {

// ------------------------------------------------------------------------------------------
// kernel parameter blocks
// ------------------------------------------------------------------------------------------
struct KArena {
    uint32_t *planes;  // [num_words(P)][n] table state
    uint32_t *pool;    // [PL_COUNT][n] pool deal's board / noble words
    uint8_t *slots;    // [n][2][128] deck records
    uint8_t *pcg;      // [n][64] engine-seed streams
    int n;
    uint8_t *deleg;    // [n/128][kDelegTasks][num_words(P) x 64] u32 staged state words (rollout-store delegation)
    uint32_t *dflags;  // [n/128][kDelegFlagWords] its flags
    uint32_t *legal;   // [2][n] legal-mask cache of the stored state (spl_layout.h)
};

struct KTables {
    const uint4 *cards;   // [90] {1,tier,points,oh_w | oh_b..oh_k | cost w,b,g,r | cost k,colour,0,0}
    const uint2 *nobles;  // [10] {1,req w,b,g | req r,k,points,0}
    const uint4 *lut;     // [kLutEntries] token-return MT outputs (top 3 bits, 10 per word)
    uint32_t mtag;        // this context's legal-mask cache tag (1..65535)
};

struct KStep {
    const int32_t *actions;
    int32_t *obs;
    int8_t *mask;
    float *reward;
    uint8_t *terminated;
    uint8_t *flags;
    int8_t *winner;
    int32_t *final_obs;
    int32_t *next_actions;
    float *ep_return;
    uint32_t *ep_count;
    uint8_t *info;             // nullable: [4][n] info planes + truncated (spl_step)
    uint8_t *obs_u8;           // nullable: [n][300] compact observation instead of obs (k_step_ws)
    const uint8_t *gate_terminated, *gate_flags;  // nullable: the dual step's gate (spl_step_args_t)
    unsigned long long *errors;  // nullable: running count of tables with an error flag (spl_step)
    const uint64_t *ply_base;  // nullable: device counter added to `ply` (graph replays)
    uint64_t *fault;           // nullable: the context's host-mapped fault word (spl_ctx_faults)
    uint64_t fault_tag;        // what a faulting launch writes there (the context's launch serial)
    uint64_t policy_seed;
    uint64_t ply;
    int64_t table0;
    int autoreset;
    int policy;
};

constexpr int kObsDim = 297;
constexpr int kObsU8 = 300;  // compact observation row (spl_step_args_t.obs_u8): 297 bytes + move_count >> 8 + 2 zero

// Ablation switches for profiling builds only (tools/ablate.py); the product build defines none.
#ifndef SPL_ABL
#define SPL_ABL 0
#endif
constexpr int ABL_LEGAL_PRE = 1, ABL_APPLY = 2, ABL_LEGAL_POST = 4, ABL_FINAL = 8, ABL_RESET = 16, ABL_ENCODE = 32,
              ABL_STORE = 64, ABL_MASK_STORE = 128, ABL_SMALL_OUT = 256, ABL_TAB_STORE = 512, ABL_OBS_STORE = 1024,
              ABL_LOAD = 2048, ABL_TOKLIM = 4096, ABL_NOBLE = 8192, ABL_DECK_GATHER = 16384, ABL_LUT_GATHER = 32768;
__device__ __forceinline__ bool abl(int bit) { return (SPL_ABL & bit) != 0; }

// Bounds-check build (-DSPL_BOUNDS_CHECK; libsplendor_amd_checked.so, tests/test_gpu_bounds_check.py):
// index and range invariants are tested at run time and violations recorded as bits of
// g_bounds_flags (an atomic OR: a checked run never faults, it reports).  The product build
// compiles every check out.
#ifdef SPL_BOUNDS_CHECK
__device__ uint32_t g_bounds_flags;
#define SPL_CHECK(cond, bit)                                              \
    do {                                                                  \
        if (!(cond)) atomicOr(&g_bounds_flags, (uint32_t)(bit));          \
    } while (0)
#else
#define SPL_CHECK(cond, bit) \
    do {                     \
    } while (0)
#endif
enum : uint32_t {
    BC_TABLE = 1, BC_SLOT = 2, BC_DECK = 4, BC_LUT = 8, BC_SCRATCH = 16, BC_BYTE = 32, BC_ROWS = 64, BC_CARD = 128,
    BC_SPIN = 256,  // a wave gave up waiting for an LDS hand-off (dealer rollout)
    BC_BARRIER = 512  // a wave of a multi-team workgroup made another number of s_barriers than 1 + K
};

// Phase stamps for the diagnostic build only (-DSPL_STAMPS, tools/stamps.py): lane 0 of every
// wave records s_memrealtime (100 MHz) at phase boundaries of k_step.  Never in the product build.
#ifdef SPL_STAMPS
__device__ uint64_t *g_stamps;
#define STAMP(i)                                                                                 \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        if ((threadIdx.x & 63) == 0 && g_stamps) g_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + (i)] = __builtin_amdgcn_s_memrealtime(); \
        __builtin_amdgcn_sched_barrier(0);                                                       \
    } while (0)
// a value instead of a time in stamp slot i (e.g. a wave's terminal-row count)
#define STAMPV(i, v)                                                                             \
    do {                                                                                         \
        if ((threadIdx.x & 63) == 0 && g_stamps) g_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 16 + (i)] = (uint64_t)(v); \
    } while (0)
// k_rollout keeps its stamps in registers (lane k holds step k's) so that stamping never waits
// on the stores in flight; they are written to g_rstamps[wave][step][kRStamps] at the end.
constexpr int kRStamps = 6;
__device__ uint64_t *g_rstamps;
#define RSTAMP(i, k)                                                                             \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        const uint64_t tt_ = __builtin_amdgcn_s_memrealtime();                                   \
        rst_lo[i] = lane_id() == (k) ? (int)(uint32_t)tt_ : rst_lo[i];                           \
        rst_hi[i] = lane_id() == (k) ? (int)(uint32_t)(tt_ >> 32) : rst_hi[i];                   \
        __builtin_amdgcn_sched_barrier(0);                                                       \
    } while (0)
// rollout_ws (k_rollout_store_*, k_rollout_inplace_*): both waves keep kWsStamps stamps per step in registers (lane k = step k, K <= 64),
// written to g_wsstamps[workgroup][wave][step][kWsStamps] at the end.
constexpr int kWsStamps = 11;  // 0-3 per step; 4-10 sub-phases of the rules wave
__device__ uint64_t *g_wsstamps;
__device__ uint32_t *g_wshwid;  // [workgroup][wave][2]: HW_ID (SIMD, CU, SE) and XCC_ID of each wave
__device__ uint64_t *g_wsclk;   // [workgroup][4]: s_memtime / s_memrealtime at the rules wave's start and end
__device__ uint64_t *g_wsend;   // [workgroup][2]: s_memrealtime at the output wave's last step and at its end
#define WSHWID(sid, wave)                                                                        \
    do {                                                                                         \
        if (g_wshwid && lane_id() == 0) {                                                        \
            g_wshwid[((size_t)(sid) * 2 + (wave)) * 2 + 0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  \
            g_wshwid[((size_t)(sid) * 2 + (wave)) * 2 + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20); \
        }                                                                                        \
    } while (0)
#define WSSTAMP(i, k) RSTAMP(i, k)
#else
#define WSHWID(sid, wave) \
    do {                  \
    } while (0)
#define WSSTAMP(i, k) \
    do {              \
    } while (0)
#define STAMP(i) \
    do {         \
    } while (0)
#define STAMPV(i, v) \
    do {             \
    } while (0)
#define RSTAMP(i, k) \
    do {             \
    } while (0)
#endif
// Outputs a lane takes from the register-only MTStream before a LaneMT continuation takes over
// (MTStream::kMaxOut; lowered only by the test hook spl_debug_set_stream_limit, so the parity tests
// can drive every deal and token return through the continuation path).
__device__ int g_stream_limit = MTStream::kMaxOut;

// Per-lane deal scratch in LDS: an odd number of dwords, so lanes at the same Fisher-Yates
// position (the common case: lanes decrement their index in step) hit 64 different banks.
#ifndef SPL_SCRATCH_STRIDE
#define SPL_SCRATCH_STRIDE 116
#endif
constexpr int kScratchStride = SPL_SCRATCH_STRIDE;
#ifndef SPL_DELEG_EVERY
// rollout-store delegation period (spl_ctx_set_rollout_delegation): off by default.  Alternating
// A/B on one box, 12 launches per arm of 128 steps at 65 536 tables: 1999 +- 25 us off vs
// 1969 +- 34 us every 6th step, a 1.5 % gain (profiles/r03/deleg_ab_r03a.txt) -- under the 2 %
// that would pay for a cross-XCC hand-off in the headline kernel
#define SPL_DELEG_EVERY 0
#endif
#ifndef SPL_PARTNER_LEAD
// partner hand-off of the one-workgroup-per-CU rollout stores (six-wave dealer, quad; spl_ctx_set_partner_lead):
// a team hands a step's rows to its neighbouring-XCC partner when that one is this many steps ahead.
// Default 0 (off) since round 6's sc0 nt sc1 row stores (SPL_ROLL_CPOL): the teams then lag far less and
// the polls cost more than the hand-off recovers — quad lead 0 / 4 / 8: 1 873-1 898 / 1 909-1 925 /
// 1 912-1 913 us per launch (another box: lead 0 / 4 1 863-1 873 / 1 892-1 900,
// profiles/r06/quad_lead_ab_r06ad.txt); six-wave dealer (C4) 1 075-1 078 / 1 081-1 100 / 1 083-1 102
// (profiles/r06/c4_lead_ab_r06ag.txt).  With nt-only stores lead 4 had paid 2.4 % (headline,
// profiles/r06/headab_r06d.txt) and ~2 % (C4, profiles/r04/partner_ab_r04u.txt).
#define SPL_PARTNER_LEAD 0
#endif
#ifndef SPL_XCD_MAP
#define SPL_XCD_MAP 1
#endif
// Workgroup -> 64-table block, XCD-contiguous.  The dispatcher hands workgroup b to XCD b % 8, so
// with the identity map every XCD writes every eighth 76 KB chunk of a step's rollout-store block;
// mapped, XCD x's workgroups own tables [x n/8, (x+1) n/8) and each XCD streams one contiguous eighth
// of the block (store-only pattern: 880 -> 844-862 us per 64 steps on one box,
// tools/microbench_hbm_store.hip rows_x).  Only which workgroup steps which tables changes: every
// table's chain is its own, so results are identical (A/B build switch SPL_XCD_MAP=0).
__device__ __forceinline__ int wg_block_of(uint32_t b) {
    const uint32_t nb = gridDim.x;
    if (!SPL_XCD_MAP || (nb & 7u)) return (int)b;
    return (int)((b & 7u) * (nb >> 3) + (b >> 3));
}
__device__ __forceinline__ int wg_block() { return wg_block_of(blockIdx.x); }
#ifndef SPL_STEP_OBS_NT
#define SPL_STEP_OBS_NT false  // k_step_ws observation stores non-temporal (A/B switch)
#endif
// k_step_wst (at most three workgroups per CU) stores its int32 rows through the NT output stream
// (SPL_ROLL_CPOL's sc0 nt sc1): per step 17.1 -> 16.0 us at 32 768 tables, 14.8 -> 12.8 at 16 384,
// 12.7 -> 12.2 at 4 096 (profiles/r06/step_tail_store_ab_r06y.txt), where at 65 536 tables (k_step_ws)
// non-temporal rows cost 22.4 -> 23.8 us (profiles/r06/step_store_policy_ab_r06x.txt)
#ifndef SPL_STEP_TAIL_NT
#define SPL_STEP_TAIL_NT true
#endif
// k_step_ws (four workgroups per CU) stores its int32 rows as `sc1` buffer stores (system scope, temporal;
// -2 = plain): 22.35 -> 20.5 us per step at 65 536 tables; `sc0 sc1` the same, `sc0` alone as plain
// (profiles/r06/step_ws_temporal_policy_r06an.txt); non-temporal rows were slower there (23.8 us)
// the three-wave step's row policy (-3: SPL_STEP_TAIL_NT's stream): `sc1` (16), per step 15.98 -> 15.07 us at
// 32 768 tables, 20.0 -> 18.2 at 49 152, 12.85 -> 12.82 at 16 384 against sc0 nt sc1
// (profiles/r06/step_tail_sc1_ab_r06ap.txt)
#ifndef SPL_STEP_TAIL_CPOL
#define SPL_STEP_TAIL_CPOL 16
#endif
// A/B switch: spl_step's mask block store policy (-2 plain)
#ifndef SPL_STEP_MASK_CPOL
#define SPL_STEP_MASK_CPOL -2
#endif
#ifndef SPL_STEP_WS_CPOL
#define SPL_STEP_WS_CPOL 16
#endif
// A/B switch: k_step_ws stores the first (1) or second (2) half of its row block through the NT output
// stream and the other half plain (0: all plain)
#ifndef SPL_STEP_WS_SPLIT
#define SPL_STEP_WS_SPLIT 0
#endif
#ifndef SPL_STEP_BOTH_NT
#define SPL_STEP_BOTH_NT 0
#endif
struct NoOp {
    __device__ __forceinline__ void operator()() const {}
};
#ifndef SPL_WS_PRIO
#define SPL_WS_PRIO 1
#endif
// per-step rollout-store rows and masks non-temporal (1, round 2's choice) or plain (0): A/B switch
#ifndef SPL_ROLL_NT
#define SPL_ROLL_NT 1
#endif
constexpr bool kRollNT = SPL_ROLL_NT != 0;

constexpr int kMaskStreamWords = 64 * 45 / 32;  // 90

// constant tables staged per workgroup: 16-B obs-ready card records and 8-B noble records
struct __align__(16) Consts {
    uint4 cards[90];
    uint2 nobles[10];
};

// one wave's output staging
struct __align__(16) WaveBuf {
    uint64_t mask[64];
    uint32_t mbits[96];  // the wave's 64 x 45 mask bits as one stream (store_mask_block)
    uint8_t rows[64 * kObsDim];   // observation staging; also the deal scratch (64 x 112 B)
    uint8_t frows[64 * kObsDim];  // terminal observations (k_step): stored with everything else at the end
};
struct __align__(16) BlockLDS : Consts, WaveBuf {};
// k_step with W waves (64 tables each) per workgroup: one copy of the constant tables
template <int W>
struct __align__(16) StepLDS : Consts {
    WaveBuf w[W];
};

// ------------------------------------------------------------------------------------------
// small helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bget(uint32_t w, int k) { return (w >> (8 * k)) & 0xFFu; }
__device__ __forceinline__ uint32_t bset(uint32_t w, int k, uint32_t v) {
    return (w & ~(0xFFu << (8 * k))) | ((v & 0xFFu) << (8 * k));
}
__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63u); }

// Cross-lane LDS hand-off inside ONE wave (every workgroup here is a single wave).
// __syncthreads() would also emit s_waitcnt vmcnt(0): the wave would stall until its pending
// global stores drain behind every other wave's observation traffic.  LDS executes one wave's
// operations in order, so ordering the compiler (wavefront fence) and the LDS counter suffices.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
    __builtin_amdgcn_wave_barrier();
}

// Launder a value through an empty asm so that a select chain over struct members stays a
// select of VALUES: otherwise LLVM folds "c ? s.a : s.b" into a load at a selected offset,
// which pins the whole struct in scratch memory.
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    asm("" : "+v"(x));
    return x;
}
__device__ __forceinline__ int opaque(int x) {
    asm("" : "+v"(x));
    return x;
}

template <int P>
struct Tab {
    uint32_t sw[SW_COUNT];
    uint32_t pw[P][4];
};

struct Pl {
    int tok[6], bon[5], pres, nres, rev, res[3];
};

__device__ __forceinline__ Pl unpack_pl(const uint32_t w[4]) {
    Pl p;
#pragma unroll
    for (int c = 0; c < 4; ++c) p.tok[c] = (int)bget(w[0], c);
    p.tok[4] = (int)bget(w[1], 0);
    p.tok[5] = (int)bget(w[1], 1);
    p.bon[0] = (int)bget(w[1], 2);
    p.bon[1] = (int)bget(w[1], 3);
    p.bon[2] = (int)bget(w[2], 0);
    p.bon[3] = (int)bget(w[2], 1);
    p.bon[4] = (int)bget(w[2], 2);
    p.pres = (int)bget(w[2], 3);
    p.nres = (int)(w[3] & 3u);
    p.rev = (int)((w[3] >> 2) & 7u);
#pragma unroll
    for (int i = 0; i < 3; ++i) p.res[i] = (int)bget(w[3], i + 1);
    return p;
}

__device__ __forceinline__ void pack_pl(const Pl &p, uint32_t w[4]) {
#ifdef SPL_BOUNDS_CHECK
    for (int c = 0; c < 6; ++c) SPL_CHECK(p.tok[c] >= 0 && p.tok[c] <= 255, BC_BYTE);
    for (int c = 0; c < 5; ++c) SPL_CHECK(p.bon[c] >= 0 && p.bon[c] <= 255, BC_BYTE);
    SPL_CHECK(p.pres >= 0 && p.pres <= 255 && p.nres >= 0 && p.nres <= 3, BC_BYTE);
#endif
    w[0] = (uint32_t)p.tok[0] | ((uint32_t)p.tok[1] << 8) | ((uint32_t)p.tok[2] << 16) | ((uint32_t)p.tok[3] << 24);
    w[1] = (uint32_t)p.tok[4] | ((uint32_t)p.tok[5] << 8) | ((uint32_t)p.bon[0] << 16) | ((uint32_t)p.bon[1] << 24);
    w[2] = (uint32_t)p.bon[2] | ((uint32_t)p.bon[3] << 8) | ((uint32_t)p.bon[4] << 16) | ((uint32_t)p.pres << 24);
    w[3] = ((uint32_t)p.nres & 3u) | (((uint32_t)p.rev & 7u) << 2) | (((uint32_t)p.res[0] & 0xFFu) << 8) |
           (((uint32_t)p.res[1] & 0xFFu) << 16) | (((uint32_t)p.res[2] & 0xFFu) << 24);
}

template <int P>
__device__ __forceinline__ void get_player(const Tab<P> &T, int p, uint32_t w[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // launder every player's word first: an asm inside the select would be executed
        // conditionally, i.e. compiled into one branch per word
        uint32_t o[P];
#pragma unroll
        for (int q = 0; q < P; ++q) o[q] = opaque(T.pw[q][k]);
        uint32_t v = o[0];
#pragma unroll
        for (int q = 1; q < P; ++q) v = (p == q) ? o[q] : v;
        w[k] = v;
    }
}

template <int P>
__device__ __forceinline__ void put_player(Tab<P> &T, int p, const uint32_t w[4]) {
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) T.pw[q][k] = (p == q) ? w[k] : T.pw[q][k];
}

__device__ __forceinline__ void get_bank(const uint32_t *sw, int bank[6]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) bank[c] = (int)bget(sw[SW_BANK0], c);
    bank[4] = (int)bget(sw[SW_BANK1], 0);
    bank[5] = (int)bget(sw[SW_BANK1], 1);
}

__device__ __forceinline__ void put_bank(uint32_t *sw, const int bank[6]) {
#ifdef SPL_BOUNDS_CHECK
    for (int c = 0; c < 6; ++c) SPL_CHECK(bank[c] >= 0 && bank[c] <= 255, BC_BYTE);
#endif
    sw[SW_BANK0] = (uint32_t)bank[0] | ((uint32_t)bank[1] << 8) | ((uint32_t)bank[2] << 16) | ((uint32_t)bank[3] << 24);
    sw[SW_BANK1] = (sw[SW_BANK1] & 0xFFFF0000u) | (uint32_t)bank[4] | ((uint32_t)bank[5] << 8);
}

__device__ __forceinline__ int board_get(const uint32_t *sw, int k) {  // runtime k
    const uint32_t b0 = opaque(sw[SW_BOARD]), b1 = opaque(sw[SW_BOARD + 1]), b2 = opaque(sw[SW_BOARD + 2]);
    const uint32_t w = k < 4 ? b0 : (k < 8 ? b1 : b2);
    return (int)bget(w, k & 3);
}
__device__ __forceinline__ void board_set(uint32_t *sw, int k, uint32_t v) {  // runtime k
#pragma unroll
    for (int t = 0; t < 3; ++t) sw[SW_BOARD + t] = (k >> 2) == t ? bset(sw[SW_BOARD + t], k & 3, v) : sw[SW_BOARD + t];
}

__device__ __forceinline__ uint4 card_rec(const Consts &L, int id) { return L.cards[id < 90 ? id : 0]; }

__device__ __forceinline__ int card_cost(uint4 rec, int c) { return c < 4 ? (int)bget(rec.z, c) : (int)bget(rec.w, 0); }

// Packed 16-bit arithmetic for per-colour comparisons: two colours per dword, saturating
// subtraction in one v_pk_sub_u16 (clamp).  Byte fields are widened with one v_perm_b32.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t sat_sub16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, a),
                                                                      __builtin_bit_cast(u16x2, b)));
}
// bytes i and j of w as the low and high 16-bit halves
__device__ __forceinline__ uint32_t widen2(uint32_t w, int i, int j) {
    return __builtin_amdgcn_perm(0u, w, 0x0C000C00u | ((uint32_t)j << 16) | (uint32_t)i);
}

// what the player can put toward each colour: tokens + bonuses, packed (w|b, g|r, k) + gold
struct Have {
    uint32_t wb, gr, k;
    int gold;
};
__device__ __forceinline__ Have have_of(const Pl &p) {
    Have h;
    h.wb = (uint32_t)(p.tok[0] + p.bon[0]) | ((uint32_t)(p.tok[1] + p.bon[1]) << 16);
    h.gr = (uint32_t)(p.tok[2] + p.bon[2]) | ((uint32_t)(p.tok[3] + p.bon[3]) << 16);
    h.k = (uint32_t)(p.tok[4] + p.bon[4]);
    h.gold = p.tok[5];
    return h;
}

// engine/state.py:61-71 can_afford: sum over colours of max(cost - bonus - tokens, 0) <= gold
// (max(max(cost - bonus, 0) - tokens, 0) == max(cost - bonus - tokens, 0) for tokens >= 0)
__device__ __forceinline__ bool afford(const Have &h, uint4 rec) {
    const uint32_t s = sat_sub16(widen2(rec.z, 0, 1), h.wb) + sat_sub16(widen2(rec.z, 2, 3), h.gr);
    const int need = (int)(s & 0xFFFFu) + (int)(s >> 16) + max((int)bget(rec.w, 0) - (int)h.k, 0);
    return h.gold >= need;
}

// take-3 colour sets in itertools.combinations(range(5), 3) order (engine/encode.py:35)
constexpr uint64_t kTake3Masks = (0x07ull) | (0x0Bull << 5) | (0x13ull << 10) | (0x0Dull << 15) |
                                 (0x15ull << 20) | (0x19ull << 25) | (0x0Eull << 30) | (0x16ull << 35) |
                                 (0x1Aull << 40) | (0x1Cull << 45);
__device__ __forceinline__ uint32_t take3_mask(int i) { return (uint32_t)(kTake3Masks >> (5 * i)) & 31u; }

// engine/rules.py:40-93 legal_moves -> 45-bit mask
__device__ __forceinline__ uint64_t legal_mask(const uint32_t *sw, const Pl &p, const int bank[6], const Consts &L) {
    uint32_t avail = 0;
#pragma unroll
    for (int c = 0; c < 5; ++c) avail |= (bank[c] >= 1 ? 1u : 0u) << c;
    const int nav = __popc(avail);
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < 10; ++i) {  // :45-58 reduced take-3 rule
        const uint32_t cm = take3_mask(i);
        const bool ok = nav >= 3 ? ((cm & avail) == cm) : (nav >= 1 && (avail & cm) == avail);
        m |= (uint64_t)ok << i;
    }
#pragma unroll
    for (int c = 0; c < 5; ++c) m |= (uint64_t)(bank[c] >= 4) << (10 + c);  // :61-63
    const bool can_res = p.nres < 3;
    const Have h = have_of(p);
    // every card record is read unconditionally (missing cards read record 0) and combined with
    // bitwise ops: `present && afford(card_rec(...))` compiled into 15 branches, each an LDS read
    // followed by its own lgkmcnt(0) wait — 15 serial LDS round trips per legal mask
    uint4 rec[15];
#pragma unroll
    for (int k = 0; k < 12; ++k) rec[k] = card_rec(L, (int)bget(sw[SW_BOARD + k / 4], k % 4));
#pragma unroll
    for (int i = 0; i < 3; ++i) rec[12 + i] = card_rec(L, p.res[i]);
#pragma unroll
    for (int k = 0; k < 12; ++k) {  // :66-80
        const uint32_t present = bget(sw[SW_BOARD + k / 4], k % 4) != 0xFFu ? 1u : 0u;
        const uint32_t aff = afford(h, rec[k]) ? 1u : 0u;
        m |= (uint64_t)(present & aff) << (15 + k);
        m |= (uint64_t)(present & (can_res ? 1u : 0u)) << (27 + k);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) m |= (uint64_t)(can_res && bget(sw[SW_DECK], t) > 0) << (39 + t);  // :83-86
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // :89-91
        const uint32_t held = i < p.nres ? 1u : 0u;
        const uint32_t aff = afford(h, rec[12 + i]) ? 1u : 0u;
        m |= (uint64_t)(held & aff) << (42 + i);
    }
    return m;
}

// engine/rules.py:40-93 restricted to one action (the env only needs mask[a]) ...
__device__ __forceinline__ bool action_legal(const uint32_t *sw, const Pl &p, const int bank[6], int a,
                                             const Consts &L) {
    if (a < 10) {
        uint32_t avail = 0;
#pragma unroll
        for (int c = 0; c < 5; ++c) avail |= (bank[c] >= 1 ? 1u : 0u) << c;
        const int nav = __popc(avail);
        const uint32_t cm = take3_mask(a);
        return nav >= 3 ? ((cm & avail) == cm) : (nav >= 1 && (avail & cm) == avail);
    }
    if (a < 15) {
        const int c = a - 10;
        const int b = c == 0 ? bank[0] : (c == 1 ? bank[1] : (c == 2 ? bank[2] : (c == 3 ? bank[3] : bank[4])));
        return b >= 4;
    }
    if (a < 27) {
        const int id = board_get(sw, a - 15);
        return id != 0xFF && afford(have_of(p), card_rec(L, id));
    }
    if (a < 39) return p.nres < 3 && board_get(sw, a - 27) != 0xFF;
    if (a < 42) return p.nres < 3 && bget(sw[SW_DECK], a - 39) > 0;
    const int i = a - 42;
    const int r0 = opaque(p.res[0]), r1 = opaque(p.res[1]), r2 = opaque(p.res[2]);
    return i < p.nres && afford(have_of(p), card_rec(L, i == 0 ? r0 : (i == 1 ? r1 : r2)));
}

// ... and whether ANY move is legal: with a non-gold colour in the bank some take-3 always is
// (rules.py:45-58), otherwise fall back to the full mask (rare).
__device__ __forceinline__ bool any_legal(const uint32_t *sw, const Pl &p, const int bank[6], const Consts &L) {
    const bool some_colour = bank[0] > 0 || bank[1] > 0 || bank[2] > 0 || bank[3] > 0 || bank[4] > 0;
    return some_colour || legal_mask(sw, p, bank, L) != 0ull;
}

// engine/rules.py:101-122 _pay_for_card
__device__ __forceinline__ void pay_for_card(Pl &p, int bank[6], uint4 rec) {
    const int gold_avail = p.tok[5];
    int gold_spent = 0;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        const int disc = max(card_cost(rec, c) - p.bon[c], 0);
        const int spend = min(p.tok[c], disc);
        p.tok[c] -= spend;
        bank[c] += spend;
        const int rem = disc - spend;
        gold_spent += rem > 0 ? min(rem, gold_avail - gold_spent) : 0;
    }
    p.tok[5] -= gold_spent;
    bank[5] += gold_spent;
    const int colour = (int)bget(rec.w, 1);
#pragma unroll
    for (int c = 0; c < 5; ++c) p.bon[c] += colour == c ? 1 : 0;
    p.pres += (int)bget(rec.x, 2);
}

__device__ __forceinline__ uint8_t *slot_rec(const KArena &A, int t, int slot) {
    SPL_CHECK(t >= 0 && t < A.n, BC_TABLE);
    SPL_CHECK(slot >= 0 && slot < kSlotRecords, BC_SLOT);
    return A.slots + ((size_t)t * kSlotRecords + slot) * kSlotBytes;
}
// slot-record ring status (spl_layout.h)
__device__ __forceinline__ int active_of(uint32_t misc) { return (int)((misc >> ST_ACTIVE_SHIFT) & 3u); }
__device__ __forceinline__ int pend_of(uint32_t misc) { return (int)((misc >> ST_PEND_SHIFT) & 3u); }
__device__ __forceinline__ uint32_t ring_bits(int active, int pend) {
    return ((uint32_t)active << ST_ACTIVE_SHIFT) | ((uint32_t)pend << ST_PEND_SHIFT);
}
__device__ __forceinline__ const uint8_t *live_rec(const KArena &A, int t, uint32_t misc) {
    return slot_rec(A, t, active_of(misc));
}

// engine/rules.py:125-129 _refill_slot / deck.pop() of tier t.  `top` is the card at
// deck_len-1 of that tier, gathered from the live record at the top of the step (one action
// pops at most one card, from the tier the action names: pop_tier()).
__device__ __forceinline__ uint32_t deck_pop(uint32_t *sw, uint32_t top, int t) {
    const int len = (int)bget(sw[SW_DECK], t);
    if (len <= 0) return 0xFFu;
    sw[SW_DECK] = bset(sw[SW_DECK], t, (uint32_t)(len - 1));
    return top;
}

// legal_moves of every fresh deal (engine/rules.py:40-93 on state.py:181-211's table): every
// take-3 and take-2 (bank 4 of each colour), every visible and blind reserve, no purchase
constexpr uint64_t kFreshDealMask = ((1ull << 15) - 1ull) | (((1ull << 15) - 1ull) << 27);

// tier an action pops from: buy visible (:216-225) and reserve visible (:226-240) refill the
// slot's tier, reserve blind (:241-249) draws from its tier; -1 for every other action
__device__ __forceinline__ int pop_tier(int a) {
    return (a >= 15 && a < 27) ? (a - 15) >> 2 : ((a >= 27 && a < 39) ? (a - 27) >> 2 : ((a >= 39 && a < 42) ? a - 39 : -1));
}

// pick the r-th colour (ascending) among non-gold colours the player holds
__device__ __forceinline__ void return_one(Pl &p, int bank[6], int r) {
    int seen = 0;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        const bool has = p.tok[c] > 0;
        const bool hit = has && seen == r;
        p.tok[c] -= hit ? 1 : 0;
        bank[c] += hit ? 1 : 0;
        seen += has ? 1 : 0;
    }
}

__device__ __forceinline__ int non_gold_kinds(const Pl &p) {
    int n = 0;
#pragma unroll
    for (int c = 0; c < 5; ++c) n += p.tok[c] > 0 ? 1 : 0;
    return n;
}

// engine/rules.py:150-185 auto_return_tokens on the full CPython MT stream (rare: seeds
// outside the precomputed table, or a table entry that ran out of draws).
__device__ __forceinline__ void token_return_mt(Pl &p, int bank[6], int remaining, uint64_t seed, uint32_t *mtx) {
    MTStream ms;
    ms.init(seed);
    bool done = false;
    auto draw = [&](uint32_t y) {  // rng.choice(choices) on output y
        const int nch = non_gold_kinds(p);
        const int kb = bit_length((uint32_t)nch);
        const int r = (int)(y >> (32 - kb));
        if (r < nch) {  // accepted
            return_one(p, bank, r);
            remaining -= 1;
        }
    };
    const int limit = min(g_stream_limit, MTStream::kMaxOut);
    for (int j = 0;; ++j) {
        done = done || remaining <= 0 || non_gold_kinds(p) == 0;
        if (!__any(!done)) break;
        if (j >= limit) break;  // lanes still returning continue below
        const uint32_t y = ms.next(j);
        if (!done) draw(y);
    }
    // Continuation past the streamed outputs (crafted states with hundreds of tokens to return):
    // one lane at a time, its full MT19937 state in the LDS region mtx, from output kMaxOut on.
    for (uint64_t slow = __ballot(!done); slow; slow &= slow - 1) {
        if (lane_id() == __ffsll((unsigned long long)slow) - 1) {
            LaneMT mt{mtx, 0};
            mt.init(seed);
            mt.start_at(limit);
            while (remaining > 0 && non_gold_kinds(p) > 0) draw(mt.next());
        }
    }
    if (remaining > 0 && p.tok[5] > 0) {
        const int give = min(remaining, p.tok[5]);
        p.tok[5] -= give;
        bank[5] += give;
    }
}

// token-return table index of (turn_count, to_play, sum(tokens), sum(bank)), -1 outside it
__device__ __forceinline__ int lut_key(int turn_count, int to_play, int total, int bank_total) {
    const bool in_lut = turn_count < kLutTc && to_play < kLutTp && total >= 11 && total <= 13 && bank_total < kLutSb;
    return in_lut ? ((turn_count * kLutTp + to_play) * kLutSt + (total - 11)) * kLutSb + bank_total : -1;
}

// The table entry action `a` will consult, predicted from the pre-action state so its load
// can start with the state loads: takes and reserves move tokens bank -> player exactly as
// apply_action does; buys only lower the mover's total (-1: no prediction).
__device__ __forceinline__ int predict_lut_key(const Pl &p, const int bank[6], int a, int turn_count, int to_play) {
    int total = 0, bank_total = 0, delta = 0;
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        total += p.tok[c];
        bank_total += bank[c];
    }
    if (a < 10) {
        const uint32_t cm = take3_mask(a);
#pragma unroll
        for (int c = 0; c < 5; ++c) delta += (((cm >> c) & 1u) && bank[c] >= 1) ? 1 : 0;
    } else if (a < 15) {
        delta = 2;
    } else if (a >= 27 && a < 42) {
        delta = bank[5] > 0 ? 1 : 0;
    } else {
        return -1;
    }
    return total + delta > 10 ? lut_key(turn_count, to_play, total + delta, bank_total - delta) : -1;
}

// engine/rules.py:150-185 auto_return_tokens on the table entry `e` (top 3 bits of the first
// 40 outputs of the seeded stream, 10 per word).  One draw per iteration for every lane still
// returning: rng.choice -> _randbelow(n) takes the top bit_length(n) bits of one output and
// rejects r >= n; an accepted r returns one token of the r-th held non-gold colour.  The loop
// exit is wave-uniform and the body predicated, so divergent rejection counts cost no nested
// control flow.  Returns false if the lane needs more than the table's 40 outputs.
__device__ __forceinline__ bool token_return_lut(Pl &p, int bank[6], int remaining, uint4 e) {
    // On this path the mover holds 11..13 tokens, so every count fits a nibble: `tk` holds the
    // five non-gold counts, `list` the held colours in ascending order (CPython's `choices`
    // list, rebuilt after every draw in the reference) and `n` its length.  A draw reads the
    // r-th entry of the list; a colour that runs out is cut out of it.  All 32-bit ops.
    uint32_t tk = 0, list = 0;
    int n = 0;
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        tk |= (uint32_t)p.tok[c] << (4 * c);
        const bool has = p.tok[c] > 0;
        list |= has ? (uint32_t)c << (4 * n) : 0u;
        n += has ? 1 : 0;
    }
    bool active = remaining > 0 && n > 0;
    // every lane draws at the same position, so the output word and bit offset are uniform
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t w = q == 0 ? e.x : (q == 1 ? e.y : (q == 2 ? e.z : e.w));
#pragma unroll 1
        for (int j = 0; j < 10; ++j) {
            if (!__any(active)) goto drawn;
            // _randbelow(n): top bit_length(n) of the 3 stored bits; shift 3 - bit_length(n)
            // for n = 1..5 is 2, 1, 1, 0, 0 (nibbles of 0x1120)
            const uint32_t r = __builtin_amdgcn_ubfe(w, 3u * (uint32_t)j, 3u) >> ((0x1120u >> (4 * n)) & 15u);
            const bool acc = active && (int)r < n;
            const uint32_t c4 = 4u * __builtin_amdgcn_ubfe(list, 4u * r, 4u);  // nibble of the colour in tk
            tk -= acc ? (1u << c4) : 0u;
            const bool out = acc && ((tk >> c4) & 15u) == 0u;
            const uint32_t low = (1u << (4u * r)) - 1u;  // cut entry r out of the list
            list = out ? ((list & low) | ((list >> ((4u * r + 4u) & 31u)) << (4u * r))) : list;
            n -= out ? 1 : 0;
            remaining -= acc ? 1 : 0;
            active = active && remaining > 0 && n > 0;
        }
    }
drawn:
    if (remaining > 0 && n > 0) return false;  // table outputs exhausted
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        const int now = (int)((tk >> (4 * c)) & 15u);
        bank[c] += p.tok[c] - now;
        p.tok[c] = now;
    }
    if (remaining > 0 && p.tok[5] > 0) {              // :179-184 then gold
        const int give = min(remaining, p.tok[5]);
        p.tok[5] -= give;
        bank[5] += give;
    }
    return true;
}

// engine/rules.py:188-193 _enforce_token_limit -> :150-185 auto_return_tokens.  `pre_key` /
// `pre_e` are the prefetched table entry (predict_lut_key); any other key is loaded here.
__device__ __forceinline__ void enforce_token_limit(Pl &p, int bank[6], int turn_count, int to_play,
                                                    const uint4 *lut, int pre_key, uint4 pre_e, uint32_t *mtx) {
    int total = 0, bank_total = 0;
#pragma unroll
    for (int c = 0; c < 6; ++c) total += p.tok[c];
    if (total <= 10) return;
#pragma unroll
    for (int c = 0; c < 6; ++c) bank_total += bank[c];
    const int key = lut_key(turn_count, to_play, total, bank_total);
    const bool in_lut = key >= 0;
    bool need_mt = !in_lut;
    if (in_lut) {
        SPL_CHECK(key < kLutEntries, BC_LUT);
        const uint4 e = key == pre_key ? pre_e : lut[key];
        Pl p2 = p;
        int bank2[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) bank2[c] = bank[c];
        if (token_return_lut(p2, bank2, total - 10, e)) {
            p = p2;
#pragma unroll
            for (int c = 0; c < 6; ++c) bank[c] = bank2[c];
        } else {
            need_mt = true;
        }
    }
    if (need_mt) {
        const uint64_t seed = ((uint64_t)turn_count * 1315423911ull) ^ ((uint64_t)to_play * 2654435761ull) ^
                              ((uint64_t)total * 97531ull) ^ ((uint64_t)bank_total * 31337ull);
        token_return_mt(p, bank, total - 10, seed, mtx);
    }
}

// engine/rules.py:132-147 _grant_noble_if_applicable (first visible noble in slot order)
__device__ __forceinline__ void grant_noble(uint32_t *sw, Pl &p, int to_play, const Consts &L) {
    const int nn = (int)bget(sw[SW_DECK], 3);
    uint32_t owners = (sw[SW_NOB1] >> 8) & 0x7FFFu;
    bool granted = false;
    const uint32_t bon_wb = (uint32_t)p.bon[0] | ((uint32_t)p.bon[1] << 16);
    const uint32_t bon_gr = (uint32_t)p.bon[2] | ((uint32_t)p.bon[3] << 16);
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int idx = s < 4 ? (int)bget(sw[SW_NOB0], s) : (int)bget(sw[SW_NOB1], 0);
        const bool visible = s < nn && ((owners >> (3 * s)) & 7u) == 0 && idx < 10;
        const uint2 rec = L.nobles[idx < 10 ? idx : 0];
        // requirement minus bonus, saturated, is zero in every colour
        const uint32_t req_wb = widen2(rec.x, 1, 2);
        const uint32_t req_gr = __builtin_amdgcn_perm(rec.y, rec.x, 0x0C040C03u);  // x.byte3 | y.byte0
        const bool meets = (sat_sub16(req_wb, bon_wb) | sat_sub16(req_gr, bon_gr)) == 0u &&
                           (int)bget(rec.y, 1) <= p.bon[4];
        const bool take = !granted && visible && meets;
        owners |= take ? ((uint32_t)(to_play + 1) << (3 * s)) : 0u;
        p.pres += take ? (int)bget(rec.y, 2) : 0;
        granted = granted || take;
    }
    sw[SW_NOB1] = (sw[SW_NOB1] & 0xFFu) | (owners << 8);
}

// engine/rules.py:290-303 compute_winner: key (prestige, -cards, -reserved); tie of the top
// two keys -> None
template <int P>
__device__ __forceinline__ int compute_winner(const Tab<P> &T) {
    // track the top two keys as values (a runtime-indexed key[] array would go to scratch)
    int best = -1;
    uint32_t kbest = 0, ksecond = 0;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        const Pl p = unpack_pl(T.pw[q]);
        const int nb = p.bon[0] + p.bon[1] + p.bon[2] + p.bon[3] + p.bon[4];
        const uint32_t key = ((uint32_t)p.pres << 16) | ((uint32_t)(1023 - nb) << 4) | (uint32_t)(15 - p.nres);
        if (q == 0) {
            best = 0;
            kbest = key;
        } else if (key >= kbest) {
            ksecond = kbest;
            kbest = key;
            best = q;
        } else if (q == 1 || key >= ksecond) {
            ksecond = key;
        }
    }
    return kbest == ksecond ? -1 : best;
}

__device__ __forceinline__ int get_to_play(const uint32_t *sw) { return (int)bget(sw[SW_BANK1], 2); }
__device__ __forceinline__ int get_turn(const uint32_t *sw) { return (int)bget(sw[SW_BANK1], 3); }
__device__ __forceinline__ int get_moves(const uint32_t *sw) { return (int)(sw[SW_MISC] & 0xFFFFu); }
__device__ __forceinline__ int get_winner(const uint32_t *sw) { return (int)(sw[SW_MISC] >> 24) - 1; }
__device__ __forceinline__ bool is_terminal(const uint32_t *sw) {
    return (sw[SW_MISC] & ST_GAME_OVER) && get_to_play(sw) == 0;
}

// sub-phase stamp hook of step_rules (diagnostic builds pass a stamping lambda)
struct NoStamp {
    __device__ __forceinline__ void operator()(int) const {}
};

// engine/rules.py:196-287 apply_action on the current player (action known legal)
template <int P, class Stamp>
__device__ __forceinline__ void apply_action(Tab<P> &T, int a, uint32_t top, const Consts &L, const uint4 *lut,
                                             int pre_key, uint4 pre_e, uint32_t *mtx, Stamp stamp) {
    uint32_t *sw = T.sw;
    const int tp = get_to_play(sw);
    uint32_t w[4];
    get_player(T, tp, w);
    Pl p = unpack_pl(w);
    int bank[6];
    get_bank(sw, bank);
    if (a < 10) {  // :201-210 take-3 (only colours still in the bank)
        const uint32_t cm = take3_mask(a);
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            const bool take = ((cm >> c) & 1u) && bank[c] >= 1;
            bank[c] -= take ? 1 : 0;
            p.tok[c] += take ? 1 : 0;
        }
    } else if (a < 15) {  // :211-215 take-2
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            bank[c] -= (a - 10) == c ? 2 : 0;
            p.tok[c] += (a - 10) == c ? 2 : 0;
        }
    } else if (a < 27) {  // :216-225 buy visible, refill
        const int k = a - 15;
        pay_for_card(p, bank, card_rec(L, board_get(sw, k)));
        board_set(sw, k, deck_pop(sw, top, k >> 2));
    } else if (a < 39) {  // :226-240 reserve visible, gold if any, refill
        const int k = a - 27;
        const int card = board_get(sw, k);
#pragma unroll
        for (int i = 0; i < 3; ++i) p.res[i] = p.nres == i ? card : p.res[i];
        p.rev |= 1 << p.nres;
        p.nres += 1;
        const bool gold = bank[5] > 0;
        bank[5] -= gold ? 1 : 0;
        p.tok[5] += gold ? 1 : 0;
        board_set(sw, k, deck_pop(sw, top, k >> 2));
    } else if (a < 42) {  // :241-249 reserve blind (hidden), gold if any
        const int card = (int)deck_pop(sw, top, a - 39);
#pragma unroll
        for (int i = 0; i < 3; ++i) p.res[i] = p.nres == i ? card : p.res[i];
        p.rev &= ~(1 << p.nres);
        p.nres += 1;
        const bool gold = bank[5] > 0;
        bank[5] -= gold ? 1 : 0;
        p.tok[5] += gold ? 1 : 0;
    } else {  // :250-255 buy reserved: list.pop(i) shifts later slots
        const int i = a - 42;
        const int r0 = opaque(p.res[0]), r1 = opaque(p.res[1]), r2 = opaque(p.res[2]);
        const int card = i == 0 ? r0 : (i == 1 ? r1 : r2);
        p.res[0] = i == 0 ? r1 : r0;
        p.res[1] = i <= 1 ? r2 : r1;
        p.res[2] = 0xFF;
        p.rev = (p.rev & ((1 << i) - 1)) | ((p.rev >> (i + 1)) << i);
        p.nres -= 1;
        pay_for_card(p, bank, card_rec(L, card));
    }
    stamp(8);
    if (!abl(ABL_NOBLE)) grant_noble(sw, p, tp, L);                         // :260
    stamp(9);
    if (!abl(ABL_TOKLIM)) enforce_token_limit(p, bank, get_turn(sw), tp, lut, pre_key, pre_e, mtx);  // :261
    stamp(10);
    uint32_t misc = sw[SW_MISC];
    if (p.pres >= 15) misc |= ST_GAME_OVER;                                 // :264-265
    pack_pl(p, w);
    put_player(T, tp, w);
    put_bank(sw, bank);
    const int moves = (int)(misc & 0xFFFFu) + 1;                            // :268-272
    const int ntp = (tp + 1) % P;
    const int turn = moves / 2 + 1;
    misc = (misc & 0xFFFF0000u) | (uint32_t)moves;
    sw[SW_BANK1] = (sw[SW_BANK1] & 0x0000FFFFu) | ((uint32_t)ntp << 16) | ((uint32_t)min(turn, 255) << 24);
    if (turn >= 100) {                                                      // :275-279
        misc |= ST_GAME_OVER | ST_TURN_LIMIT;
        misc &= 0x00FFFFFFu;  // winner None
    } else if ((misc & ST_GAME_OVER) && ntp == 0) {                         // :282-285
        sw[SW_MISC] = misc;
        const int wnr = compute_winner(T);
        misc = (misc & 0x00FFFFFFu) | ((uint32_t)(wnr + 1) << 24);
    }
    sw[SW_MISC] = misc;
}

// ------------------------------------------------------------------------------------------
// observation (engine/encode.py:124-187) into the wave's LDS row block, as bytes
// ------------------------------------------------------------------------------------------
// The wave's rows are packed back to back (row r at byte 297r), so most fields of a lane's row
// sit at unaligned LDS addresses: written field by field they compile to unaligned ds_write_b96
// / b32 accesses that stall the LDS pipe (SQ_LDS_UNALIGNED_STALL) and to ~35 byte writes per row.
// Instead each lane assembles its 297 bytes as 75 dwords in registers (R[j] = bytes 4j..4j+3;
// every offset is a compile-time constant, so R stays in VGPRs) and writes the ALIGNED dwords
// that start inside its row, shifted into place with v_alignbyte_b32; the dword that straddles
// rows L and L+1 is completed with row L+1's first bytes (its bank counts) taken from lane L+1.

// n bytes of v at byte offset o of the row (o, n compile-time after unrolling)
__device__ __forceinline__ void rput(uint32_t (&R)[76], int o, int n, uint32_t v) {
    if (n < 4) v &= (1u << (8 * n)) - 1u;
    const int j = o >> 2, sh = (o & 3) * 8;
    R[j] |= v << sh;
    if (sh != 0 && (o & 3) + n > 4) R[j + 1] |= v >> (32 - sh);
}

__device__ __forceinline__ void rput_card13(uint32_t (&R)[76], int o, uint4 rec, bool present) {
    rput(R, o, 4, present ? rec.x : 0u);
    rput(R, o + 4, 4, present ? rec.y : 0u);
    rput(R, o + 8, 4, present ? rec.z : 0u);
    rput(R, o + 12, 1, present ? rec.w : 0u);
}

// The 297 observation bytes of table T as dwords R[0..74] (R[75] = 0).
template <int P>
__device__ __forceinline__ void build_row(const Tab<P> &T, const Consts &L, uint32_t (&R)[76]) {
    const uint32_t *sw = T.sw;
    const int tp = get_to_play(sw);
#pragma unroll
    for (int j = 0; j < 76; ++j) R[j] = 0u;
    rput(R, 0, 4, sw[SW_BANK0]);                // bank :128
    rput(R, 4, 2, sw[SW_BANK1]);
    uint32_t me[4], op[4];
    get_player(T, tp, me);                      // current :131-135
    get_player(T, (tp + 1) % P, op);            // opponent = next player :138-142
    rput(R, 6, 4, me[0]);
    rput(R, 10, 4, me[1]);
    rput(R, 14, 4, me[2]);
    rput(R, 18, 1, me[3] & 3u);
    rput(R, 19, 4, op[0]);
    rput(R, 23, 4, op[1]);
    rput(R, 27, 4, op[2]);
    rput(R, 31, 1, op[3] & 3u);
#pragma unroll
    for (int k = 0; k < 12; ++k) {              // board :144-147
        const int id = (int)bget(sw[SW_BOARD + k / 4], k % 4);
        rput_card13(R, 32 + 13 * k, card_rec(L, id), id != 0xFF);
    }
    const int mn = (int)(me[3] & 3u), on = (int)(op[3] & 3u), orev = (int)((op[3] >> 2) & 7u);
#pragma unroll
    for (int i = 0; i < 3; ++i) {               // own reserved, always revealed :151-155
        const bool pr = i < mn;
        rput_card13(R, 188 + 14 * i, card_rec(L, (int)bget(me[3], i + 1)), pr);
        rput(R, 188 + 14 * i + 13, 1, pr ? 1u : 0u);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {               // opponent reserved, hidden -> zeros :158-168
        const bool pr = i < on && ((orev >> i) & 1);
        rput_card13(R, 230 + 14 * i, card_rec(L, (int)bget(op[3], i + 1)), pr);
        rput(R, 230 + 14 * i + 13, 1, pr ? 1u : 0u);
    }
    const int nn = (int)bget(sw[SW_DECK], 3);
    const uint32_t owners = (sw[SW_NOB1] >> 8) & 0x7FFFu;
#pragma unroll
    for (int i = 0; i < 3; ++i) {               // nobles[:3] :171-178
        const int idx = (int)bget(sw[SW_NOB0], i);
        const bool pr = i < nn && ((owners >> (3 * i)) & 7u) == 0 && idx < 10;
        const uint2 rec = L.nobles[idx < 10 ? idx : 0];
        rput(R, 272 + 6 * i, 4, pr ? rec.x : 0u);
        rput(R, 276 + 6 * i, 2, pr ? rec.y : 0u);
    }
    rput(R, 290, 3, sw[SW_DECK]);               // deck sizes :180-181
    rput(R, 293, 1, (uint32_t)get_turn(sw));    // misc :183-186
    rput(R, 294, 1, (uint32_t)tp);
    rput(R, 295, 1, (uint32_t)get_moves(sw));   // > 255 patched after the block store
    rput(R, 296, 1, is_terminal(sw) ? 1u : 0u);
}

// Row of table T into rows_base[297*lane ...].  Every lane of the wave must call it (the row
// boundaries are shared with the neighbouring lanes); rows of lanes whose table is not needed
// are written too and simply not stored.
template <int P>
__device__ __forceinline__ void encode_row(const Tab<P> &T, uint8_t *rows_base, const Consts &L) {
    uint32_t R[76];
    build_row(T, L, R);
    // bytes 297..299: the next lane's row bytes 0..2 (its bank counts)
    R[74] |= (uint32_t)__shfl_down((int)R[0], 1) << 8;
    const int lane = lane_id();
    const uint32_t o0 = (4u - ((uint32_t)lane & 3u)) & 3u;  // row 297*lane starts at lane mod 4
    uint32_t *dst = reinterpret_cast<uint32_t *>(rows_base + kObsDim * lane + o0);
#pragma unroll
    for (int j = 0; j < 74; ++j) dst[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], o0);
    if (o0 == 0u) dst[74] = R[74];
}

// Half of encode_row: staged dwords [0, kRowHalf) (Half 0) or [kRowHalf, 75) (Half 1) of every
// lane's row, so two waves of a workgroup encode one block in parallel.  build_row is inlined
// with constant indices, so each half computes only the row bytes its dwords take.
constexpr int kRowHalf = 37;
template <int Half, int P>
__device__ __forceinline__ void encode_row_half(const Tab<P> &T, uint8_t *rows_base, const Consts &L) {
    uint32_t R[76];
    build_row(T, L, R);
    if (Half == 1) R[74] |= (uint32_t)__shfl_down((int)R[0], 1) << 8;
    const int lane = lane_id();
    const uint32_t o0 = (4u - ((uint32_t)lane & 3u)) & 3u;
    uint32_t *dst = reinterpret_cast<uint32_t *>(rows_base + kObsDim * lane + o0);
    constexpr int j0 = Half == 0 ? 0 : kRowHalf, j1 = Half == 0 ? kRowHalf : 74;
#pragma unroll
    for (int j = j0; j < j1; ++j) dst[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], o0);
    if (Half == 1 && o0 == 0u) dst[74] = R[74];
}

// The compact observation row (spl_step_args_t.obs_u8) of table T at rows_base[300*lane ...]:
// the row's 297 bytes, move_count >> 8, two zero bytes — 75 aligned dwords per row (no
// neighbouring-lane bytes).  Part 0: dwords [0, kRowHalf), 1: [kRowHalf, 75), 2: all.
template <int Part, int P>
__device__ __forceinline__ void encode_row_u8(const Tab<P> &T, uint8_t *rows_base, const Consts &L) {
    uint32_t R[76];
    build_row(T, L, R);
    R[74] = (R[74] & 0xFFu) | ((uint32_t)(get_moves(T.sw) >> 8) << 8);
    uint32_t *dst = reinterpret_cast<uint32_t *>(rows_base + kObsU8 * lane_id());
    constexpr int j0 = Part == 1 ? kRowHalf : 0, j1 = Part == 0 ? kRowHalf : 75;
#pragma unroll
    for (int j = j0; j < j1; ++j) dst[j] = R[j];
}

// Observation of table T written by its own lane straight to dst[0..296] (int32; 297 dword
// stores): the rare path for terminal rows that do not fit the pipelined kernel's hand-off.
template <int P>
__device__ __forceinline__ void store_row_direct(const Tab<P> &T, const Consts &L, int32_t *dst) {
    uint32_t R[76];
    build_row(T, L, R);
#pragma unroll
    for (int e = 0; e < kObsDim; ++e) dst[e] = e == 295 ? get_moves(T.sw) : (int32_t)bget(R[e >> 2], e & 3);
}

// Block store of this wave's staged rows: obs[t0 .. t0+rows) as int32, 16 B per lane-store.
// LDS reads are issued in groups of 5 before their stores: one read-wait per store halves the
// store rate (tools/microbench_store.hip: 2.7 -> 5.2 TB/s).
// One 16-byte store per lane per instruction, typed as a native 4 x i32 vector indexed in vector
// units: with `int4` and 32-bit element indexing the compiler versions the loop and, in the
// unrolled copy, splits every store into four strided dword stores (half the store bandwidth).
typedef int v4i __attribute__((ext_vector_type(4)));

// Output-stream store of one 16-byte vector.  NT (the per-step rollout store, written once and
// not read back by this launch): non-temporal, so the 5 GB stream does not push the token table,
// deck records and state out of L2 / the Infinity Cache — the rules wave's gathers stay fast
// (rollout store 1225 -> 1109 us per 64 steps at 65 536 tables).  In-place outputs keep plain
// stores: their block stays Infinity-Cache resident for the consumer (NT: 794 -> 1020 us).
template <bool NT>
__device__ __forceinline__ void st_v4(v4i *p, v4i v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Cache policy of the NT output stream (the rollout store's per-step rows and masks): >= 0 a buffer store
// with that cache-policy immediate (gfx950: sc0 = 1, nt = 2, sc1 = 16) on a resource over the block; -1 the
// compiler's non-temporal store (`global_store_dwordx4 … nt`).  Default 19 = `sc0 nt sc1` (system scope,
// non-temporal): headline 1 941-1 952 against 1 975-2 002 us per launch with `nt` alone, four alternations
// on one box, 1.4 % on another; without nt 12 % slower (profiles/r06/store_policy_ab_r06u_v.txt)
#ifndef SPL_ROLL_CPOL
#define SPL_ROLL_CPOL 19
#endif
// A/B switch: the rollout store's terminal rows and small outputs (reward, terminated, flags, winner)
// through the same policy (0: plain stores)
#ifndef SPL_ROLL_SMALL_NT
#define SPL_ROLL_SMALL_NT 0
#endif
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
// 16-byte output stores into one wave-uniform block under cache policy CP: -2 plain, -1 the compiler's
// non-temporal store, >= 0 a buffer store with that cache-policy immediate
template <int CP>
struct V4Sink {
    v4i *out;
    __amdgpu_buffer_rsrc_t rs;
    __device__ __forceinline__ explicit V4Sink(void *p) : out(reinterpret_cast<v4i *>(p)) {
        if constexpr (CP >= 0) rs = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, 0x7FFFFFF0, 0x00020000);
    }
    __device__ __forceinline__ void put(int i, v4i v) const {
        if constexpr (CP >= 0) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v), rs, i * 16, 0, CP);
        else st_v4<CP == -1>(out + i, v);
    }
};
// the policy of an output stream: the NT stream (SPL_ROLL_CPOL) or plain stores
constexpr int stream_cpol(bool nt) { return nt ? SPL_ROLL_CPOL : -2; }

__device__ __forceinline__ v4i expand4(uint32_t w) {
    v4i v = {(int)(w & 0xFFu), (int)((w >> 8) & 0xFFu), (int)((w >> 16) & 0xFFu), (int)(w >> 24)};
    return v;
}

// Part [d0, d1) (LDS words, multiples of 64*5 except the end) of a FULL wave's observation block.
template <bool NT = false>
__device__ __forceinline__ void store_obs_range(const uint8_t *rows_lds, int32_t *dst, int d0, int d1) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows_lds);
    const V4Sink<stream_cpol(NT)> out(dst);
    constexpr int U = 5;
    int d = d0 + lane_id();
#pragma unroll 1
    for (; d + 64 * (U - 1) < d1; d += 64 * U) {
        uint32_t w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = src[d + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) out.put(d + 64 * u, expand4(w[u]));
    }
    uint32_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = (d + 64 * u < d1) ? src[d + 64 * u] : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (d + 64 * u < d1) out.put(d + 64 * u, expand4(w[u]));
}
constexpr int kObsBlockWords = 64 * kObsDim / 4;  // 4752 LDS words = 4752 16-byte stores per wave
constexpr int kObsSplit = 64 * 5 * 7;             // 2240: 35 stores per lane in the first part

// Block store of this wave's observation rows: LDS bytes [rows][297] -> int32 [rows][297] at
// dst (16-byte aligned: 64-row blocks are 76032 B).  Dword d of the block is LDS word d.
// R = the workgroup's table count (64, or 32 in the half-populated two-wave rollout).
template <int R = 64, bool NT = false, int CP = stream_cpol(NT)>
__device__ __forceinline__ void store_obs_block(const uint8_t *rows_lds, int rows, int32_t *dst) {
    const int nbytes = rows * kObsDim;
    const int full = nbytes >> 2;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows_lds);
    const V4Sink<CP> out(dst);
    constexpr int U = 5;
    int d = lane_id();
    if (rows == R) {  // every wave but a ragged last one: compile-time trip count
        constexpr int kFull = R * kObsDim / 4;  // 64 rows: 4752 = 14 x 320 + 272
#pragma unroll 1
        for (int it = 0; it < kFull / (64 * U); ++it, d += 64 * U) {
            uint32_t w[U];
#pragma unroll
            for (int u = 0; u < U; ++u) w[u] = src[d + 64 * u];
#pragma unroll
            for (int u = 0; u < U; ++u) out.put(d + 64 * u, expand4(w[u]));
        }
        uint32_t w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = (d + 64 * u < kFull) ? src[d + 64 * u] : 0u;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (d + 64 * u < kFull) out.put(d + 64 * u, expand4(w[u]));
        return;
    }
    for (; d < full; d += 64) out.put(d, expand4(src[d]));
    for (int b = (full << 2) + lane_id(); b < nbytes; b += 64) dst[b] = (int32_t)rows_lds[b];
}

// store_obs_block (64 rows) with `mid()` issued between its first and second half: work that fills the
// wave's store-issue stalls instead of following the whole block (k_step_wso's legal mask)
template <bool NT, class Mid, bool NT2 = NT>
__device__ __forceinline__ void store_obs_block_mid(const uint8_t *rows_lds, int rows, int32_t *dst, Mid mid) {
    if (rows != 64) {
        mid();
        store_obs_block<64, NT>(rows_lds, rows, dst);
        return;
    }
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows_lds);
    const V4Sink<stream_cpol(NT)> out(dst);
    const V4Sink<stream_cpol(NT2)> out2(dst);  // the second half (and the tail) may take another store policy
    constexpr int U = 5, kFull = 64 * kObsDim / 4, kIters = kFull / (64 * U);  // 4752 = 14 x 320 + 272
    int d = lane_id();
#pragma unroll 1
    for (int it = 0; it < kIters / 2; ++it, d += 64 * U) {
        uint32_t w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = src[d + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) out.put(d + 64 * u, expand4(w[u]));
    }
    __asm__ volatile("" ::: "memory");
    mid();
    __asm__ volatile("" ::: "memory");
#pragma unroll 1
    for (int it = kIters / 2; it < kIters; ++it, d += 64 * U) {
        uint32_t w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = src[d + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) out2.put(d + 64 * u, expand4(w[u]));
    }
    uint32_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = (d + 64 * u < kFull) ? src[d + 64 * u] : 0u;
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (d + 64 * u < kFull) out2.put(d + 64 * u, expand4(w[u]));
}

// Block store of `rows` compact rows (300 bytes each) staged in LDS to dst (16-byte aligned).
__device__ __forceinline__ void store_obs_u8_block(const uint8_t *rows_lds, int rows, uint8_t *dst) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows_lds);
    const int words = rows * (kObsU8 / 4), chunks = words >> 2;
    v4i *out = reinterpret_cast<v4i *>(dst);
    for (int c = lane_id(); c < chunks; c += 64) {
        const v4i v = {(int)src[4 * c], (int)src[4 * c + 1], (int)src[4 * c + 2], (int)src[4 * c + 3]};
        out[c] = v;
    }
    for (int w = 4 * chunks + lane_id(); w < words; w += 64) reinterpret_cast<uint32_t *>(dst)[w] = src[w];
}

// The compact rows (spl_step_args_t.obs_u8 layout: 297 bytes, move_count >> 8, two zero bytes) of
// the wave's staged 297-byte rows, stored beside their int32 block when a step writes both: 75 dwords
// per row, consecutive lanes on consecutive dwords (256-byte stores); dword j < 74 of row r is the
// staged bytes 297 r + 4 j .. + 3 (one v_alignbyte of the two staged dwords around them), dword 74
// is byte 296, move_count >> 8 (`mhi` of lane r, whose table is row r), 0, 0.  Every lane runs
// every iteration (the row's high byte comes by shuffle), the stores are predicated.  With a 16-byte
// aligned dst each lane builds four consecutive dwords (one 16-byte store; a chunk crosses at most one
// row end, whose dword 74 belongs to the chunk's first row), 19 iterations for 64 rows instead of 75.
__device__ __forceinline__ void store_u8_from_rows(const uint8_t *rows_lds, int rows, uint8_t *dst, uint32_t mhi) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(rows_lds);
    uint32_t *out = reinterpret_cast<uint32_t *>(dst);
    constexpr int kWords = kObsU8 / 4;  // 75
    const int total = rows * kWords;
    int q_first = 0;
    if (((uintptr_t)dst & 15u) == 0) {
        const int chunks = total >> 2;
        v4i *out4 = reinterpret_cast<v4i *>(dst);
        for (int it = 0; it < (chunks + 63) / 64; ++it) {
            const int c = lane_id() + 64 * it, cc = c < chunks ? c : chunks - 1;
            const int q0 = 4 * cc, r0 = q0 / kWords, j0 = q0 - kWords * r0;
            const uint32_t h = (uint32_t)__shfl((int)mhi, r0);
            v4i v;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const bool next = j0 + i >= kWords;  // past row r0's end: row r0 + 1 from its byte 0
                const int j = next ? j0 + i - kWords : j0 + i;
                const int b = kObsDim * (next ? r0 + 1 : r0) + 4 * j;
                uint32_t w = __builtin_amdgcn_alignbyte(src[(b >> 2) + 1], src[b >> 2], (uint32_t)(b & 3));
                if (j0 + i == kWords - 1) w = (w & 0xFFu) | (h << 8);
                v[i] = (int)w;
            }
            if (c < chunks) out4[c] = v;
        }
        q_first = chunks << 2;
    }
    for (int it = 0; it < (total - q_first + 63) / 64; ++it) {
        const int q = q_first + lane_id() + 64 * it, qq = q < total ? q : total - 1;
        const int r = qq / kWords, j = qq - kWords * r;
        const int b = kObsDim * r + 4 * j;  // staged byte; b / 4 + 1 <= 4 677 < 64 * 300 / 4
        uint32_t v = __builtin_amdgcn_alignbyte(src[(b >> 2) + 1], src[b >> 2], (uint32_t)(b & 3));
        const uint32_t h = (uint32_t)__shfl((int)mhi, r);
        if (j == kWords - 1) v = (v & 0xFFu) | (h << 8);
        if (q < total) out[q] = v;
    }
}

// Block store of this wave's masks: mask[t0 .. t0+rows) as int8 [rows][45].  The 64 x 45 mask
// bits are first laid out as ONE bit stream in LDS (row r at bits 45r..45r+44; each stream
// dword is cut from at most two rows), so every output dword is one nibble of the stream,
// spread to 4 bytes by a multiply: bit i of n moves to bit 8i in n * 0x204081.
template <bool NT = false, int CP = stream_cpol(NT)>
__device__ __forceinline__ void store_mask_block(const uint64_t *mask, uint32_t *mbits, int rows, int8_t *dst) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int w = lane_id() + 64 * k;  // stream dword w: bits 32w .. 32w+31
        if (w < kMaskStreamWords) {
            const int r0 = (32 * w) / 45, c0 = 32 * w - 45 * r0;  // first bit: row r0, column c0
            const uint64_t m0 = mask[r0], m1 = r0 + 1 < 64 ? mask[r0 + 1] : 0ull;
            // columns c0..44 of row r0, then row r0+1 from column 0
            const uint64_t lo = m0 >> c0, hi = (c0 > 13) ? (m1 << (45 - c0)) : 0ull;
            mbits[w] = (uint32_t)(lo | hi);
        }
    }
    wave_lds_sync();
    if ((rows == 64 || rows == 32) && ((uintptr_t)dst & 15u) == 0) {  // 180 (90) x 16 B
        const V4Sink<CP> out4(dst);
        const int nc = rows * 45 / 16;
        for (int c = lane_id(); c < nc; c += 64) {
            const uint32_t half = (mbits[c >> 1] >> (16 * (c & 1))) & 0xFFFFu;  // stream bits 16c..16c+15
            v4i v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = (int)((((half >> (4 * q)) & 0xFu) * 0x00204081u) & 0x01010101u);
            out4.put(c, v);
        }
        return;
    }
    const int nbytes = rows * 45;
    const int full = nbytes >> 2;
    uint32_t *out = reinterpret_cast<uint32_t *>(dst);
    for (int d = lane_id(); d < full; d += 64) {
        const uint32_t nib = (mbits[d >> 3] >> (4 * (d & 7))) & 0xFu;
        out[d] = (nib * 0x00204081u) & 0x01010101u;
    }
    for (int b = (full << 2) + lane_id(); b < nbytes; b += 64)
        dst[b] = (int8_t)((mbits[b >> 5] >> (b & 31)) & 1u);
}

// ------------------------------------------------------------------------------------------
// deal: engine/state.py:181-211 initial_state's shuffles, from one engine seed
// ------------------------------------------------------------------------------------------
// Fisher–Yates (Lib/random.py:389-394) over tier 1, 2, 3 decks then the nobles, driven by ONE
// uniform loop over MT outputs: every lane advances its own stream by one output per
// iteration and its own shuffle state machine accepts or rejects it (_randbelow), so the cost
// is the wave's maximum output count, not the sum of per-draw maxima.
struct Deal {
    uint32_t board[3], nob0, nob1;  // SW_BOARD.., SW_NOB0, SW_NOB1 of the dealt table
};
__device__ __forceinline__ Deal empty_deal() { return Deal{{0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, 0xFFFFFFFFu, 0xFFu}; }

__device__ __forceinline__ uint32_t deal_into(uint32_t seed, int P, uint8_t *rec, uint8_t *scr, Deal &out,
                                              uint32_t *mtx) {
    for (int i = 0; i < 100; ++i) scr[i] = (uint8_t)(i < 90 ? i : i - 90);
    MTStream ms;
    ms.init(seed);
    int d = 0, base = 0, i = 39;
    uint32_t flags = 0;
    // _randbelow(i + 1) on output y; a rejected draw (or a finished lane, or `on` false) swaps x[i]
    // with itself.  The caller's LDS reads of the two bytes overlap the next output's computation.
    auto shuffle_step = [&](uint32_t y, bool on, auto &&between) {
        const int n = i + 1;
        const int r = (int)(y >> (32 - bit_length((uint32_t)n)));
        const bool acc = on && d < 4 && r < n;
        const int ai = base + i, ar = base + (acc ? r : i);
        SPL_CHECK(ai >= 0 && ai < 100 && ar >= 0 && ar < 100, BC_SCRATCH);
        const uint8_t xi = scr[ai], xr = scr[ar];
        between();
        scr[ai] = xr;
        scr[ar] = xi;
        const int i2 = acc ? i - 1 : i;
        const bool adv = acc && i2 == 0;  // deck finished: tier 2, tier 3, then the nobles
        d += adv ? 1 : 0;
        base = adv ? (d == 1 ? 40 : (d == 2 ? 70 : 90)) : base;
        i = adv ? (d == 1 ? 29 : (d == 2 ? 19 : 9)) : i2;
    };
    const int limit = min(g_stream_limit, MTStream::kMaxOut);
    uint32_t y = ms.next(0);
    for (int j = 0;; ++j) {
        if (!__any(d < 4)) break;
        if (j >= limit) break;  // lanes still shuffling continue below
        shuffle_step(y, true, [&] {
            if (j + 1 < limit) y = ms.next(j + 1);
        });
    }
    // Continuation past the streamed outputs (never met in natural play): one lane at
    // a time, its full MT19937 state in the LDS region mtx, from output kMaxOut on.
    for (uint64_t slow = __ballot(d < 4); slow; slow &= slow - 1) {
        if (lane_id() == __ffsll((unsigned long long)slow) - 1) {
            LaneMT mt{mtx, 0};
            mt.init(seed);
            mt.start_at(limit);
            while (d < 4) shuffle_step(mt.next(), true, [] {});
        }
    }
    // deck bytes (list order; the 4 dealt cards per tier sit past deck_len)
    const uint32_t *s1 = reinterpret_cast<const uint32_t *>(scr);  // 4-byte aligned scratch
    uint32_t *r1 = reinterpret_cast<uint32_t *>(rec);
#pragma unroll
    for (int q = 0; q < 24; ++q) r1[q] = s1[q];
#pragma unroll
    for (int t = 0; t < 3; ++t) {  // board[tier][i] = deck.pop()
        const int b = tier_base(t), n = tier_size(t);
        out.board[t] = (uint32_t)scr[b + n - 1] | ((uint32_t)scr[b + n - 2] << 8) | ((uint32_t)scr[b + n - 3] << 16) |
                       ((uint32_t)scr[b + n - 4] << 24);
    }
    const int nn = P + 1 < 10 ? P + 1 : 10;  // state.py:194 (<= 5 for P <= 4)
    out.nob0 = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) out.nob0 |= (s < nn ? (uint32_t)scr[90 + s] : 0xFFu) << (8 * s);
    out.nob1 = nn > 4 ? (uint32_t)scr[94] : 0xFFu;
    uint32_t *rw = reinterpret_cast<uint32_t *>(rec);
#pragma unroll
    for (int k = 0; k < 3; ++k) rw[kRecTail / 4 + k] = out.board[k];
    rw[kRecTail / 4 + 3] = out.nob0;
    rw[kRecTail / 4 + 4] = out.nob1;
    rw[kRecSeed / 4] = seed;
    return flags;
}

// the board / noble words of a dealt record (its bytes 96..115)
__device__ __forceinline__ Deal rec_deal(const uint8_t *rec) {
    const uint32_t *rw = reinterpret_cast<const uint32_t *>(rec);
    Deal d;
#pragma unroll
    for (int k = 0; k < 3; ++k) d.board[k] = rw[kRecTail / 4 + k];
    d.nob0 = rw[kRecTail / 4 + 3];
    d.nob1 = rw[kRecTail / 4 + 4];
    return d;
}

template <int P>
__device__ __forceinline__ void fresh_state(Tab<P> &T, uint32_t status, const Deal &d) {
    constexpr uint32_t nn = P + 1 < 10 ? P + 1 : 10;
    T.sw[SW_BANK0] = 0x04040404u;                       // DEFAULT_BANK, state.py:26-33
    T.sw[SW_BANK1] = 4u | (5u << 8) | (0u << 16) | (1u << 24);  // to_play 0, turn_count 1
    T.sw[SW_MISC] = status;                              // move_count 0, winner None
    T.sw[SW_BOARD] = d.board[0];
    T.sw[SW_BOARD + 1] = d.board[1];
    T.sw[SW_BOARD + 2] = d.board[2];
    T.sw[SW_DECK] = 36u | (26u << 8) | (16u << 16) | (nn << 24);  // 40, 30, 20 minus the 4 dealt
    T.sw[SW_NOB0] = d.nob0;
    T.sw[SW_NOB1] = d.nob1;
#pragma unroll
    for (int q = 0; q < P; ++q) {
        T.pw[q][0] = T.pw[q][1] = T.pw[q][2] = 0u;
        T.pw[q][3] = 0xFFFFFF00u;
    }
}

__device__ __forceinline__ Pcg64 load_pcg(const KArena &A, int t) {
    const uint64_t *p = reinterpret_cast<const uint64_t *>(A.pcg + (size_t)t * kPcgBytes);
    const uint32_t *q = reinterpret_cast<const uint32_t *>(p + 4);
    Pcg64 g;
    g.s_hi = p[0];
    g.s_lo = p[1];
    g.inc_hi = p[2];
    g.inc_lo = p[3];
    g.has32 = q[0];
    g.u32 = q[1];
    return g;
}
__device__ __forceinline__ void store_pcg(const KArena &A, int t, const Pcg64 &g) {
    uint64_t *p = reinterpret_cast<uint64_t *>(A.pcg + (size_t)t * kPcgBytes);
    uint32_t *q = reinterpret_cast<uint32_t *>(p + 4);
    p[0] = g.s_hi;
    p[1] = g.s_lo;
    p[2] = g.inc_hi;
    p[3] = g.inc_lo;
    q[0] = g.has32;
    q[1] = g.u32;
}

__device__ __forceinline__ Deal load_pool(const KArena &A, int t) {
    SPL_CHECK(t >= 0 && t < A.n, BC_TABLE);
    Deal d;
#pragma unroll
    for (int k = 0; k < 3; ++k) d.board[k] = A.pool[(size_t)(PL_BOARD + k) * A.n + t];
    d.nob0 = A.pool[(size_t)PL_NOB0 * A.n + t];
    d.nob1 = A.pool[(size_t)PL_NOB1 * A.n + t];
    return d;
}
__device__ __forceinline__ void store_pool(const KArena &A, int t, const Deal &d) {
    SPL_CHECK(t >= 0 && t < A.n, BC_TABLE);
#pragma unroll
    for (int k = 0; k < 3; ++k) A.pool[(size_t)(PL_BOARD + k) * A.n + t] = d.board[k];
    A.pool[(size_t)PL_NOB0 * A.n + t] = d.nob0;
    A.pool[(size_t)PL_NOB1 * A.n + t] = d.nob1;
}

// Deal the next episode into slot record `slot` from the table's engine-seed stream
// (envs/splendor_env.py:43-44: reset() continues self.np_random).  Returns SPL_F_* bits.
// A table never reset with a seed has no stream: it deals engine seed 0 (documented in
// splendor_amd.h) and its record stays unseeded.
template <int P>
__device__ __forceinline__ uint32_t deal_next(const KArena &A, int t, int slot, uint8_t *scr, Deal &d, uint32_t *mtx) {
    Pcg64 g = load_pcg(A, t);
    uint32_t seed = 0u;
    if (g.valid()) {
        seed = g.engine_seed();
        store_pcg(A, t, g);
    }
    return deal_into(seed, P, slot_rec(A, t, slot), scr, d, mtx);
}

template <int P>
__device__ __forceinline__ void load_tab(Tab<P> &T, const KArena &A, int t) {
    SPL_CHECK(t >= 0 && t < A.n, BC_TABLE);
#pragma unroll
    for (int w = 0; w < SW_COUNT; ++w) T.sw[w] = A.planes[(size_t)w * A.n + t];
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) T.pw[q][k] = A.planes[(size_t)pw_index(q, k) * A.n + t];
}

// The table state and its legal-mask cache entry: `legal` is legal_moves of T (as computed under the
// context tagged `tag`), or anything with tag 0 when the storing kernel does not know it.  Every
// kernel that stores state goes through here, so no stale mask survives a state change.
template <int P>
__device__ __forceinline__ void store_words(const Tab<P> &T, const KArena &A, int t) {  // state words only
    SPL_CHECK(t >= 0 && t < A.n, BC_TABLE);
#pragma unroll
    for (int w = 0; w < SW_COUNT; ++w) A.planes[(size_t)w * A.n + t] = T.sw[w];
#pragma unroll
    for (int q = 0; q < P; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) A.planes[(size_t)pw_index(q, k) * A.n + t] = T.pw[q][k];
}
__device__ __forceinline__ void store_legal(const KArena &A, int t, uint64_t legal, uint32_t tag) {
    A.legal[t] = (uint32_t)legal;
    A.legal[A.n + t] = ((uint32_t)(legal >> 32) & kLegalHiBits) | (tag << kLegalTagShift);
}
template <int P>
__device__ __forceinline__ void store_tab(const Tab<P> &T, const KArena &A, int t, uint64_t legal, uint32_t tag) {
    store_words(T, A, t);
    store_legal(A, t, legal, tag);
}

// the cached legal mask of table t's stored state, if it was computed under context tag `tag`
struct LegalCache {
    uint32_t lo, hi;
    // tag 0 is "unknown" on both sides: an entry a crafted upload left, and a context without a tag of its
    // own (card_table_tag ran out) never trusts an entry
    __device__ __forceinline__ bool known(uint32_t tag) const { return tag != 0u && (hi >> kLegalTagShift) == tag; }
    __device__ __forceinline__ uint64_t mask() const { return (uint64_t)lo | ((uint64_t)(hi & kLegalHiBits) << 32); }
};
__device__ __forceinline__ LegalCache load_legal(const KArena &A, int t) {
    return LegalCache{A.legal[t], A.legal[A.n + t]};
}

__device__ __forceinline__ void load_tables_lds(Consts &L, const KTables &Tb) {
    for (int i = lane_id(); i < 90; i += 64) L.cards[i] = Tb.cards[i];
    if (lane_id() < 10) L.nobles[lane_id()] = Tb.nobles[lane_id()];
}
// The same tables by LDS-DMA from ONE wave (global_load_lds, 16 B per lane: 90 card records, then the
// 80-B noble array as five 16-B pieces): no registers and no LDS write instructions, and the issuing
// wave's own vmcnt covers their landing — a later s_waitcnt vmcnt(0) of that wave makes them readable
// to it, and a barrier after that to the workgroup.
typedef __attribute__((address_space(3))) void lds_void_t;
__device__ __forceinline__ void dma_tables_lds(Consts &L, const KTables &Tb) {
    const int lane = lane_id();
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(Tb.cards + lane), (lds_void_t *)&L.cards[0], 16, 0, 0);
    if (lane < 26)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(Tb.cards + 64 + lane), (lds_void_t *)&L.cards[64],
                                         16, 0, 0);
    if (lane < 5)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint8_t *>(Tb.nobles) + 16 * lane,
                                         (lds_void_t *)&L.nobles[0], 16, 0, 0);
}

template <int P>
__device__ __forceinline__ uint64_t legal_of(const Tab<P> &T, const Consts &L) {
    uint32_t w[4];
    get_player(T, get_to_play(T.sw), w);
    const Pl p = unpack_pl(w);
    int bank[6];
    get_bank(T.sw, bank);
    return legal_mask(T.sw, p, bank, L);
}

// the uniform policy's Philox(seed; table, ply) word: independent of the state, so a wave with spare
// time can draw it ahead (the dealer rollout's output wave, two steps ahead of the rules wave)
__device__ __forceinline__ uint32_t uniform_draw(uint64_t seed, uint64_t table, uint64_t ply) {
    return philox4x32(make_uint4((uint32_t)table, (uint32_t)(table >> 32), (uint32_t)ply, (uint32_t)(ply >> 32)),
                      make_uint2((uint32_t)seed, (uint32_t)(seed >> 32))).x;
}
// uniform-random legal action from a drawn word: scaled to the legal count, the k-th legal action
__device__ __forceinline__ int sample_uniform_word(uint64_t m, uint32_t rx) {
    const int n = __popcll(m);
    if (n == 0) return 0;
    int k = (int)(((uint64_t)rx * (uint64_t)n) >> 32);
    // position of the k-th set bit
    uint64_t mm = m;
    int pos = 0;
#pragma unroll
    for (int width = 32; width >= 1; width >>= 1) {
        const uint64_t low = mm & ((1ull << width) - 1ull);
        const int c = __popcll(low);
        const bool up = k >= c;
        k -= up ? c : 0;
        pos += up ? width : 0;
        mm = up ? (mm >> width) : low;
    }
    return pos;
}
// uniform-random legal action: Philox(seed; table, ply) scaled to the legal count
__device__ __forceinline__ int sample_uniform(uint64_t m, uint64_t seed, uint64_t table, uint64_t ply) {
    return sample_uniform_word(m, uniform_draw(seed, table, ply));
}

// scripts/eval_suite.py opponents over a 45-bit legal mask; their random choices are Philox
// draws (sample_uniform over the preferred subset) where the reference calls np.random.choice.
constexpr uint64_t kBuyBits = (((1ull << 12) - 1ull) << 15) | (7ull << 42);  // 15..26, 42..44
constexpr uint64_t kTake2Bits = 0x1Full << 10, kTake3Bits = 0x3FFull, kReserveBits = ((1ull << 15) - 1ull) << 27;
__device__ __forceinline__ int lowest_action(uint64_t m) { return m ? __ffsll((unsigned long long)m) - 1 : 0; }

template <int P>
__device__ __forceinline__ int policy_action(int policy, uint64_t m, const Tab<P> &T, const Consts &L,
                                             uint64_t seed, uint64_t table, uint64_t ply) {
    if (policy == SPL_POLICY_GREEDY_V1) {  // eval_suite.py:9-29: first legal buy, take-2, take-3, reserve
        const uint64_t pick = (m & kBuyBits) ? (m & kBuyBits)
                              : (m & kTake2Bits) ? (m & kTake2Bits)
                              : (m & kTake3Bits) ? (m & kTake3Bits)
                              : (m & kReserveBits) ? (m & kReserveBits) : m;
        return lowest_action(pick);
    }
    if (policy == SPL_POLICY_BASIC_PRIORITY) {  // eval_suite.py:32-78
        const uint64_t vis = m & (((1ull << 12) - 1ull) << 15);
        uint64_t pick;
        if (vis) {  // visible buys with the most points (board points: obs[32 + 13k + 2])
            int best = -1;
            uint64_t best_set = 0;
#pragma unroll
            for (int k = 0; k < 12; ++k) {
                const bool legal = (vis >> (15 + k)) & 1ull;
                const int pts = (int)bget(card_rec(L, board_get(T.sw, k)).x, 2);
                const bool better = legal && pts > best, tie = legal && pts == best;
                best_set = better ? (1ull << (15 + k)) : (tie ? (best_set | (1ull << (15 + k))) : best_set);
                best = better ? pts : best;
            }
            pick = best_set;
        } else {
            pick = (m & (7ull << 42)) ? (m & (7ull << 42))
                   : (m & kTake3Bits) ? (m & kTake3Bits)
                   : (m & kTake2Bits) ? (m & kTake2Bits)
                   : (m & kReserveBits) ? (m & kReserveBits) : 0ull;
            if (!pick) return lowest_action(m);
        }
        return sample_uniform(pick, seed, table, ply);
    }
    return sample_uniform(m, seed, table, ply);
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------

// Token-return table: for every (turn_count, to_play, sum(tokens), sum(bank)) in the domain,
// the top 3 bits of the first 40 outputs of random.Random(seed) (engine/rules.py:170-176).
__global__ __launch_bounds__(64) void k_build_lut(uint4 *lut) {
    const int e = blockIdx.x * 64 + lane_id();
    if (e >= kLutEntries) return;
    const int sb = e % kLutSb, st = 11 + (e / kLutSb) % kLutSt, tp = (e / (kLutSb * kLutSt)) % kLutTp,
              tc = e / (kLutSb * kLutSt * kLutTp);
    const uint64_t seed = ((uint64_t)tc * 1315423911ull) ^ ((uint64_t)tp * 2654435761ull) ^ ((uint64_t)st * 97531ull) ^
                          ((uint64_t)sb * 31337ull);
    MTStream ms;
    ms.init(seed);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int j = 0; j < kLutOutputs; ++j) {
        const uint32_t top = ms.next(j) >> 29;
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] |= (j / 10 == q) ? top << (3 * (j % 10)) : 0u;
    }
    lut[e] = make_uint4(w[0], w[1], w[2], w[3]);
}

// ---- one env step of one table, shared by k_step and k_rollout ----------------------------

// Loads a step needs beyond the table state, issued as early as the action is known: the deck
// card the action pops and the token-return table entry it consults (predict_lut_key).
struct StepPre {
    uint32_t top;
    int key;
    uint4 e;
};

template <int P>
__device__ __forceinline__ StepPre step_prefetch(const Tab<P> &T, int action, bool valid, const KArena &A, int t,
                                                 const KTables &Tb) {
    StepPre pre{0xFFu, -1, make_uint4(0u, 0u, 0u, 0u)};
    const bool live_tab = valid && !is_terminal(T.sw);
    const int ptier = pop_tier(action);
    if (live_tab && ptier >= 0) {
        const int len = (int)bget(T.sw[SW_DECK], ptier);
        const uint8_t *live = live_rec(A, t, T.sw[SW_MISC]);
        SPL_CHECK(len <= tier_size(ptier), BC_DECK);
        if (len > 0) pre.top = abl(ABL_DECK_GATHER) ? (uint32_t)(len + 3 * ptier) : live[tier_base(ptier) + len - 1];
    }
    if (live_tab && action >= 0 && action < SPL_NUM_ACTIONS) {
        const int tp = get_to_play(T.sw);
        uint32_t pw4[4];
        get_player(T, tp, pw4);
        int bank[6];
        get_bank(T.sw, bank);
        pre.key = predict_lut_key(unpack_pl(pw4), bank, action, get_turn(T.sw), tp);
        SPL_CHECK(pre.key < kLutEntries, BC_LUT);
        if (pre.key >= 0) pre.e = abl(ABL_LUT_GATHER) ? make_uint4(0x12345678u, 0x9abcdef0u, 0x0fedcba9u, (uint32_t)pre.key) : Tb.lut[pre.key];
    }
    return pre;
}

constexpr uint64_t kMaskDeferred = 1ull << 63;  // step_rules(defer_mask): legal mask still to evaluate

struct StepOut {
    uint32_t flags;
    float reward;
    bool term;
    uint64_t mask;  // info["action_mask"] after the step (before any autoreset)
};

// envs/splendor_env.py:51-90 on the table in registers.  `known` (k_rollout after its first
// step): `known_mask` is legal_moves of the table's current state, computed by the previous step,
// so "any legal move?" and mask[action] need no re-evaluation.
template <int P, class Stamp = NoStamp>
__device__ __forceinline__ StepOut step_rules(Tab<P> &T, int action, const StepPre &pre, bool valid, const Consts &L,
                                              const KTables &Tb, uint32_t *mtx, bool known = false,
                                              uint64_t known_mask = 0ull, bool defer_mask = false,
                                              Stamp stamp = Stamp()) {
    StepOut o{0u, 0.0f, false, 0ull};
    bool want_mask = false;
    if (valid) {
        if (is_terminal(T.sw)) {                                  // :53-54 RuntimeError
            o.flags = SPL_F_AFTER_TERMINAL;
        } else {
            const bool in_range = action >= 0 && action < SPL_NUM_ACTIONS;
            uint32_t pw4[4];
            get_player(T, get_to_play(T.sw), pw4);
            const Pl cur = unpack_pl(pw4);
            int bank[6];
            get_bank(T.sw, bank);
            // :55 mask = legal_moves(state): only "any legal?" and mask[action] are needed here
            bool anyl, ok;
            if (known) {
                anyl = known_mask != 0ull;
                ok = in_range && ((known_mask >> (action & 63)) & 1ull);
            } else {
                anyl = abl(ABL_LEGAL_PRE) || any_legal(T.sw, cur, bank, L);
                ok = abl(ABL_LEGAL_PRE) || (in_range && action_legal(T.sw, cur, bank, action, L));
            }
            if (!anyl) {                                          // :56-61 no legal move: draw
                T.sw[SW_MISC] = (T.sw[SW_MISC] | ST_GAME_OVER) & 0x00FFFFFFu;
                T.sw[SW_BANK1] &= 0xFF00FFFFu;                    // to_play = 0
                o.term = true;
                o.flags = SPL_F_DRAW;
            } else if (!in_range) {                               // :62-63 ValueError, mask of the unchanged state
                o.flags = SPL_F_OOB;
                want_mask = true;
            } else if (!ok) {                                     // :64-66 illegal, mask of the unchanged state
                o.flags = SPL_F_ILLEGAL;
                o.reward = -0.01f;
                want_mask = true;
            } else {
                STAMP(2);
                stamp(4);
                if (!abl(ABL_APPLY)) apply_action(T, action, pre.top, L, Tb.lut, pre.key, pre.e, mtx, stamp);  // :68
                STAMP(3);
                stamp(5);
                o.term = is_terminal(T.sw);                       // :70
                if (o.term) {                                     // :71-80
                    const int w = get_winner(T.sw);
                    const bool tl = (T.sw[SW_MISC] & ST_TURN_LIMIT) != 0;
                    o.reward = (w < 0 && tl) ? -0.1f : (w < 0 ? 0.0f : (w == P - 1 ? 1.0f : -1.0f));
                    o.flags |= tl ? SPL_F_TURN_LIMIT : 0u;        // :82-83
                } else {
                    want_mask = true;                             // :81
                }
            }
        }
    }
    stamp(6);
    // one legal_moves evaluation per lane (a single call site keeps one copy in the code).
    // defer_mask: left to the caller (kMaskDeferred marks the lanes that need it; k_step_ws
    // evaluates it after handing the state to its output wave)
    if (defer_mask) o.mask = want_mask ? kMaskDeferred : 0ull;
    else if (want_mask) o.mask = abl(ABL_LEGAL_POST) ? (uint64_t)action : legal_of(T, L);
    return o;
}

// player 0's final reward of a finished episode (envs/splendor_env.py:92-115)
template <int P>
__device__ __forceinline__ float final_reward_p0(const Tab<P> &T) {
    const int w = get_winner(T.sw);
    const bool tl = (T.sw[SW_MISC] & ST_TURN_LIMIT) != 0;
    return w < 0 ? (tl ? -0.1f : 0.0f) : (w == 0 ? 1.0f : -1.0f);
}

// Reset to the next episode of the table's engine-seed stream (envs/splendor_env.py:43-44:
// reset() continues self.np_random): the live record moves to the next pool record, whose
// board / noble words `pool` holds.  With every pool record consumed since the last refill the
// next one is dealt inline — correct, only slower.  When the pool record after it is dealt, its
// words are gathered into `pool` for the next reset (the caller stores them to the pool
// planes); returns true in that case.
template <int P>
__device__ __forceinline__ bool flip_to_pool(Tab<P> &T, const KArena &A, int t, Deal &pool, uint8_t *scr,
                                             uint32_t *mtx, uint32_t &flags) {
    constexpr int kPools = kSlotRecords - 1;
    const uint32_t misc = T.sw[SW_MISC];
    const int a = active_of(misc), pend = pend_of(misc);
    const int nxt = (a + 1) % kSlotRecords;
    if (pend >= kPools) flags |= deal_next<P>(A, t, nxt, scr, pool, mtx);
    const int pend2 = pend >= kPools ? kPools : pend + 1;  // the old live record is free now
    fresh_state(T, ring_bits(nxt, pend2), pool);
    if (pend2 < kPools) pool = rec_deal(slot_rec(A, t, (nxt + 1) % kSlotRecords));
    return pend2 < kPools;
}

// One pool refill of table t (spl_refill's unit of work; status `misc` has pend > 0): re-deal the
// earliest consumed record in ring order (the next episode's deal comes first in the engine-seed
// stream).  When that record is the next pool, its words go to `pool` (`pool_dirty`).  Returns
// the new status word.
template <int P>
__device__ __forceinline__ uint32_t refill_table(const KArena &A, int t, uint32_t misc, uint8_t *scr, uint32_t *mtx,
                                                 Deal &pool, bool &pool_dirty) {
    const int pend = pend_of(misc);
    const int slot = (active_of(misc) + kSlotRecords - pend) % kSlotRecords;
    Deal d;
    deal_next<P>(A, t, slot, scr, d, mtx);
    if (pend == kSlotRecords - 1) {
        pool = d;
        pool_dirty = true;
    }
    return (misc & ~ST_PEND) | ((uint32_t)(pend - 1) << ST_PEND_SHIFT);
}

// same-step autoreset of a terminal table; `pool_dirty` is set when the pool planes changed
template <int P>
__device__ __forceinline__ void autoreset_table(Tab<P> &T, const KArena &A, int t, Deal &pool, uint8_t *scr,
                                                uint32_t *mtx, StepOut &o, bool &pool_dirty) {
    pool_dirty |= flip_to_pool<P>(T, A, t, pool, scr, mtx, o.flags);
    o.flags |= SPL_F_RESET;
    o.mask = kFreshDealMask;
}

// Terminal rows staged in L.frows (bits of `fin`) -> final_obs rows of this wave.
__device__ __forceinline__ void store_final_rows(const uint8_t *rows_lds, uint64_t fin, int32_t *final_obs, int t0) {
    while (fin) {
        const int r = __ffsll((unsigned long long)fin) - 1;
        fin &= fin - 1;
        int32_t *dst = final_obs + (size_t)(t0 + r) * kObsDim;
        for (int e = lane_id(); e < kObsDim; e += 64) dst[e] = (int32_t)rows_lds[r * kObsDim + e];
    }
}

// ---- column-parallel rows (round 4) --------------------------------------------------------
// A terminal table's info["final_observation"] row encoded by the whole wave: lane l owns bytes
// e = l + 64 i (i < 5) of the ONE row and stores them as int32, coalesced (five 256-byte dword
// stores).  encode_row's lane-per-row form costs every lane a whole row even when one or two of the
// wave's 64 tables ended (random 4-player games end every ~30 steps: most steps), which made the
// 4-player output wave's encode 4.4 us against 2.6 us at 2 players.  Here a byte is one or two LDS
// reads plus a few VALU ops, driven by a per-lane recipe built once per launch (col_recipe): which
// state word holds it (absolute, or a word of the player to move / the next player), which byte of
// that word, and whether it names a card / noble whose record byte is the value
// (engine/encode.py:124-187; the same fields as build_row).
enum : uint32_t {
    CK_BYTE = 0,      // the byte itself
    CK_NRES = 1,      // & 3 (n_reserved of PW3)
    CK_BOARD = 2,     // board card id -> record byte f (0 when the slot is empty)
    CK_OWN_RES = 3,   // own reserved card slot s (PW3 byte s + 1) -> record byte f, f == 13: present
    CK_OPP_RES = 4,   // opponent's reserved slot s: as own, hidden (not revealed) -> zeros
    CK_NOBLE = 5,     // visible noble slot s (SW_NOB0 byte s) -> noble record byte f
    CK_MOVES = 6,     // move_count, the full value (no byte patch needed)
    CK_TERMINAL = 7,  // game_over and to_play == 0
    CK_NONE = 8       // past the row
};
// recipe: word (5 bits) | rel << 5 (0 absolute, 1 to_play's PW, 2 next player's PW) | byte << 7 |
//         kind << 9 | f << 13 | s << 17
__device__ __forceinline__ uint32_t col_recipe(int e) {
    auto R = [](int w, int rel, int b, uint32_t kind, int f = 0, int s = 0) {
        return (uint32_t)w | ((uint32_t)rel << 5) | ((uint32_t)b << 7) | (kind << 9) | ((uint32_t)f << 13) |
               ((uint32_t)s << 17);
    };
    if (e >= kObsDim) return R(0, 0, 0, CK_NONE);
    if (e < 4) return R(SW_BANK0, 0, e, CK_BYTE);                                   // bank :128
    if (e < 6) return R(SW_BANK1, 0, e - 4, CK_BYTE);
    if (e < 32) {                                                                    // players :131-142
        const int rel = e < 19 ? 1 : 2, q = e - (e < 19 ? 6 : 19);
        return q < 12 ? R(q >> 2, rel, q & 3, CK_BYTE) : R(3, rel, 0, CK_NRES);
    }
    if (e < 188) {                                                                   // board :144-147
        const int k = (e - 32) / 13;
        return R(SW_BOARD + k / 4, 0, k % 4, CK_BOARD, (e - 32) % 13);
    }
    if (e < 272) {                                                                   // reserved :151-168
        const bool own = e < 230;
        const int q = e - (own ? 188 : 230), s = q / 14;
        return R(3, own ? 1 : 2, s + 1, own ? CK_OWN_RES : CK_OPP_RES, q % 14, s);
    }
    if (e < 290) {                                                                   // nobles[:3] :171-178
        const int s = (e - 272) / 6;
        return R(SW_NOB0, 0, s, CK_NOBLE, (e - 272) % 6, s);
    }
    if (e < 293) return R(SW_DECK, 0, e - 290, CK_BYTE);                            // deck sizes :180-181
    if (e == 293) return R(SW_BANK1, 0, 3, CK_BYTE);                                // turn_count :183
    if (e == 294) return R(SW_BANK1, 0, 2, CK_BYTE);                                // to_play :184
    if (e == 295) return R(SW_MISC, 0, 0, CK_MOVES);                                // move_count :185
    return R(SW_MISC, 0, 0, CK_TERMINAL);                                           // terminal :186
}
struct ColRecipes {
    uint32_t r[5];
};
__device__ __forceinline__ ColRecipes col_recipes() {
    ColRecipes c;
#pragma unroll
    for (int i = 0; i < 5; ++i) c.r[i] = col_recipe(lane_id() + 64 * i);
    return c;
}

// One table's observation row, column-parallel (wave-uniform call): word w of the table's state is
// st[w * stride] in LDS (st and stride uniform); v[i] = column lane + 64 i of the row.
template <int P>
__device__ __forceinline__ void row_columns(const uint32_t *st, int stride, const Consts &L, const ColRecipes &C,
                                            uint32_t (&v)[5]) {
    const uint32_t bank1 = st[SW_BANK1 * stride], misc = st[SW_MISC * stride];
    const int tp = (int)bget(bank1, 2), np = (tp + 1) % P;
    const uint32_t deck = st[SW_DECK * stride], owners = (st[SW_NOB1 * stride] >> 8) & 0x7FFFu;
    const uint8_t *cb = reinterpret_cast<const uint8_t *>(L.cards);
    const uint8_t *nb = reinterpret_cast<const uint8_t *>(L.nobles);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t r = C.r[i];
        const int w0 = (int)(r & 31u), rel = (int)((r >> 5) & 3u), b = (int)((r >> 7) & 3u);
        const uint32_t kind = (r >> 9) & 15u;
        const int f = (int)((r >> 13) & 15u), s = (int)((r >> 17) & 3u);
        const int widx = rel == 0 ? w0 : pw_index(rel == 1 ? tp : np, w0);
        const uint32_t w = st[widx * stride];
        const uint32_t byte = bget(w, b);
        // the record byte a card / noble kind reads (address clamped: read unconditionally)
        const bool is_noble = kind == CK_NOBLE;
        const uint32_t id = byte < (is_noble ? 10u : 90u) ? byte : 0u;
        const uint32_t rec = is_noble ? (uint32_t)nb[id * 8 + (f < 6 ? f : 0)] : (uint32_t)cb[id * 16 + (f < 13 ? f : 0)];
        const int nres = (int)(w & 3u), rev = (int)((w >> 2) & 7u);
        const bool res_pr = s < nres && (kind == CK_OWN_RES || ((rev >> s) & 1));
        const bool nob_pr = s < (int)bget(deck, 3) && ((owners >> (3 * s)) & 7u) == 0u && byte < 10u;
        uint32_t out = byte;
        out = kind == CK_NRES ? (w & 3u) : out;
        out = kind == CK_BOARD ? (byte != 0xFFu ? rec : 0u) : out;
        out = (kind == CK_OWN_RES || kind == CK_OPP_RES) ? (res_pr ? (f == 13 ? 1u : rec) : 0u) : out;
        out = is_noble ? (nob_pr ? rec : 0u) : out;
        out = kind == CK_MOVES ? (misc & 0xFFFFu) : out;
        out = kind == CK_TERMINAL ? (((misc & ST_GAME_OVER) && tp == 0) ? 1u : 0u) : out;
        v[i] = out;
    }
}
template <int P>
__device__ __forceinline__ void store_row_columns(const uint32_t *st, int stride, const Consts &L, const ColRecipes &C,
                                                  int32_t *dst) {
    uint32_t v[5];
    row_columns<P>(st, stride, L, C, v);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const int e = lane_id() + 64 * i;
        if (e < kObsDim) dst[e] = (int32_t)v[i];
    }
}
// the same through the NT output stream's cache policy (SPL_ROLL_CPOL; dst wave-uniform)
template <int P>
__device__ __forceinline__ void store_row_columns_nt(const uint32_t *st, int stride, const Consts &L, const ColRecipes &C,
                                                     int32_t *dst) {
#if SPL_ROLL_CPOL >= 0
    uint32_t v[5];
    row_columns<P>(st, stride, L, C, v);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, kObsDim * 4, 0x00020000);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const int e = lane_id() + 64 * i;
        if (e < kObsDim) __builtin_amdgcn_raw_buffer_store_b32(v[i], rs, e * 4, 0, SPL_ROLL_CPOL);
    }
#else
    store_row_columns<P>(st, stride, L, C, dst);
#endif
}
// spl_step_args_t.gate_*: the dual step's opponent moves only where the agent's move was applied
// and left the game running (wrappers/dual_step_native.py:120-140, spl_dual_gate); elsewhere its
// action becomes -1 (out of range: no move), written back so the caller sees the gated action.
__device__ __forceinline__ int gated_action(const KStep &S, int t) {
    int action = S.actions[t];
    if (S.gate_terminated && (S.gate_terminated[t] != 0 || (S.gate_flags[t] & (SPL_F_ILLEGAL | SPL_F_OOB)) != 0)) {
        action = -1;
        const_cast<int32_t *>(S.actions)[t] = -1;
    }
    return action;
}

// spl_step's gymnasium info planes (illegal_action, draw, turn_limit as 0/1 bytes; truncated = 0) and the running
// count of tables whose flags carry the reference's exceptions (out-of-range action, step after
// termination): one atomic per wave that has any.  Wave-uniform call (the ballot).
__device__ __forceinline__ void store_step_info(const KStep &S, int n, int t, bool valid, uint32_t f) {
    if (S.info && valid) {
        S.info[t] = (f & SPL_F_ILLEGAL) ? 1 : 0;
        S.info[(size_t)n + t] = (f & SPL_F_DRAW) ? 1 : 0;
        S.info[2 * (size_t)n + t] = (f & SPL_F_TURN_LIMIT) ? 1 : 0;
        S.info[3 * (size_t)n + t] = 0;  // truncated
    }
    if (S.errors) {
        const uint64_t bad = __ballot(valid && (f & (SPL_F_OOB | SPL_F_AFTER_TERMINAL)) != 0);
        if (bad && lane_id() == __ffsll((unsigned long long)bad) - 1)
            atomicAdd(S.errors, (unsigned long long)__popcll(bad));
    }
}

// SplendorEnv.step for every table (envs/splendor_env.py:51-90) + same-step autoreset.
//
// Every global load of the step (state, action, pool deal words, the deck card the action
// pops, the token-return table entry it consults) is issued in the first microseconds, before
// any wave has started its stores; from there to the block stores at the end the wave touches
// only registers and LDS.  A load issued later would queue behind the other waves' observation
// writes (tens of MB in flight) and its wave would become the kernel's tail.
//
// W waves per workgroup (64 tables each, independent except for the shared constant tables):
// fewer, larger workgroups reach the whole chip sooner than 64-thread ones.
template <int P, int W>
__global__ __launch_bounds__(64 * W) void k_step(KArena A, KTables Tb, KStep S) {
    __shared__ StepLDS<W> SL;
    Consts &L = SL;
    const int wave = W == 1 ? 0 : (int)(threadIdx.x >> 6);
    WaveBuf &B = SL.w[wave];
    const int lane = lane_id();
    const int t0 = (blockIdx.x * W + wave) * 64;
    const int t = t0 + lane;
    const bool valid = t < A.n;
    const int rows = max(0, min(64, A.n - t0));
    STAMP(0);
    if (W == 1) {
        load_tables_lds(L, Tb);
    } else {
        for (int i = threadIdx.x; i < 90; i += 64 * W) L.cards[i] = Tb.cards[i];
        if (threadIdx.x < 10) L.nobles[threadIdx.x] = Tb.nobles[threadIdx.x];
    }

    Tab<P> T;
    int action = 0;
    Deal pool = empty_deal();
    if (valid && !abl(ABL_LOAD)) {
        load_tab(T, A, t);
        action = gated_action(S, t);
        if (S.autoreset) pool = load_pool(A, t);
    } else {
        fresh_state(T, 0u, empty_deal());
    }
    if (W == 1) wave_lds_sync();
    else __syncthreads();  // the constant tables (nothing stored yet: no store drain to wait for)
    const StepPre pre = step_prefetch(T, action, valid, A, t, Tb);
    STAMP(1);

    // LDS for a token-return continuation (LaneMT): the observation rows past the deal scratch
    uint32_t *const mtx = reinterpret_cast<uint32_t *>(&B.rows[64 * kScratchStride]);
    StepOut o = step_rules(T, action, pre, valid, L, Tb, mtx);
    // autoreset 2: a table terminal on entry is re-dealt without a move (dual-step opponent phase)
    const bool entry_reset = valid && S.autoreset == 2 && (o.flags & SPL_F_AFTER_TERMINAL);
    if (entry_reset) o.flags = 0u;
    const bool ended = valid && (o.term || entry_reset);
    const int8_t wnr = (int8_t)get_winner(T.sw);
    STAMP(4);

    // terminal observation for gymnasium's info["final_observation"], staged in LDS and stored
    // with everything else at the end
    const bool want_final = S.autoreset && S.final_obs != nullptr && !abl(ABL_FINAL);
    const uint64_t fin = __ballot(ended && want_final);
    if (__any(ended && want_final)) encode_row(T, B.frows, L);  // rows of other lanes are not stored
    const int fin_moves = get_moves(T.sw);
    const float ep_add = (valid && o.term) ? final_reward_p0(T) : 0.0f;
    STAMP(5);
    bool pool_dirty = false;
    if (ended && S.autoreset && !abl(ABL_RESET))
        autoreset_table(T, A, t, pool, &B.rows[lane * kScratchStride], mtx, o, pool_dirty);
    STAMP(6);
    wave_lds_sync();  // deal scratch (rows) free again

    // observation + mask of the current state, block stores
    if (!abl(ABL_ENCODE)) encode_row(T, B.rows, L);
    B.mask[lane] = o.mask;
    STAMP(7);
    wave_lds_sync();
    STAMP(8);
    if (!abl(ABL_STORE)) {
        if (!abl(ABL_OBS_STORE)) store_obs_block(B.rows, rows, S.obs + (size_t)t0 * kObsDim);
        STAMP(9);
        if (!abl(ABL_MASK_STORE)) store_mask_block(B.mask, B.mbits, rows, S.mask + (size_t)t0 * 45);
    }
    store_final_rows(B.frows, fin, S.final_obs, t0);
    STAMP(10);
    if (valid && o.term) {  // no-return atomics: nothing to wait for
        if (S.ep_return) unsafeAtomicAdd(&S.ep_return[t], ep_add);
        if (S.ep_count) atomicAdd(&S.ep_count[t], 1u);
    }
    // move_count above 255 (crafted states only) does not fit the byte staging: patch it after
    // this wave's block stores of the same dwords have left
    const bool patch = valid && get_moves(T.sw) > 255;
    const bool fpatch = ended && want_final && fin_moves > 255;
    if (__any(patch || fpatch)) {
        __builtin_amdgcn_s_waitcnt(0);
        if (patch) S.obs[(size_t)t * kObsDim + 295] = get_moves(T.sw);
        if (fpatch) S.final_obs[(size_t)t * kObsDim + 295] = fin_moves;
    }
    store_step_info(S, A.n, t, valid, o.flags);
    if (valid) {
        if (!abl(ABL_SMALL_OUT)) {
            S.reward[t] = o.reward;
            S.terminated[t] = o.term ? 1 : 0;
            S.flags[t] = (uint8_t)o.flags;
            if (S.winner) S.winner[t] = wnr;
        }
        if (S.next_actions) {
            const uint64_t ply = S.ply + (S.ply_base ? *S.ply_base : 0ull);
            S.next_actions[t] = policy_action(S.policy, o.mask, T, L, S.policy_seed, (uint64_t)(S.table0 + t), ply);
        }
        if (!abl(ABL_TAB_STORE)) store_tab(T, A, t, o.mask, Tb.mtag);
        if (pool_dirty) store_pool(A, t, pool);
    }
    STAMP(11);
}

// K consecutive env steps of every table with the device uniform-random policy: exactly K
// k_step launches with next_actions fed back as the next launch's actions (plies ply ..
// ply+K-1), without the launch boundaries.  The table state stays in registers; each step's
// block stores are issued and left to drain while the wave computes the next step, and the
// next step's deck-card / token-table gathers are issued a whole step ahead.  Step k's outputs
// go to block k of each output array when `per_step` (rollout storage [K][n][...]), else every
// step overwrites block 0.
//
// refill != 0 (a pool refill is due in this launch): the refill is fused — each wave re-deals its
// tables' earliest consumed pool record (k_refill's work) at a step of its own, spread over the
// K steps.  The deal is a long serial integer chain per lane; inside the rollout it runs while
// this wave's stores drain and the other waves keep HBM busy, where a separate k_refill launch
// leaves HBM idle for its whole duration.  Trajectories do not depend on when a refill happens
// (deals are taken from each table's engine-seed stream in episode order either way).
// Fused pool refills of one rollout launch: `count` refills (one per refill period the launch
// crosses), one per segment of K / count steps, each workgroup at its own offset within the segment
// so that deals (VALU-bound) overlap other workgroups' stores.  Results do not depend on the slots.
struct RefillSlots {
    int seg, count, off;
    __device__ __forceinline__ bool due(int k) const { return count > 0 && k < seg * count && k % seg == off; }
};
// `key` staggers the refill step per workgroup (per team in the multi-team kernels); results do not
// depend on the schedule
__device__ __forceinline__ RefillSlots refill_slots(int K, int count, uint32_t key = blockIdx.x) {
    RefillSlots r{1, 0, 0};
    if (count > 0) {
        r.count = min(count, K);
        r.seg = K / r.count;
        r.off = (int)(((key * 0x9E3779B1u) >> 16) % (uint32_t)r.seg);
    }
    return r;
}

template <int P>
__global__ __launch_bounds__(64) void k_rollout(KArena A, KTables Tb, KStep S, int K, int per_step, int refill) {
    __shared__ BlockLDS L;
    const RefillSlots rs = refill_slots(K, S.autoreset ? refill : 0);
    const int lane = lane_id();
    uint32_t *const deal_mtx = reinterpret_cast<uint32_t *>(&L.rows[64 * kScratchStride]);  // LaneMT continuation
    const int t0 = blockIdx.x * 64;
    const int t = t0 + lane;
    const bool valid = t < A.n;
    const int rows = min(64, A.n - t0);
    load_tables_lds(L, Tb);

    Tab<P> T;
    int action = 0;
    Deal pool = empty_deal();
    if (valid) {
        load_tab(T, A, t);
        action = S.actions[t];
        if (S.autoreset) pool = load_pool(A, t);
    } else {
        fresh_state(T, 0u, empty_deal());
    }
    StepPre pre = step_prefetch(T, action, valid, A, t, Tb);
    bool pool_dirty = false;
    const uint64_t ply0 = S.ply + (S.ply_base ? *S.ply_base : 0ull);
    const bool want_final = S.autoreset && S.final_obs != nullptr;
    // A wave may have 63 memory instructions in flight; a step's ~90 stores would stall it until
    // its own first stores drained.  So the obs block leaves in two parts: the first with the
    // step's other outputs, the rest after the NEXT step's rules (from the same LDS rows, before
    // anything overwrites them), and the wave computes while each part drains.
    int32_t *obs_tail = nullptr;  // second part of the previous step's obs block, not yet issued
    uint64_t cur_mask = 0ull;     // legal_moves of the current state, once a step has computed it
#ifdef SPL_STAMPS
    int rst_lo[kRStamps] = {0}, rst_hi[kRStamps] = {0};
#endif
    for (int k = 0; k < K; ++k) {
        const size_t blk = per_step ? (size_t)k * (size_t)A.n : 0;
        wave_lds_sync();  // previous step's LDS reads done (rows, mask, frows)
        RSTAMP(0, k);
        // token-return continuation (LaneMT) in frows: rows still hold the last step's obs tail
        StepOut o = step_rules(T, action, pre, valid, L, Tb, reinterpret_cast<uint32_t *>(L.frows), k > 0, cur_mask);
        RSTAMP(1, k);
        if (obs_tail) store_obs_range(L.rows, obs_tail, kObsSplit, kObsBlockWords);
        obs_tail = nullptr;
        if (rs.due(k)) {  // fused pool refill (wave-uniform)
            wave_lds_sync();  // the tail's LDS reads are done: the rows serve as deal scratch
            if (valid && pend_of(T.sw[SW_MISC]) > 0)
                T.sw[SW_MISC] = refill_table<P>(A, t, T.sw[SW_MISC], &L.rows[lane * kScratchStride], deal_mtx, pool,
                                                pool_dirty);
        }
        RSTAMP(2, k);
        const int8_t wnr = (int8_t)get_winner(T.sw);
        const uint64_t fin = __ballot(valid && o.term && want_final);
        if (__any(valid && o.term && want_final)) encode_row(T, L.frows, L);  // rows of other lanes are not stored
        const int fin_moves = get_moves(T.sw);
        if (valid && o.term) {  // per termination, as k_step (same float rounding)
            if (S.ep_return) unsafeAtomicAdd(&S.ep_return[t], final_reward_p0(T));
            if (S.ep_count) atomicAdd(&S.ep_count[t], 1u);
        }
        if (valid && o.term && S.autoreset)
            autoreset_table(T, A, t, pool, &L.rows[lane * kScratchStride], deal_mtx, o, pool_dirty);
        wave_lds_sync();
        if (!abl(ABL_ENCODE)) encode_row(T, L.rows, L);
        L.mask[lane] = o.mask;
        wave_lds_sync();
        RSTAMP(3, k);
        // the policy's next action and its prefetches go out before this step's stores
        action = policy_action(S.policy, o.mask, T, L, S.policy_seed, (uint64_t)(S.table0 + t), ply0 + (uint64_t)k);
        cur_mask = o.mask;
        if (k + 1 < K) pre = step_prefetch(T, action, valid, A, t, Tb);
        int32_t *obs = S.obs + blk * kObsDim;
        const bool patch = valid && get_moves(T.sw) > 255;
        const bool fpatch = valid && o.term && want_final && fin_moves > 255;
        const bool split = rows == 64 && !__any(patch || fpatch);  // crafted states store at once
        if (abl(ABL_OBS_STORE)) {
        } else if (split) {
            store_obs_range(L.rows, obs + (size_t)t0 * kObsDim, 0, kObsSplit);
            obs_tail = obs + (size_t)t0 * kObsDim;
        } else {
            store_obs_block(L.rows, rows, obs + (size_t)t0 * kObsDim);
        }
        store_mask_block(L.mask, L.mbits, rows, S.mask + blk * 45 + (size_t)t0 * 45);
        int32_t *fobs = want_final ? S.final_obs + blk * kObsDim : nullptr;
        if (want_final) store_final_rows(L.frows, fin, fobs, t0);
        if (!split && __any(patch || fpatch)) {  // move_count > 255: crafted states only (see k_step)
            __builtin_amdgcn_s_waitcnt(0);
            if (patch) obs[(size_t)t * kObsDim + 295] = get_moves(T.sw);
            if (fpatch) fobs[(size_t)t * kObsDim + 295] = fin_moves;
        }
        if (valid) {
            S.reward[blk + t] = o.reward;
            S.terminated[blk + t] = o.term ? 1 : 0;
            S.flags[blk + t] = (uint8_t)o.flags;
            if (S.winner) S.winner[blk + t] = wnr;
        }
        RSTAMP(4, k);
    }
    if (obs_tail) store_obs_range(L.rows, obs_tail, kObsSplit, kObsBlockWords);
#ifdef SPL_STAMPS
    if (g_rstamps) {
        RSTAMP(5, 0);  // kernel end for this wave (lane 0)
        if (lane < K && lane < 16)
            for (int i = 0; i < kRStamps; ++i)
                g_rstamps[((size_t)blockIdx.x * 16 + lane) * kRStamps + i] =
                    ((uint64_t)(uint32_t)rst_hi[i] << 32) | (uint32_t)rst_lo[i];
    }
#endif
    if (valid) {
        if (S.next_actions) S.next_actions[t] = action;
        store_tab(T, A, t, cur_mask, K > 0 ? Tb.mtag : 0u);  // cur_mask: the last step's mask of this state
        if (pool_dirty) store_pool(A, t, pool);
    }
}

// ---- two-wave pipelined rollout -----------------------------------------------------------
// k_rollout as a two-stage pipeline per 64 tables: workgroup = 2 waves, lane l of both = table
// t0 + l.  The RULES wave runs the steps (SplendorEnv.step, autoreset, policy, small outputs,
// fused refill) and hands each step's table state to the OUTPUT wave through LDS; the output
// wave encodes the observation rows (and the terminal rows) and issues the step's block stores
// while the rules wave already computes the next step.  With one wave per table block, a step
// was the rules' dependency chains PLUS the store issue stalls of one instruction stream
// (k_rollout: 12.4 us of the 15 us step with the observation stores compiled out); split over
// two waves on two SIMDs, the step costs the longer of the two stages.
//
// Hand-off per step k (buffers k & 1, so the rules wave refills buffer b only after the output
// wave has passed the next barrier, i.e. finished with it): the state words after the step
// (post-autoreset), the info mask, and the terminal (pre-autoreset) states of the first kTerm
// terminal lanes; the rules wave writes any further terminal rows itself (store_row_direct).
// One s_barrier per step; LDS ordering by lgkmcnt(0) only — a workgroup fence would add
// vmcnt(0) and make each wave wait for its own global stores.
//
// LDS per workgroup must stay <= 40 KB so that four workgroups (a 65 536-table grid) are resident
// per CU.  At 3-4 players the larger state and terminal hand-off would overflow that, so the deal
// scratch shrinks to the 100 bytes a deal uses (stride 25 dwords: odd, conflict-free byte lanes),
// 3 players list at most 8 terminal states per step, and at 4 players the scratch lives inside the
// rules wave's own state slot st[k & 1]: a deal (fused refill or inline autoreset deal) runs
// before that slot is written for step k, and the output wave finished reading it (step k - 2)
// before the hand-off barrier of step k - 1.
// partner hand-off (rollout store kernels): another wave of the team (the dealer, or the rules wave of
// the two-wave kernel) polls the pair's flag words so the output wave never waits on a global load
// behind its own row stores (one in-order vmcnt)
struct PtShared {
    uint32_t pepoch;  // output wave -> poller: this launch's counter
    uint32_t seq[2];  // output wave -> poller: tasks posted (pseq), partner tasks seen (cseq)
    uint64_t in[3];   // poller -> output wave: partner progress; pseq << 32 | my next slot's flag;
                      // cseq << 32 | the partner's next slot's flag
    uint64_t qcons[2];  // quad kernel: in[2] by the parity of the rules step that polled it (the output
                        // wave's step k reads the rules wave's step k - 1, published before the barrier
                        // the output wave has passed: guide row 3's barrier between poll and loads)
};

template <int P>
struct __align__(16) WsLDS : Consts {
    static constexpr int kW = SW_COUNT + 4 * P;  // state words per table
    PtShared pt;
    static constexpr int kTerm = P == 3 ? 7 : (P == 4 ? 15 : 16);  // terminal states listed per step (3p: 7, room for PtShared)
    static constexpr int kScrStride = P == 2 ? kScratchStride : 100;
    static constexpr bool kScrInSlot = P == 4;
    static_assert(!kScrInSlot || kW * 64 * 4 >= 64 * kScrStride, "scratch must fit the state slot");
    uint32_t st[2][kW][64];
    uint32_t tst[2][kTerm][kW];
    uint32_t small[2][64];  // the step's reward / terminated / flags / winner / episode event (pack_small)
    uint64_t mask[2][64];
    uint64_t fin[2];
    uint32_t mbits[96];
    uint8_t rows[64 * kObsDim];
    uint8_t scr[kScrInSlot ? 16 : 64 * kScrStride];  // the rules wave's deal scratch (P < 4)
    uint32_t mtx[kScrInSlot ? 624 : 0];               // deal continuation (LaneMT) at P = 4 (none below)
    __device__ __forceinline__ uint8_t *scratch(int b, int lane) {
        return kScrInSlot ? reinterpret_cast<uint8_t *>(&st[b][0][0]) + lane * kScrStride : &scr[lane * kScrStride];
    }
    // LDS for a deal's LaneMT continuation: this step's free state slot, unless it holds the scratch
    __device__ __forceinline__ uint32_t *deal_mtx(int b) { return kScrInSlot ? mtx : &st[b][0][0]; }
};
static_assert(sizeof(WsLDS<2>) <= 40960 && sizeof(WsLDS<3>) <= 40960 && sizeof(WsLDS<4>) <= 40960,
              "the two-wave rollout needs four workgroups per CU");

template <int P>
__device__ __forceinline__ uint32_t tab_word(const Tab<P> &T, int w) {
    return w < SW_COUNT ? T.sw[w] : T.pw[(w - SW_COUNT) >> 2][(w - SW_COUNT) & 3];
}
template <int P>
__device__ __forceinline__ void set_tab_word(Tab<P> &T, int w, uint32_t v) {
    if (w < SW_COUNT) T.sw[w] = v;
    else T.pw[(w - SW_COUNT) >> 2][(w - SW_COUNT) & 3] = v;
}

// The rules wave's per-step small outputs, packed for the hand-off: the OUTPUT wave issues every
// global write of a step.  A store the rules wave issued would sit in its vmcnt queue ahead of
// the next step's deck / token-table gathers (gfx9 counts loads and stores in one in-order
// counter), so each step's first use of a gathered value would wait for a write acknowledgement
// from behind the whole chip's observation stream: 12.8 -> 19.6 us per step once that stream
// goes to HBM instead of the Infinity Cache (rollout store, 65 536 tables).
// bits 0-7 flags, 8 terminated, 9 valid, 10-12 winner + 1, 13-15 reward code, 16-17 code of
// player 0's final reward (envs/splendor_env.py:92-115), 18 episode ended (ep_return / ep_count).
__device__ __forceinline__ uint32_t reward_code(float r) {
    return r == 0.0f ? 0u : (r == -0.01f ? 1u : (r == -0.1f ? 2u : (r == 1.0f ? 3u : 4u)));
}
__device__ __forceinline__ float reward_of_code(uint32_t c) {
    return c == 0u ? 0.0f : (c == 1u ? -0.01f : (c == 2u ? -0.1f : (c == 3u ? 1.0f : -1.0f)));
}
// player 0's final reward is one of 0, -1, -0.1, 1 (final_reward_p0)
__device__ __forceinline__ uint32_t ep_code(float r) { return r == 0.0f ? 0u : (r == -1.0f ? 1u : (r == -0.1f ? 2u : 3u)); }
__device__ __forceinline__ float ep_of_code(uint32_t c) {
    return c == 0u ? 0.0f : (c == 1u ? -1.0f : (c == 2u ? -0.1f : 1.0f));
}
__device__ __forceinline__ uint32_t pack_small(bool valid, const StepOut &o, int winner, bool ep, float ep_add) {
    return (o.flags & 0xFFu) | (o.term ? 1u << 8 : 0u) | (valid ? 1u << 9 : 0u) | ((uint32_t)(winner + 1) & 7u) << 10 |
           reward_code(o.reward) << 13 | ep_code(ep_add) << 16 | (ep ? 1u << 18 : 0u);
}

__device__ __forceinline__ void ws_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes have landed
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// SplendorEnv.step for every table with the rules / output split of the two-wave rollout, for ONE step:
// 128-thread workgroups of 64 tables.  The RULES wave loads, steps and autoresets its tables and
// hands the new state words (and the pre-reset words of tables that just ended) to the OUTPUT
// wave through LDS; the output wave encodes and stores the observation rows (terminal rows first)
// while the rules wave evaluates the legal mask of the new state (engine legal_moves,
// envs/splendor_env.py:81) and stores the masks, small outputs, next action and state.  The
// output wave also stages the constant tables while the rules wave's state loads
// are in flight.  (Terminal rows written per lane by the rules wave instead: 27.5 -> 29.0 us.)  Same outputs, bit for bit, as k_step (the GPU parity suite runs through it).
// The TAIL wave (round 6; k_step_wst_<P>p): a third wave per 64 tables takes the legal mask of the new
// state (engine legal_moves, envs/splendor_env.py:81), the mask block, the fused policy's next action
// and the legal-mask cache entry off the rules wave's tail; hand-off 2 (rules -> output: row halves
// staged) becomes an LDS counter, so the tail wave never waits on the other two after hand-off 1.
// Without it (k_step_ws_<P>p, round 5's two waves) the rules wave evaluates the mask after hand-off 2.
// Same outputs either way.  Measured alternating on one box (profiles/r06/stepab_r06g_h.txt, graph
// events per step): 16 384 tables 17.4 -> 14.7 us with the tail wave; 65 536 tables 22.4 -> 22.9 us
// (four workgroups per CU: 12 waves share the SIMDs and the LDS) — so spl_step picks it by grid size
// (spl_ctx_set_step_tail: auto = at most ctx->step_tail_blocks workgroups).  Its rows leave as sc0 nt sc1
// stores (SPL_STEP_TAIL_NT): 14.8 -> 12.8 us at 16 384 tables.

template <int P>
struct __align__(16) StepWsLDS : Consts {
    static constexpr int kW = SW_COUNT + 4 * P;  // state words per table
    uint32_t st[kW][64];   // state after the step (and autoreset)
    uint32_t fst[kW][64];  // pre-reset state of the tables that ended (final_observation)
    uint64_t mask[64];
    uint64_t omask[64];    // rules -> tail wave: each lane's step mask (kMaskDeferred: legal_moves to evaluate)
    uint32_t halves;       // rules -> output wave: row halves staged (hand-off 2 with the tail wave)
    uint32_t mbits[96];
    // observation staging (rows of 297 bytes, or 300 for obs_u8); before hand-off 1 the rules wave's
    // deal scratch + LaneMT
    alignas(16) uint8_t rows[64 * kObsU8];
};
static_assert(sizeof(StepWsLDS<4>) <= 40960, "k_step_ws_* needs four workgroups per CU");

// Bounded LDS waits (the dealer rollout's and the three-wave step's): a wait that runs out faults the
// launch — the serial goes to the context's host-mapped fault word — instead of spinning forever.
constexpr uint32_t kSpinLimit = 1u << 22;
__device__ uint32_t g_spin_limit = kSpinLimit;
__device__ __forceinline__ void signal_fault(const KStep &S) {
    if (S.fault && lane_id() == 0)  // a vector store (system scope: write-through to the host-mapped word)
        __hip_atomic_store(S.fault, S.fault_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// hand-off 2 of the three-wave step (rules -> output wave) as an LDS counter: a bounded wait (a lost
// hand-off faults the launch loudly, as the dealer rollout's waits do, instead of spinning)
__device__ __forceinline__ void step_publish(uint32_t *p) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's row halves have landed in LDS
    if (lane_id() == 0) __hip_atomic_store(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool step_wait(const uint32_t *p) {
    const uint32_t limit = g_spin_limit;
    for (uint32_t spins = 0;; ++spins) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // later LDS reads stay below the poll
        if (v) return true;
        if (spins >= limit) {
            SPL_CHECK(false, BC_SPIN);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// kShape: 0 two waves (the rules wave takes the new state's mask), 1 three waves (the TAIL wave takes
// it), 2 two waves with the OUTPUT wave taking it in the middle of its row-block stores (k_step_wso)
template <int P, int kShape>
__device__ __forceinline__ void step_ws(StepWsLDS<P> &L, KArena A, KTables Tb, KStep S) {
    constexpr bool kStepTail = kShape == 1, kOMask = kShape == 2, kRulesMask = kShape == 0;
    constexpr int kW = StepWsLDS<P>::kW;
    const int lane = lane_id();
    const int role = (int)(threadIdx.x >> 6);  // 0 rules, 1 output, 2 tail (kStepTail)
    const bool rules_wave = role == 0;
    const int t0 = wg_block() * 64;
    const int t = t0 + lane;
    const bool valid = t < A.n;
    const int rows = min(64, A.n - t0);
    const bool want_final = S.autoreset && S.final_obs != nullptr;
    const bool compact = S.obs_u8 != nullptr && S.obs == nullptr;  // obs_u8 rows instead of int32 obs rows
    STAMP(0);
    if (kStepTail && rules_wave && lane == 0) L.halves = 0u;  // read only after hand-off 1
    if (rules_wave) {
        __builtin_amdgcn_s_setprio(SPL_WS_PRIO);  // as in the rollout: 27.9 -> 27.3 us
        Tab<P> T;
        int action = 0;
        Deal pool = empty_deal();
        // the constant tables by LDS-DMA first: they land while the state loads are in flight, and the
        // vmcnt(0) below (which the state needs anyway) covers them — no staging wave, no hand-off 0
        // (a barrier that the stamps put at 2.8 us, ~0.7 us after the state had landed)
        dma_tables_lds(L, Tb);
        LegalCache lc{0u, 0u};
        if (valid) {
            load_tab(T, A, t);
            lc = load_legal(A, t);  // legal_moves of this state, stored by the kernel that stored the state
            action = gated_action(S, t);
            if (S.autoreset) pool = load_pool(A, t);
        } else {
            fresh_state(T, 0u, empty_deal());
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): state, action, pool and the tables' DMA have landed
        const StepPre pre = step_prefetch(T, action, valid, A, t, Tb);
        STAMP(1);
        uint32_t *const mtx = reinterpret_cast<uint32_t *>(&L.rows[64 * kScratchStride]);
        // the pre-step check (envs/splendor_env.py:55-66: any legal move? is the action legal?) from the
        // cached mask where it is this context's; tables whose cache is unknown (after an upload, or under
        // another card table) evaluate legal_moves as before
        StepOut o = step_rules(T, action, pre, valid, L, Tb, mtx, valid && lc.known(Tb.mtag), lc.mask(), true);
        // autoreset 2: a table terminal on entry is re-dealt without a move (dual-step opponent phase)
        const bool entry_reset = valid && S.autoreset == 2 && (o.flags & SPL_F_AFTER_TERMINAL);
        if (entry_reset) o.flags = 0u;
        const bool ended = valid && (o.term || entry_reset);
        const int8_t wnr = (int8_t)get_winner(T.sw);
        STAMP(2);
        const bool fin_me = ended && want_final;
        if (fin_me) {
#pragma unroll
            for (int w = 0; w < kW; ++w) L.fst[w][lane] = tab_word(T, w);
        }
        // terminal rows: stored by this wave after hand-off 2, column-parallel (store_row_columns)
        const uint64_t fin_all = __ballot(fin_me);
        const float ep_add = (valid && o.term) ? final_reward_p0(T) : 0.0f;
        bool pool_dirty = false;
        if (ended && S.autoreset)
            autoreset_table(T, A, t, pool, &L.rows[lane * kScratchStride], mtx, o, pool_dirty);
#pragma unroll
        for (int w = 0; w < kW; ++w) L.st[w][lane] = tab_word(T, w);
        if (!kRulesMask) L.omask[lane] = o.mask;  // the tail / output wave evaluates the deferred lanes' masks
        STAMP(3);
        ws_sync();  // hand-off 1: state words (deal scratch in `rows` free again)
        // this wave encodes the first half of every row while the output wave encodes the second
        // (encode 2.7 -> ~1.4 us before the obs stores start)
        if (abl(ABL_ENCODE)) {
        } else if (compact) encode_row_u8<0>(T, L.rows, L);
        else encode_row_half<0>(T, L.rows, L);
        if (kStepTail) step_publish(&L.halves);  // hand-off 2 (the tail wave takes no part)
        else ws_sync();                          // hand-off 2: first row halves staged
        STAMP(4);
        if (fin_all && !abl(ABL_FINAL)) {  // info["final_observation"] rows: each by the whole wave, from its listed words
            // (four rows at a time, their LDS lookups overlapped, measured slower: 23.4 vs 23.2 us per step
            // at 65 536 tables, 19.5 vs 18.1 at 16 384; profiles/r05/fin_group_ab_r05zz4.txt)
            const ColRecipes crc = col_recipes();
            for (uint64_t m = fin_all; m; m &= m - 1) {
                const int r = __ffsll((unsigned long long)m) - 1;
                store_row_columns<P>(&L.fst[0][r], 64, L, crc, S.final_obs + (size_t)(t0 + r) * kObsDim);
            }
        }
        STAMP(7);
        STAMPV(9, __popcll(fin_all) | (__popcll(__ballot((o.mask & kMaskDeferred) != 0)) << 8));
        if (kRulesMask) {
            if (o.mask & kMaskDeferred) o.mask = abl(ABL_LEGAL_POST) ? (uint64_t)action : legal_of(T, L);
            STAMP(5);
            // masks and small outputs leave from this wave while the output wave streams the rows
            L.mask[lane] = o.mask;
            wave_lds_sync();
            if (!abl(ABL_MASK_STORE)) store_mask_block<false, SPL_STEP_MASK_CPOL>(L.mask, L.mbits, rows, S.mask + (size_t)t0 * 45);
        }
        STAMP(8);
        store_step_info(S, A.n, t, valid, o.flags);
        if (valid) {
            S.reward[t] = o.reward;
            S.terminated[t] = o.term ? 1 : 0;
            S.flags[t] = (uint8_t)o.flags;
            if (S.winner) S.winner[t] = wnr;
            if (o.term) {
                if (S.ep_return) unsafeAtomicAdd(&S.ep_return[t], ep_add);
                if (S.ep_count) atomicAdd(&S.ep_count[t], 1u);
            }
            if (!kRulesMask) {
                store_words(T, A, t);  // the legal-mask cache entry is the tail / output wave's
            } else {
                if (S.next_actions) {
                    const uint64_t ply = S.ply + (S.ply_base ? *S.ply_base : 0ull);
                    S.next_actions[t] = policy_action(S.policy, o.mask, T, L, S.policy_seed, (uint64_t)(S.table0 + t), ply);
                }
                store_tab(T, A, t, o.mask, Tb.mtag);  // o.mask: legal_moves of the stored (stepped, autoreset) state
            }
            if (pool_dirty) store_pool(A, t, pool);
        }
        STAMP(6);
    } else if (role == 1) {
        STAMP(1);
        STAMP(2);
        ws_sync();  // hand-off 1 (the rules wave's table DMA landed before it)
        STAMP(3);
        Tab<P> T;
#pragma unroll
        for (int w = 0; w < kW; ++w) set_tab_word(T, w, L.st[w][lane]);
        if (abl(ABL_ENCODE)) {
        } else if (compact) encode_row_u8<1>(T, L.rows, L);
        else encode_row_half<1>(T, L.rows, L);
        if (kStepTail) {
            if (!step_wait(&L.halves)) signal_fault(S);  // hand-off 2 lost: the launch says so (rows stale)
        } else {
            ws_sync();  // hand-off 2
        }
        STAMP(4);
        STAMP(5);
        uint64_t m = 0ull;  // kOMask: the new state's legal mask, evaluated between the row stores
        auto mask_now = [&]() {
            m = L.omask[lane];
            if (m & kMaskDeferred) m = abl(ABL_LEGAL_POST) ? 0ull : legal_of(T, L);
        };
        if (compact) {
            store_obs_u8_block(L.rows, rows, S.obs_u8 + (size_t)t0 * kObsU8);
            if (kOMask) mask_now();
        } else {
            if (abl(ABL_OBS_STORE)) {
                if (kOMask) mask_now();
            } else if (kOMask) {
                store_obs_block_mid<SPL_STEP_OBS_NT>(L.rows, rows, S.obs + (size_t)t0 * kObsDim, mask_now);
            } else if (!kStepTail && SPL_STEP_BOTH_NT && S.obs_u8) {  // A/B: with the compact copy (the dual step's
                // opponent step, whose int32 rows go back to the caller and are not read on the device) as NT rows
                store_obs_block<64, true>(L.rows, rows, S.obs + (size_t)t0 * kObsDim);
            } else if (!kStepTail && SPL_STEP_WS_SPLIT != 0) {  // A/B: half the block NT (SPL_ROLL_CPOL), half plain
                store_obs_block_mid<SPL_STEP_WS_SPLIT == 1, NoOp, SPL_STEP_WS_SPLIT == 2>(L.rows, rows, S.obs + (size_t)t0 * kObsDim, NoOp());
            } else {
                constexpr int kCp = kStepTail ? (SPL_STEP_TAIL_CPOL != -3 ? SPL_STEP_TAIL_CPOL : stream_cpol(SPL_STEP_TAIL_NT))
                                              : (SPL_STEP_OBS_NT ? SPL_ROLL_CPOL : SPL_STEP_WS_CPOL);
                store_obs_block<64, false, kCp>(L.rows, rows, S.obs + (size_t)t0 * kObsDim);
            }
            if (S.obs_u8)  // both outputs: the compact copy of the same rows (a fused actor's input)
                store_u8_from_rows(L.rows, rows, S.obs_u8 + (size_t)t0 * kObsU8, valid ? (uint32_t)get_moves(T.sw) >> 8 : 0u);
        }
        STAMP(6);
        if (kOMask) {  // the mask block, the fused policy's action and the legal-mask cache entry
            L.mask[lane] = m;
            wave_lds_sync();
            if (!abl(ABL_MASK_STORE)) store_mask_block<false, SPL_STEP_MASK_CPOL>(L.mask, L.mbits, rows, S.mask + (size_t)t0 * 45);
            if (valid) {
                if (S.next_actions) {
                    const uint64_t ply = S.ply + (S.ply_base ? *S.ply_base : 0ull);
                    S.next_actions[t] = policy_action(S.policy, m, T, L, S.policy_seed, (uint64_t)(S.table0 + t), ply);
                }
                store_legal(A, t, m, Tb.mtag);  // m: legal_moves of the state the rules wave stores
            }
        }
        if (!compact && __any(valid && get_moves(T.sw) > 255)) {  // patch after this wave's block stores of the same dwords
            __builtin_amdgcn_s_waitcnt(0);
            if (valid && get_moves(T.sw) > 255) S.obs[(size_t)t * kObsDim + 295] = get_moves(T.sw);
        }
        STAMP(7);
    } else if (kStepTail) {
        // the TAIL wave: from hand-off 1 on, the new state's legal mask (engine legal_moves, deferred
        // lanes only: reset tables carry the fresh deal's, terminal ones none), the mask block, the fused
        // policy's next action and the legal-mask cache entry
        ws_sync();  // hand-off 1
        Tab<P> T;
#pragma unroll
        for (int w = 0; w < kW; ++w) set_tab_word(T, w, L.st[w][lane]);
        uint64_t m = L.omask[lane];
        if (m & kMaskDeferred) m = abl(ABL_LEGAL_POST) ? 0ull : legal_of(T, L);
        L.mask[lane] = m;
        wave_lds_sync();
        if (!abl(ABL_MASK_STORE)) store_mask_block<false, SPL_STEP_MASK_CPOL>(L.mask, L.mbits, rows, S.mask + (size_t)t0 * 45);
        if (valid) {
            if (S.next_actions) {
                const uint64_t ply = S.ply + (S.ply_base ? *S.ply_base : 0ull);
                S.next_actions[t] = policy_action(S.policy, m, T, L, S.policy_seed, (uint64_t)(S.table0 + t), ply);
            }
            store_legal(A, t, m, Tb.mtag);  // m: legal_moves of the state the rules wave stores
        }
    }
}

// one kernel name per player count and shape (see RolloutKernel)
template <int P, int kShape>
struct StepWsKernel;
#define SPL_STEP_WS_KERNEL(NAME, P_, SHAPE_)                                                    \
    __global__ __launch_bounds__(SHAPE_ == 1 ? 192 : 128) void NAME(KArena A, KTables Tb, KStep S) { \
        __shared__ StepWsLDS<P_> L;                                                              \
        step_ws<P_, SHAPE_>(L, A, Tb, S);                                                        \
    }                                                                                            \
    template <>                                                                                  \
    struct StepWsKernel<P_, SHAPE_> {                                                            \
        static constexpr void (*fn)(KArena, KTables, KStep) = NAME;                              \
    };
SPL_STEP_WS_KERNEL(k_step_ws_2p, 2, 0)
SPL_STEP_WS_KERNEL(k_step_ws_3p, 3, 0)
SPL_STEP_WS_KERNEL(k_step_ws_4p, 4, 0)
SPL_STEP_WS_KERNEL(k_step_wst_2p, 2, 1)
SPL_STEP_WS_KERNEL(k_step_wst_3p, 3, 1)
SPL_STEP_WS_KERNEL(k_step_wst_4p, 4, 1)
SPL_STEP_WS_KERNEL(k_step_wso_2p, 2, 2)
SPL_STEP_WS_KERNEL(k_step_wso_3p, 3, 2)
SPL_STEP_WS_KERNEL(k_step_wso_4p, 4, 2)
#undef SPL_STEP_WS_KERNEL

// Rollout-store delegation (rollout_ws<P, 64, true>, spl_ctx_set_rollout_delegation).  The
// XCCs of an MI355X do not drain stores equally fast: with the rollout store's own write pattern
// and nothing else running (tools/microbench_store_xcc.hip), workgroups on odd XCCs (odd blockIdx)
// finish ~20 % after those on even XCCs, whichever addresses they write; in the kernel the slowest
// XCC sets the launch time.  So workgroups pair up (2q on an even XCC, 2q+1 on the odd one next to
// it), and on every `every`-th step the odd one stages its 64 tables' state words after the step
// (4.3 KB at 2 players, against the 76 KB block it would store; it skips that step's encode) and
// its even partner, done with its own steps first, encodes and stores the rows into the rollout
// store (staging the encoded rows as bytes, 19 KB a block, measured ~1 % slower and moved 0.06 GB
// more per launch).  Cross-XCC hand-off (the guide's valid form):
// payload stored sc1 (write-through), the ready flag stored sc1 only after the payload has
// completed, the consumer polls sc1 and loads the payload sc1 behind an agent-scope acquire.
// Nothing waits unboundedly: a consumer that does not see a task within its time limit gives up,
// and the producer stores every task whose `taken` flag it does not see itself (a row stored
// twice is the same row).  Launch epochs live in the arena (each side counts its own launches),
// so flags from earlier launches, graph replays included, never match.
struct Deleg {
    bool on, producer;
    int pair, every;
    uint32_t epoch;
};
__device__ __forceinline__ bool deleg_step(int k, int K, int every) {
    return every > 0 && k % every == every / 2 - 1 && k + 2 < K && k / every < kDelegTasks;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, 0x7FFFFFF0, 0x00020000);
}
constexpr int kSc1 = 16;  // buffer-op aux bit: sc1 (write-through store / L1-bypassing load)
// a flag poll: relaxed agent-scope atomic load = global_load_dword sc1 (MI355X_MICROARCH.md: L1
// bypassed, L2-served), the poll form of the guide's hand-off rows
__device__ __forceinline__ uint32_t flag_load(const uint32_t *f) {
    return __hip_atomic_load(const_cast<uint32_t *>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void flag_store(uint32_t *f, uint32_t v) {  // lane 0 only
    if (lane_id() == 0) __builtin_amdgcn_raw_buffer_store_b32(v, rsrc_of(f), 0, 0, kSc1);
}
// a delegated step: the wave's 64 tables' state words after the step -> a delegation slot
// ([word][lane], 256 contiguous bytes per word), sc1 (write-through) dword stores: relaxed agent-scope
// atomic stores = global_store_dword sc1; slots are 128-byte aligned (kDelegPayload = 50 lines), so each
// 128-byte line is written whole by one store instruction of this wave (the guide's row 3 store cell)
template <int P>
__device__ __forceinline__ void stage_state(const Tab<P> &T, uint8_t *slot) {
    uint32_t *const base = reinterpret_cast<uint32_t *>(slot);
#pragma unroll
    for (int w = 0; w < num_words(P); ++w)
        __hip_atomic_store(base + w * 64 + lane_id(), tab_word(T, w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
static_assert(kDelegPayload % 128 == 0, "partner / delegation slots stay 128-byte aligned");
// a delegation slot -> the staged tables' state (sc1 loads)
template <int P>
__device__ __forceinline__ void unstage_state(const uint8_t *slot, Tab<P> &T) {
    const __amdgpu_buffer_rsrc_t r = rsrc_of(slot);
    uint32_t v[num_words(P)];
#pragma unroll
    for (int w = 0; w < num_words(P); ++w)
        v[w] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, (w * 64 + lane_id()) * 4, 0, kSc1);
#pragma unroll
    for (int w = 0; w < num_words(P); ++w) set_tab_word(T, w, v[w]);
}

// ---- the dealer wave (rollout for grids of at most two workgroups per CU) ----------------------
// A pool refill deal is a ~90 us serial integer chain per wave (MT19937 init, stream, Fisher-Yates).
// Fused into the rules wave it stalls that wave's steps for its whole length: at 4 players a
// 128-step launch needs ~8 of them per table, ~45 % of the rules wave's time on a half-full chip
// (C4's 32 768 tables per GPU).  When the grid leaves room for a third wave per workgroup (two
// workgroups of 64 tables per CU: 6 waves on 4 SIMDs), a DEALER wave deals instead, beside the
// rules and output waves:
//   * the rules wave owns the ring bookkeeping (status word: live record, pend = consumed records
//     not yet requested) and posts a batch -- one record per table, the earliest consumed one, the
//     next in the engine-seed stream -- whenever the dealer is idle and some table has pend > 0;
//   * the dealer owns the engine-seed streams (PCG64 records) and the deal scratch; it deals the
//     batch into the slot records (global) and the board / noble words into LDS, drains its stores
//     (s_waitcnt vmcnt(0): the waves of a workgroup share one L1, so that is the workgroup-scope
//     release), then counts the batch done;
//   * a table that ends while its next record is in flight waits for the batch; one whose pool is
//     spent (all three records consumed) posts a batch of its own and waits (the old inline deal).
// Deals are taken from each stream in episode order either way, so results do not depend on when
// a batch runs.  The three waves hand off through LDS counters (no s_barrier: the dealer cannot
// join a per-step barrier while it runs a 90 us deal).
struct DealerLDS {
    static constexpr int kStride = 100;  // deal scratch bytes per lane (25 dwords: odd, conflict-free)
    uint8_t scr[64 * kStride];
    uint32_t mtx[624];        // the dealer's LaneMT continuation (one lane at a time)
    uint32_t rdeal[5][64];    // board / noble words of the last batch's deals ([word][lane])
    uint8_t rq[64];           // slot record to deal per table, 0xFF = none
    uint32_t dreq, ddone;     // batches posted (rules wave) / dealt (dealer)
    uint32_t rdone, odone;    // steps handed off by the rules wave / finished by the output wave
    uint32_t stop;            // rules wave: no more batches
    uint32_t rnd[2][64];      // the uniform policy's words of step k in slot k & 1, drawn by the output wave at step k - 2
    uint32_t abort;           // a wait ran out (lds_wait_ge): every later wait returns at once
};
template <int P>
struct __align__(16) WsDealLDS : WsLDS<P> {
    DealerLDS dl;
};
static_assert(sizeof(WsDealLDS<2>) <= 81920 && sizeof(WsDealLDS<3>) <= 81920 && sizeof(WsDealLDS<4>) <= 81920,
              "the dealer rollout needs two workgroups per CU");

__device__ __forceinline__ uint32_t lds_poll(const uint32_t *p) {
    const uint32_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // later LDS reads stay below the poll
    return __builtin_amdgcn_readfirstlane(v);
}
// lane 0 publishes `v` after this wave's earlier LDS writes have landed
__device__ __forceinline__ void lds_publish(uint32_t *p, uint32_t v) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    if (lane_id() == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// Every wait is bounded (~2^22 polls, a fraction of a second; a legitimate wait is one deal, ~0.1 ms)
// so that a lost hand-off never leaves waves spinning on the GPU.  A wait that runs out FAULTS the
// workgroup, loudly, in every build (round 4; was a silent abort in the release library):
//   * it sets the workgroup's abort word, so every later wait of the three waves returns false at once;
//   * the rules wave stops stepping and leaves its tables' state unstored, the output wave stops storing
//     and marks SPL_F_FAULT in the flags of every step it did not store, the dealer stops dealing —
//     nothing reads or writes through an index taken from an unsettled hand-off;
//   * the launch's serial goes into the context's host-mapped fault word (signal_fault), which
//     spl_ctx_faults reads without synchronising (Engine / SplendorVectorEnv / bench.py raise on it).
// spl_debug_set_spin_limit lowers the limit so a test can force the path (BC_SPIN still marks it in
// the bounds-check build).
// true once *p >= v; false when the wait ran out or another wave of the workgroup already faulted
__device__ __forceinline__ bool lds_wait_ge(DealerLDS &D, const uint32_t *p, uint32_t v) {
    const uint32_t limit = g_spin_limit;
    for (uint32_t spins = 0; lds_poll(p) < v; ++spins) {
        if (spins >= limit || lds_poll(&D.abort)) {
            SPL_CHECK(false, BC_SPIN);
            if (lane_id() == 0) __hip_atomic_store(&D.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}
__device__ __forceinline__ Deal deal_of_lds(const DealerLDS &D, int lane) {
    return Deal{{D.rdeal[0][lane], D.rdeal[1][lane], D.rdeal[2][lane]}, D.rdeal[3][lane], D.rdeal[4][lane]};
}

// ---- partner hand-off (six-wave dealer rollout, per-step outputs; ctx partner_lead) -------------
// Under the rollout store's write stream the XCCs do not keep the same pace: the C4 share's stamps put
// the teams of one or two XCCs 7-16 % behind the rest (their observation-row stores issue slower;
// without the row stores every XCC runs the same period, profiles/r04/wsstamps4_r04k.txt), and the
// launch ends with the slowest team.  So a team that falls behind hands whole steps of observation
// rows to the same team of the workgroup on the neighbouring XCC (blockIdx b ^ 1), whose OUTPUT wave
// encodes and stores them between its own steps:
//   * each side's output wave publishes its progress (steps done) every step and reads the partner's
//     from its dealer's snapshot; when the partner is `lead` or more steps ahead and the next task
//     slot is free (by a snapshot of that slot's flag), the step's state words go to the slot (sc1 stores, ~6 KB) instead of the encode
//     and the 76 KB row block, and the slot's flag turns READY(launch, step) after a vmcnt(0) at the
//     top of the next step (the guide's drained-sc1 hand-off: sc1 payload, vmcnt(0), sc1 flag);
//   * at the top of each step the partner's output wave looks at the snapshot of the next slot's flag
//     and takes at most one READY task: an agent-scope compare-and-swap READY -> TAKEN,
//     the words loaded sc1, encoded and stored, the slot freed; after its own steps it keeps serving
//     until the partner's DONE word shows (bounded by time: a partner that never finishes keeps its
//     tasks);
//   * at the end the producer posts DONE and claims back, by the same compare-and-swap, every task
//     still READY, and stores those rows itself: each task's rows are stored once, by its flag's winner.
// (The dealer wave as the consumer took too few tasks: a deal keeps it busy ~90 us at a time.  It does
// poll the pair's flag words for its output wave between batches (pt_poll: LDS snapshots tagged with
// the sequence numbers they are for), so that the output wave issues no global load it must wait for
// behind its own row stores in the one in-order vmcnt; polled by the output wave itself, the hand-off
// made every team slower than it won.)
// Masks, small outputs and terminal rows stay with the producer; rows are encoded by the same code
// from the same words, so results do not depend on who stores them.  Launch counters (one per side,
// in the arena, zeroed with it; both sides count the same launches) tag every flag, so nothing from
// an earlier launch or graph replay matches.
struct PartnerLink {
    bool on;
    int side, lead;    // lead < 0: hand off whenever a slot is free (tests)
    uint32_t e;        // this launch's counter value
    uint32_t *fl;      // the pair's flag lines
    uint8_t *pay;      // the pair's payload slots
    int t0p;           // the partner team's first table
    __device__ __forceinline__ uint32_t *line(int l) const { return fl + l * kFlagLine; }
    __device__ __forceinline__ uint8_t *slot(int j) const { return pay + (size_t)j * kDelegPayload; }
};
constexpr uint32_t kPtReady = 1u, kPtTaken = 2u;
constexpr uint64_t kPartnerWait = 500000;  // 5 ms of s_memrealtime (100 MHz): the consumer's wait for DONE
__device__ __forceinline__ uint32_t pt_flag(uint32_t e, int k, uint32_t st) { return e << 16 | (uint32_t)k << 2 | st; }
__device__ unsigned long long g_partner_stats[2];  // tasks stored by the partner / claimed back (diagnostics)

// READY(launch, step) posted by an agent-scope atomic add (the guide's row 3: "each storing wave for
// itself", after that wave's s_waitcnt vmcnt(0)).  `seen` is the producer's snapshot of the slot's flag
// when it chose the slot: 0 or a value of an earlier launch, which nobody else writes in this launch (the
// consumer writes only flags READY in this launch), so adding target - seen leaves exactly `target`.
__device__ __forceinline__ void pt_post_ready(uint32_t *f, uint32_t target, uint32_t seen) {
    if (lane_id() == 0) (void)__hip_atomic_fetch_add(f, target - seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lane 0 moves a task flag READY -> TAKEN (agent scope: performed past the XCC's L2); wave-uniform
__device__ __forceinline__ bool pt_claim(uint32_t *f, uint32_t ready) {
    uint32_t seen = 0u;
    if (lane_id() == 0) {
        seen = ready;
        __hip_atomic_compare_exchange_strong(f, &seen, (ready & ~3u) | kPtTaken, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane(seen) == ready;
}
// one task's rows: the staged words -> rows in LDS -> the row block (whole wave, 64 full rows)
template <int P>
__device__ __forceinline__ void pt_store_task(const uint8_t *slot, uint8_t *rows_lds, const Consts &C, int32_t *dst) {
    Tab<P> T;
    unstage_state(slot, T);
    encode_row(T, rows_lds, C);
    wave_lds_sync();
    store_obs_block<64, kRollNT>(rows_lds, 64, dst);
    wave_lds_sync();  // the block's LDS reads are done before the next task's rows land
}
// consumer (the partner team's output wave): `v` = the flag of the partner's slot cseq; if it is READY,
// claim it and store the task's rows (staged through `rows`); true if the slot held a task.  Which
// form makes the staged words visible (MI355X_MICROARCH.md, "Valid forms" / the hand-off table):
//   acquire = false: the quad kernel in its steps — the flag was polled by the rules wave (global_load_dword
//     sc1) before an s_barrier this wave has passed since (row 3: agent-atomic flag, barrier between the
//     poll and every load, sc1 global stores / buffer_load_dword sc1 loads, one workgroup per CU);
//   acquire = true: everywhere else (the six-wave dealer, whose poller is not separated from this wave by
//     a barrier, and every drain after the steps) — the consumer's "always" form: one poll, the claim,
//     ONE agent acquire, then the loads (this wave's own loads need no further wait).
template <int P>
__device__ __forceinline__ bool pt_serve_v(const PartnerLink &pl, uint32_t &cseq, uint32_t v, uint8_t *rows,
                                           const Consts &C, int32_t *obs, int n, bool acquire) {
    if ((v & 3u) != kPtReady || (v >> 16) != pl.e) return false;
    const int j = (pl.side ^ 1) * kPartnerSlots + (int)(cseq % kPartnerSlots);
    ++cseq;  // tasks fill the ring in order: the next one is in the next slot, whoever stores this one
    uint32_t *f = pl.line(pt_ready_line(j));
    if (!pt_claim(f, v)) return true;
    if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int k = (int)((v >> 2) & 0x3FFFu);
    pt_store_task<P>(pl.slot(j), rows, C, obs + ((size_t)k * (size_t)n + (size_t)pl.t0p) * kObsDim);
    // the slot's words were read (the encode used them) before it is free again; no vmcnt wait: the
    // rows' stores need not have completed
    __asm__ volatile("" ::: "memory");
    flag_store(f, 0u);
    if (lane_id() == 0) atomicAdd(&g_partner_stats[0], 1ull);
    return true;
}
__device__ __forceinline__ uint32_t pt_next_flag(const PartnerLink &pl, uint32_t cseq) {
    return flag_load(pl.line(pt_ready_line((pl.side ^ 1) * kPartnerSlots + (int)(cseq % kPartnerSlots))));
}
// consumer, after its own steps: serve until the partner's DONE word shows (or kPartnerWait passes)
template <int P>
__device__ __forceinline__ void pt_drain(const PartnerLink &pl, uint32_t &cseq, uint8_t *rows, const Consts &C,
                                         int32_t *obs, int n) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (pt_serve_v<P>(pl, cseq, (uint32_t)__builtin_amdgcn_readfirstlane(pt_next_flag(pl, cseq)), rows, C, obs, n,
                          true))
            continue;
        const uint32_t dn = (uint32_t)__builtin_amdgcn_readfirstlane(flag_load(pl.line(pt_done_line(pl.side ^ 1))));
        if (dn == pl.e) {  // its READY flags were stored before DONE: what is left of them, then out
            while (pt_serve_v<P>(pl, cseq, (uint32_t)__builtin_amdgcn_readfirstlane(pt_next_flag(pl, cseq)), rows, C,
                                 obs, n, true)) {
            }
            return;
        }
        if (__builtin_amdgcn_s_memrealtime() - t_start > kPartnerWait) return;
        __builtin_amdgcn_s_sleep(8);
    }
}
// producer, at the end of its steps — and on a fault of its workgroup: the task staged
// last (if any) turns READY, DONE is posted behind every READY flag (the partner's pt_drain stops
// waiting), then every task the partner has not taken is claimed back by the same compare-and-swap
// and its rows are stored here: each handed-off step's rows are stored once, whatever happened after
template <int P>
__device__ __forceinline__ void pt_close(const PartnerLink &pl, int ppend, int ppend_k, uint32_t ppend_seen, uint32_t pseq,
                                         uint8_t *rows, const Consts &C, int32_t *obs, int n, int t0) {
    if (ppend >= 0) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the staged words have completed
        pt_post_ready(pl.line(pt_ready_line(ppend)), pt_flag(pl.e, ppend_k, kPtReady), ppend_seen);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // every READY flag has completed before DONE
    flag_store(pl.line(pt_done_line(pl.side)), pl.e);
    if (pseq == 0u) return;
    uint32_t mine = 0u;  // lane j: slot j's flag (relaxed agent load: global_load sc1)
    if (lane_id() < kPartnerSlots)
        mine = __hip_atomic_load(pl.line(pt_ready_line(pl.side * kPartnerSlots + lane_id())), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    uint64_t rm = __ballot(lane_id() < kPartnerSlots && (mine & 3u) == kPtReady && (mine >> 16) == pl.e);
    for (; rm; rm &= rm - 1) {
        const int j = __ffsll((unsigned long long)rm) - 1;
        const uint32_t vj = (uint32_t)__builtin_amdgcn_readlane((int)mine, j);
        uint32_t *f = pl.line(pt_ready_line(pl.side * kPartnerSlots + j));
        if (!pt_claim(f, vj)) continue;
        const int kk = (int)((vj >> 2) & 0x3FFFu);
        pt_store_task<P>(pl.slot(pl.side * kPartnerSlots + j), rows, C, obs + ((size_t)kk * (size_t)n + (size_t)t0) * kObsDim);
        if (lane_id() == 0) atomicAdd(&g_partner_stats[1], 1ull);
    }
}

// The dealer wave: batches until the rules wave stops and none is left.  An idle wait that runs out
// ends the dealer quietly: a batch posted after that is never dealt, so the rules wave's wait for it
// runs out and faults the launch (lds_wait_ge).  A faulted workgroup's dealer ends after its batch.
// the dealer wave's poll of the pair's words for its output wave (a snapshot; tags say which slots)
__device__ __forceinline__ void pt_publish(PtShared &X, uint32_t a, uint32_t b, uint32_t ps, uint32_t c, uint32_t cs,
                                           int qpar = -1) {
    if (lane_id() == 0) {
        __hip_atomic_store(&X.in[0], (uint64_t)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(&X.in[1], (uint64_t)ps << 32 | b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_store(qpar < 0 ? &X.in[2] : &X.qcons[qpar], (uint64_t)cs << 32 | c, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
__device__ __forceinline__ void pt_poll(PtShared &X, const PartnerLink &pl) {
    const uint32_t ps = lds_poll(&X.seq[0]), cs = lds_poll(&X.seq[1]);
    const uint32_t a = flag_load(pl.line(pt_progress_line(pl.side ^ 1)));
    const uint32_t b = flag_load(pl.line(pt_ready_line(pl.side * kPartnerSlots + (int)(ps % kPartnerSlots))));
    const uint32_t c = flag_load(pl.line(pt_ready_line((pl.side ^ 1) * kPartnerSlots + (int)(cs % kPartnerSlots))));
    pt_publish(X, (uint32_t)__builtin_amdgcn_readfirstlane(a), (uint32_t)__builtin_amdgcn_readfirstlane(b), ps,
               (uint32_t)__builtin_amdgcn_readfirstlane(c), cs);
}
__device__ __forceinline__ uint64_t lds_poll64(const uint64_t *p) {
    const uint64_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32;
}

template <int P>
__device__ __forceinline__ void dealer_loop(DealerLDS &D, const KArena &A, int t0, const PartnerLink &pl, PtShared &X) {
    const int lane = lane_id();
    const uint32_t limit = g_spin_limit;
    uint32_t done = 0;
    for (;;) {
        uint32_t req;
        for (uint32_t spins = 0;; ++spins) {
            if (lds_poll(&D.abort)) return;
            req = lds_poll(&D.dreq);
            if (req != done || lds_poll(&D.stop)) break;
            if (pl.on) pt_poll(X, pl);
            if (spins >= limit) {
                SPL_CHECK(false, BC_SPIN);
                break;
            }
            __builtin_amdgcn_s_sleep(4);
        }
        if (req == done) break;  // stopped (or idle too long), nothing pending
        const int slot = D.rq[lane];
        const int t = t0 + lane;
        if (slot != 0xFF) {
            SPL_CHECK(t < A.n && slot < kSlotRecords, BC_TABLE);
            Deal d;
            deal_next<P>(A, t, slot, &D.scr[lane * DealerLDS::kStride], d, D.mtx);
            D.rdeal[0][lane] = d.board[0];
            D.rdeal[1][lane] = d.board[1];
            D.rdeal[2][lane] = d.board[2];
            D.rdeal[3][lane] = d.nob0;
            D.rdeal[4][lane] = d.nob1;
        }
        __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0): the records and engine-seed streams are written
        lds_publish(&D.ddone, ++done);
    }
}

// the rules wave posts a batch: lanes with `want` request slot record `slot` of their table
__device__ __forceinline__ void dealer_post(DealerLDS &D, bool want, int slot, uint32_t &my_req) {
    D.rq[lane_id()] = want ? (uint8_t)slot : (uint8_t)0xFF;
    lds_publish(&D.dreq, ++my_req);
}

// The rules wave's side of the dealer after step_rules (wave-uniform call): settle a finished
// batch, make sure every table that ended has its next record dealt (waiting for the batch in
// flight, or posting one for a spent pool), run the same-step autoreset (flip_to_pool without its
// inline deal), then post a new batch when the dealer is idle.  False: a wait for the dealer faulted
// (lds_wait_ge) and T / pool were left as they were, not filled from an unsettled batch.
template <int P>
__device__ __forceinline__ bool dealer_step(DealerLDS &D, Tab<P> &T, const KArena &A, int t, bool valid, bool ends,
                                            bool autoreset, Deal &pool, bool &pool_dirty, uint32_t &my_req,
                                            uint32_t &infl, bool &pool_stale, StepOut &o) {
    constexpr int kPools = kSlotRecords - 1;
    const int lane = lane_id();
    auto settle = [&]() {  // the last batch's records are dealt; its words fill a stale `pool`
        infl = 0u;
        if (pool_stale) {
            pool = deal_of_lds(D, lane);
            pool_stale = false;
            pool_dirty = true;
        }
    };
    bool idle = lds_poll(&D.ddone) == my_req;
    if (idle) settle();
    uint32_t misc = T.sw[SW_MISC];
    int pend = pend_of(misc);
    const int nxt = (active_of(misc) + 1) % kSlotRecords;
    const bool spent = ends && pend >= kPools;  // all three pool records consumed: deal the next now
    const bool blocked = ends && !spent && (((infl >> nxt) & 1u) != 0u || pool_stale);
    if (__any(spent || blocked)) {
        if (!idle) {
            if (!lds_wait_ge(D, &D.ddone, my_req)) return false;
            settle();
            idle = true;
        }
        if (__any(spent)) {
            dealer_post(D, spent, nxt, my_req);  // nxt is the earliest consumed record when pend == 3
            if (spent) {
                pend -= 1;
                misc = (misc & ~ST_PEND) | ((uint32_t)pend << ST_PEND_SHIFT);
                pool_stale = true;
            }
            if (!lds_wait_ge(D, &D.ddone, my_req)) return false;
            settle();
        }
    }
    if (ends) {  // flip_to_pool: the next record is dealt and `pool` holds its words
        const int pend2 = pend + 1;  // the old live record is consumed
        fresh_state(T, ring_bits(nxt, pend2), pool);
        if (pend2 < kPools) {
            const int nxt2 = (nxt + 1) % kSlotRecords;
            if ((infl >> nxt2) & 1u) pool_stale = true;  // in flight: its words come with the batch
            else pool = rec_deal(slot_rec(A, t, nxt2));
        }
        pool_dirty = true;
        o.flags |= SPL_F_RESET;
        o.mask = kFreshDealMask;
        misc = T.sw[SW_MISC];
        pend = pend2;
    } else {
        T.sw[SW_MISC] = misc;
    }
    const bool want = valid && autoreset && pend > 0;
    if (idle && __any(want)) {  // refill: every table's earliest consumed record, next in its stream
        const int slot = (active_of(misc) - pend + kSlotRecords) % kSlotRecords;
        dealer_post(D, want, slot, my_req);
        if (want) {
            T.sw[SW_MISC] = (misc & ~ST_PEND) | ((uint32_t)(pend - 1) << ST_PEND_SHIFT);
            infl = 1u << slot;
            if (pend == kPools) pool_stale = true;  // the next record itself is being dealt
        }
    }
    return true;
}

// TPW = tables per workgroup: 64, or 32 for grids too small to give every SIMD a wave (e.g. the
// 32 768-table share of a 4-player 8-GPU run): twice the workgroups, lanes 32-63 idle.  The rules
// work is latency-bound at one wave per SIMD, so half-populated waves on every SIMD finish a step
// in about the time full ones take on half of them.
// kStore: per-step outputs (a [K][n][...] rollout store) or every step into the same [n][...] block;
// a template argument so that the two variants are separate kernels in a profile.
// kDealer: a third wave deals the pool refills (DealerLDS above; 64 tables per workgroup).
// A wave's role in rollout_ws (0 rules, 1 output, 2 dealer) and the block of TPW tables it serves;
// the default (role -1) takes both from the thread index and the workgroup (one block per workgroup).
struct WaveRole {
    int role, block;
};
// kTeams: 64-table teams per workgroup (the six-wave dealer 2, the quad kernel 4; one workgroup per CU)
// Barrier invariant: without a dealer wave the two waves of a team hand off through
// ws_sync(), an s_barrier of the WHOLE workgroup — in the quad kernel (kTeams = 4) all eight waves pass
// each barrier together.  That is correct only because every wave makes exactly 1 + K ws_sync() calls
// (one before the roles split, one per step) and none returns early: a per-team early exit or an extra
// barrier would deadlock the workgroup or pair different steps.  Only the dealer variants leave early
// (their fault path), and they hand off through LDS counters, not barriers.  The bounds-check build
// counts each wave's barriers and flags BC_BARRIER when a wave ends with another count.
template <int P, int TPW, bool kStore, bool kDealer = false, class LdsT = WsLDS<P>, int kTeams = 1>
__device__ __forceinline__ void rollout_ws(LdsT &L, KArena A, KTables Tb, KStep S, int K, int refill,
                                           int deleg_every, WaveRole wr = WaveRole{-1, -1}) {
    static_assert(TPW == 64 || TPW == 32, "64 or 32 tables per workgroup");
    static_assert(!kDealer || TPW == 64, "the dealer variant runs 64 tables per workgroup");
    constexpr bool per_step = kStore;
    constexpr int kW = WsLDS<P>::kW;
    const int lane = lane_id();
    const int role = wr.role >= 0 ? wr.role : (int)(threadIdx.x >> 6);
    const bool rules_wave = role == 0;
    // delegation pairs neighbouring workgroups (blockIdx b and b + 1 on adjacent XCCs): identity map
    const bool deleg_shape = TPW == 64 && kStore && !kDealer && kTeams == 1 && deleg_every >= 4;
    const int t0 = (wr.block >= 0 ? wr.block : (deleg_shape ? (int)blockIdx.x : wg_block())) * TPW;
    const int t = t0 + lane;
    const bool valid = lane < TPW && t < A.n;
    const int rows = min(TPW, A.n - t0);
    const bool want_final = S.autoreset && S.final_obs != nullptr;
    load_tables_lds(L, Tb);
    if constexpr (kDealer) {  // the hand-off counters start at zero (LDS is not initialised)
        if (rules_wave && lane == 0) {
            L.dl.dreq = L.dl.ddone = L.dl.rdone = L.dl.odone = L.dl.stop = L.dl.abort = 0u;
        }
    }
    // partner hand-off (per-step outputs, 64 tables per team; see PartnerLink): the multi-team kernels
    // only — one workgroup per CU, the guide's first measured row (the six-wave dealer and, round 5, the
    // quad kernel; not the two-wave kernel at four workgroups per CU), which pass the lead in steps as
    // deleg_every (0 = off, -1 = forced).  Team j of workgroups b and b ^ 1, both full, K < 2^14 (the
    // step fits a flag).
    PartnerLink pl{false, 0, 0, 0u, nullptr, nullptr, 0};
    if constexpr (kStore && kTeams > 1) {
        const int lead = wr.block >= 0 ? deleg_every : 0;
        if (lead != 0 && K < (1 << 14)) {
            const uint32_t b = blockIdx.x, pb = b ^ 1u;
            const int team = wr.block - kTeams * wg_block();
            const int t0p = (kTeams * wg_block_of(pb) + team) * 64;
            const int pair = (int)(b >> 1) * kTeams + team;
            if (pb < gridDim.x && t0 + 64 <= A.n && t0p + 64 <= A.n && pair < A.n / 128) {
                pl.on = true;
                pl.lead = lead;
                pl.side = (int)(b & 1u);
                pl.t0p = t0p;
                pl.fl = A.dflags + (size_t)pair * kDelegFlagWords;
                pl.pay = A.deleg + (size_t)pair * kDelegTasks * kDelegPayload;
            }
        }
        if (pl.on && role == 1) {  // this side's launch counter: the output wave counts, the poller reads it
            uint32_t *el = pl.line(pt_epoch_line(pl.side));
            uint32_t e = ((uint32_t)__builtin_amdgcn_readfirstlane(flag_load(el)) + 1u) & 0xFFFFu;
            e = e == 0u ? 1u : e;
            flag_store(el, e);
            pl.e = e;
            if (lane == 0) {
                L.pt.pepoch = e;
                L.pt.seq[0] = L.pt.seq[1] = 0u;
                L.pt.in[0] = 0ull;
                L.pt.in[1] = L.pt.in[2] = ~0ull;  // no snapshot yet (tags match no sequence number)
                L.pt.qcons[0] = L.pt.qcons[1] = ~0ull;
            }
        }
    }
    ws_sync();
    if (pl.on && role != 1) pl.e = (uint32_t)__builtin_amdgcn_readfirstlane(L.pt.pepoch);

    // stamp slot of this team (diagnostic builds): its 64-table block for the six-wave dealer, else the workgroup
    const int sid = wr.block >= 0 ? wr.block : (int)blockIdx.x;
    (void)sid;
    WSHWID(sid, rules_wave ? 0 : 1);
    // the rules wave is the critical path: it wins issue arbitration against the CU's output
    // waves (rollout store 1134 -> 1103 us per launch on one box; 1 and 3 measure the same)
    if (rules_wave) __builtin_amdgcn_s_setprio(SPL_WS_PRIO);
#ifdef SPL_STAMPS
    const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    if constexpr (kDealer) {
        if (role >= 2) {
            dealer_loop<P>(L.dl, A, t0, pl, L.pt);
            return;
        }
    }
    if (rules_wave) {
        const RefillSlots rs = refill_slots(K, (S.autoreset && !kDealer) ? refill : 0,
                                            wr.block >= 0 ? (uint32_t)wr.block : blockIdx.x);
        // dealer bookkeeping (per lane): slots whose deal is in flight (valid while a batch is
        // outstanding) and whether `pool` still lacks the next record's words
        uint32_t my_req = 0, infl = 0;
        bool pool_stale = false;
        bool faulted = false;  // a dealer hand-off ran out (wave-uniform): stop, store nothing more
        Tab<P> T;
        int action = 0;
        Deal pool = empty_deal();
        if (valid) {
            load_tab(T, A, t);
            action = S.actions[t];
            if (S.autoreset) pool = load_pool(A, t);
        } else {
            fresh_state(T, 0u, empty_deal());
        }
        StepPre pre = step_prefetch(T, action, valid, A, t, Tb);
        bool pool_dirty = false;
        const uint64_t ply0 = S.ply + (S.ply_base ? *S.ply_base : 0ull);
        uint64_t cur_mask = 0ull;
        uint32_t pv[3] = {0u, 0u, 0u}, pps = 0u, pcs = 0u;  // quad kernel's partner poller (loaded a step ahead)
        int nsync = 0;  // ws_sync() calls in the steps (the barrier invariant above)
        const uint64_t below = (1ull << lane) - 1ull;
#ifdef SPL_STAMPS
        int rst_lo[kWsStamps] = {0}, rst_hi[kWsStamps] = {0};
#endif
        for (int k = 0; k < K; ++k) {
            const int b = k & 1;
            const size_t blk = per_step ? (size_t)k * (size_t)A.n : 0;
            WSSTAMP(0, k);
            if constexpr (kDealer) {
                if (k >= 2 && !lds_wait_ge(L.dl, &L.dl.odone, (uint32_t)(k - 1))) {  // slot b: step k-2 is stored
                    faulted = true;
                    break;
                }
            }
            // token-return continuation (LaneMT) in this step's free state slot
#ifdef SPL_STAMPS
            auto sub = [&](int i) { WSSTAMP(i, k); };
            StepOut o = step_rules(T, action, pre, valid, L, Tb, &L.st[b][0][0], k > 0, cur_mask, false, sub);
#else
            StepOut o = step_rules(T, action, pre, valid, L, Tb, &L.st[b][0][0], k > 0, cur_mask);
#endif
            WSSTAMP(1, k);
            if (rs.due(k) && valid && pend_of(T.sw[SW_MISC]) > 0)  // fused pool refill
                T.sw[SW_MISC] = refill_table<P>(A, t, T.sw[SW_MISC], L.scratch(b, lane), L.deal_mtx(b), pool, pool_dirty);
            const int8_t wnr = (int8_t)get_winner(T.sw);
            const bool fin_me = valid && o.term && want_final;
            const uint64_t fin_all = __ballot(fin_me);
            const int idx = __popcll(fin_all & below);
            if (fin_me) {  // the terminal state, before the autoreset replaces it
                if (idx < WsLDS<P>::kTerm) {
#pragma unroll
                    for (int w = 0; w < kW; ++w) L.tst[b][idx][w] = tab_word(T, w);
                } else {
                    store_row_direct(T, L, S.final_obs + (blk + (size_t)t) * kObsDim);
                }
            }
            const float ep_add = (valid && o.term) ? final_reward_p0(T) : 0.0f;  // per termination, as k_step
            if constexpr (kDealer) {
                if (!dealer_step<P>(L.dl, T, A, t, valid, valid && o.term && S.autoreset, S.autoreset != 0, pool,
                                    pool_dirty, my_req, infl, pool_stale, o)) {
                    faulted = true;
                    break;
                }
            } else {
                if (valid && o.term && S.autoreset)
                    autoreset_table(T, A, t, pool, L.scratch(b, lane), L.deal_mtx(b), o, pool_dirty);
            }
            WSSTAMP(7, k);
            L.small[b][lane] = pack_small(valid, o, wnr, valid && o.term, ep_add);  // stored by the output wave
            if (kDealer && S.policy == SPL_POLICY_UNIFORM && k >= 2) {
                // the Philox word was drawn by the output wave at step k - 2 (it published odone >= k - 1
                // after writing it, which this step waited for): only the scaling stays on this chain
                if constexpr (kDealer) action = sample_uniform_word(o.mask, L.dl.rnd[b][lane]);
            } else {
                action = policy_action(S.policy, o.mask, T, L, S.policy_seed, (uint64_t)(S.table0 + t), ply0 + (uint64_t)k);
            }
            cur_mask = o.mask;
            if (k + 1 < K) pre = step_prefetch(T, action, valid, A, t, Tb);
#pragma unroll
            for (int w = 0; w < kW; ++w) L.st[b][w][lane] = tab_word(T, w);
            L.mask[b][lane] = o.mask;
            const uint64_t fin_listed = __ballot(fin_me && idx < WsLDS<P>::kTerm);  // outside the lane-0 branch
            if (lane == 0) L.fin[b] = fin_listed;
            WSSTAMP(2, k);
            if constexpr (kDealer) {
                lds_publish(&L.dl.rdone, (uint32_t)(k + 1));  // hand-off of step k
            } else {
                if (pl.on) {  // the quad kernel's partner poller (the rules wave issues no row stores): the
                              // words loaded last step go to the output wave's snapshots, then new loads
                    if (k > 0)  // the consumer's entry by this step's parity (PtShared::qcons)
                        pt_publish(L.pt, (uint32_t)__builtin_amdgcn_readfirstlane(pv[0]),
                                   (uint32_t)__builtin_amdgcn_readfirstlane(pv[1]), pps,
                                   (uint32_t)__builtin_amdgcn_readfirstlane(pv[2]), pcs, k & 1);
                    pps = lds_poll(&L.pt.seq[0]);
                    pcs = lds_poll(&L.pt.seq[1]);
                    pv[0] = flag_load(pl.line(pt_progress_line(pl.side ^ 1)));
                    pv[1] = flag_load(pl.line(pt_ready_line(pl.side * kPartnerSlots + (int)(pps % kPartnerSlots))));
                    pv[2] = flag_load(pl.line(pt_ready_line((pl.side ^ 1) * kPartnerSlots + (int)(pcs % kPartnerSlots))));
                }
                ws_sync();  // hand-off of step k
                ++nsync;
            }
            WSSTAMP(3, k);
        }
        if constexpr (kDealer) {  // no more batches; the last one lands before the state is stored
            lds_publish(&L.dl.stop, 1u);
            if (!faulted && !lds_wait_ge(L.dl, &L.dl.ddone, my_req)) faulted = true;
            if (pool_stale && !faulted) {
                pool = deal_of_lds(L.dl, lane);
                pool_dirty = true;
            }
            if (faulted) {  // the tables' state is not stored: the host sees the fault and resets
                signal_fault(S);
                return;
            }
        }
#ifdef SPL_STAMPS
        {
            const uint64_t clk1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
            if (g_wsclk && lane == 0) {
                g_wsclk[sid * 4 + 0] = clk0;
                g_wsclk[sid * 4 + 1] = rt0;
                g_wsclk[sid * 4 + 2] = clk1;
                g_wsclk[sid * 4 + 3] = rt1;
            }
        }
        if (g_wsstamps && lane < K)
            for (int i = 0; i < kWsStamps; ++i)
                g_wsstamps[(((size_t)sid * 2 + 0) * 64 + lane) * kWsStamps + i] =
                    ((uint64_t)(uint32_t)rst_hi[i] << 32) | (uint32_t)rst_lo[i];
#endif
        SPL_CHECK(kDealer || nsync == K, BC_BARRIER);
        (void)nsync;
        if (valid) {
            if (S.next_actions) S.next_actions[t] = action;
            store_tab(T, A, t, cur_mask, K > 0 ? Tb.mtag : 0u);  // cur_mask: the last step's mask of this state
            if (pool_dirty) store_pool(A, t, pool);
        }
    } else {
        const ColRecipes crc = col_recipes();  // this lane's bytes of a column-parallel terminal row
        const uint64_t ply0 = S.ply + (S.ply_base ? *S.ply_base : 0ull);  // the policy words drawn ahead (dealer)
        (void)ply0;
#ifdef SPL_STAMPS
        int rst_lo[kWsStamps] = {0}, rst_hi[kWsStamps] = {0};
#endif
        // delegation: both workgroups of a full pair take part (the same test on both sides)
        Deleg dl{false, false, (int)(blockIdx.x >> 1), deleg_every, 0u};
        if (deleg_shape && (int)(blockIdx.x | 1u) * 64 + 64 <= A.n) {
            dl.on = true;
            dl.producer = (blockIdx.x & 1u) != 0;
            uint32_t *ep = A.dflags + (size_t)dl.pair * kDelegFlagWords + (dl.producer ? DF_PROD_EPOCH : DF_CONS_EPOCH) * kFlagLine;
            dl.epoch = __builtin_amdgcn_readfirstlane(flag_load(ep)) + 1u;
            flag_store(ep, dl.epoch);
        }
        uint32_t *const dflags = A.dflags + (size_t)dl.pair * kDelegFlagWords;
        auto ready_flag = [&](int j) { return dflags + (DF_TASKS + 2 * j) * kFlagLine; };
        auto taken_flag = [&](int j) { return dflags + (DF_TASKS + 2 * j + 1) * kFlagLine; };
        auto slot_of = [&](int j) { return A.deleg + ((size_t)dl.pair * kDelegTasks + j) * kDelegPayload; };
        int pend = -1, pend_k = -1;  // producer: task staged at step pend_k, ready flag not yet set
        uint32_t staged = 0u;        // producer: tasks staged (not stored here)
        // partner hand-off: tasks posted (pseq) and the one staged but not yet READY (ppend), partner
        // tasks seen (cseq); the flags and the partner's progress come from the poller's LDS snapshots
        uint32_t pseq = 0u, cseq = 0u;
        int ppend = -1, ppend_k = 0;
        uint32_t ppend_seen = 0u;  // the staged task's slot flag as the producer saw it (pt_post_ready)
        int osync = 0;             // ws_sync() calls in the steps (the barrier invariant above)
        for (int k = 0; k < K; ++k) {
            if (pl.on) {
                if (ppend >= 0) {  // the task staged last step: its words have completed, then READY
                    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                    pt_post_ready(pl.line(pt_ready_line(ppend)), pt_flag(pl.e, ppend_k, kPtReady), ppend_seen);
                    ppend = -1;
                }
                // at most one of the partner's tasks per step, between this team's steps (the poller's
                // snapshot of its next slot, if it is for the task this wave expects).  The quad kernel
                // reads the snapshot its rules wave published at step k - 1, before the s_barrier of step
                // k - 1 that this wave has passed (PtShared::qcons); the six-wave dealer acquires instead.
                const uint64_t nx = kDealer ? lds_poll64(&L.pt.in[2]) : lds_poll64(&L.pt.qcons[(k + 1) & 1]);
                if ((uint32_t)(nx >> 32) == cseq &&
                    pt_serve_v<P>(pl, cseq, (uint32_t)nx, L.rows, L, S.obs, A.n, kDealer) && lane == 0)
                    __hip_atomic_store(&L.pt.seq[1], cseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if constexpr (kDealer) {
                if (!lds_wait_ge(L.dl, &L.dl.rdone, (uint32_t)(k + 1))) {  // hand-off of step k
                    // steps k.. are not stored: their flags say so (the blocks keep stale rows)
                    for (int j = per_step ? k : 0; j < K && (per_step || j == 0); ++j)
                        if (valid) S.flags[(per_step ? (size_t)j * (size_t)A.n : 0) + t] = (uint8_t)SPL_F_FAULT;
                    // steps before k that were handed to the partner: DONE, and those it has not taken are
                    // stored here (they were stepped before the fault)
                    if (pl.on) pt_close<P>(pl, ppend, ppend_k, ppend_seen, pseq, L.rows, L, S.obs, A.n, t0);
                    signal_fault(S);
                    return;
                }
            } else {
                ws_sync();  // hand-off of step k
                ++osync;
            }
            WSSTAMP(0, k);
            const int b = k & 1;
            const size_t blk = per_step ? (size_t)k * (size_t)A.n : 0;
            Tab<P> T;
#pragma unroll
            for (int w = 0; w < kW; ++w) set_tab_word(T, w, L.st[b][w][lane]);
            // terminal rows (info["final_observation"]) first: each by the whole wave, column-parallel,
            // straight from its listed state words (no staging, no LDS barrier)
            // (readfirstlane returns int: widen through uint32_t, or bit 31 sign-extends into lanes 32-63)
            uint64_t fin = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)L.fin[b]) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(L.fin[b] >> 32)) << 32);
            if (fin) {
                int32_t *fobs = S.final_obs + blk * kObsDim;
                for (int idx = 0; fin; fin &= fin - 1, ++idx) {
                    const int r = __ffsll((unsigned long long)fin) - 1;
                    if constexpr (per_step && SPL_ROLL_SMALL_NT)
                        store_row_columns_nt<P>(&L.tst[b][idx][0], 1, L, crc, fobs + (size_t)(t0 + r) * kObsDim);
                    else
                        store_row_columns<P>(&L.tst[b][idx][0], 1, L, crc, fobs + (size_t)(t0 + r) * kObsDim);
                }
            }
            const bool big_moves = __any(valid && get_moves(T.sw) > 255);
            const bool deleg_now = dl.producer && deleg_step(k, K, dl.every);
            bool handed = false;  // partner hand-off of this step's rows
            uint32_t sf = 0u;     // the snapshot of the slot's flag it would go to
            if (pl.on && !big_moves) {
                const uint32_t pp = (uint32_t)lds_poll64(&L.pt.in[0]);
                const uint64_t ms = lds_poll64(&L.pt.in[1]);
                sf = (uint32_t)ms;
                const bool ahead = pl.lead < 0 || ((pp >> 16) == pl.e && (int)(pp & 0xFFFFu) >= k + pl.lead);
                // the slot is free (or stale), by a snapshot taken for this very slot
                handed = ahead && (uint32_t)(ms >> 32) == pseq && ((sf & 3u) == 0u || (sf >> 16) != pl.e);
            }
            if (handed) {
                const int j = pl.side * kPartnerSlots + (int)(pseq % kPartnerSlots);
                stage_state(T, pl.slot(j));
                ppend = j;
                ppend_k = k;
                ppend_seen = (uint32_t)__builtin_amdgcn_readfirstlane(sf);
                ++pseq;
                if (lane == 0) __hip_atomic_store(&L.pt.seq[0], pseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (!deleg_now || big_moves) {  // a delegated step's rows are encoded by the partner
                encode_row(T, L.rows, L);
                wave_lds_sync();
            }
            WSSTAMP(1, k);
            int32_t *obs = S.obs + blk * kObsDim;
            if (handed) {
            } else if (deleg_now) {
                const int j = k / dl.every;
                if (big_moves) {  // a patched row: stored here, the partner skips the task
                    store_obs_block<TPW, kRollNT>(L.rows, rows, obs + (size_t)t0 * kObsDim);
                    flag_store(ready_flag(j), dl.epoch << 1 | 1u);
                } else {
                    stage_state(T, slot_of(j));
                    staged |= 1u << j;
                    pend = j;
                    pend_k = k;
                }
            } else if (abl(ABL_OBS_STORE)) {
            } else if (per_step) {
                store_obs_block<TPW, kRollNT>(L.rows, rows, obs + (size_t)t0 * kObsDim);
            } else {
                store_obs_block<TPW, false>(L.rows, rows, obs + (size_t)t0 * kObsDim);
            }
            WSSTAMP(2, k);
            if (abl(ABL_MASK_STORE)) {
            } else if (per_step) {
                store_mask_block<kRollNT>(L.mask[b], L.mbits, rows, S.mask + blk * 45 + (size_t)t0 * 45);
            } else {
                store_mask_block<false>(L.mask[b], L.mbits, rows, S.mask + blk * 45 + (size_t)t0 * 45);
            }
            const uint32_t sm = L.small[b][lane];
            if constexpr (per_step && SPL_ROLL_SMALL_NT && SPL_ROLL_CPOL >= 0) {  // A/B: the NT stream's policy
                const size_t o = blk + (size_t)t0;  // this wave's 64 tables of step k (wave-uniform)
                const auto rsr = __builtin_amdgcn_make_buffer_rsrc(S.reward + o, (short)0, 256, 0x00020000);
                const auto rst = __builtin_amdgcn_make_buffer_rsrc(S.terminated + o, (short)0, 64, 0x00020000);
                const auto rsf = __builtin_amdgcn_make_buffer_rsrc(S.flags + o, (short)0, 64, 0x00020000);
                if (sm & (1u << 9)) {
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, reward_of_code((sm >> 13) & 7u)), rsr,
                                                          (t - t0) * 4, 0, SPL_ROLL_CPOL);
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((sm >> 8) & 1u), rst, t - t0, 0, SPL_ROLL_CPOL);
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(sm & 0xFFu), rsf, t - t0, 0, SPL_ROLL_CPOL);
                }
                if (S.winner) {
                    const auto rsw = __builtin_amdgcn_make_buffer_rsrc(S.winner + o, (short)0, 64, 0x00020000);
                    if (sm & (1u << 9))
                        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((int)((sm >> 10) & 7u) - 1), rsw, t - t0, 0, SPL_ROLL_CPOL);
                }
            }
            if (sm & (1u << 9)) {  // valid lane: the rules wave's small outputs and episode statistics
                if constexpr (!(per_step && SPL_ROLL_SMALL_NT && SPL_ROLL_CPOL >= 0) && !(SPL_ABL & ABL_SMALL_OUT)) {
                    S.reward[blk + t] = reward_of_code((sm >> 13) & 7u);
                    S.terminated[blk + t] = (uint8_t)((sm >> 8) & 1u);
                    S.flags[blk + t] = (uint8_t)(sm & 0xFFu);
                    if (S.winner) S.winner[blk + t] = (int8_t)((int)((sm >> 10) & 7u) - 1);
                }
                if (sm & (1u << 18)) {  // same per-table order and float rounding as k_step
                    if (S.ep_return) unsafeAtomicAdd(&S.ep_return[t], ep_of_code((sm >> 16) & 3u));
                    if (S.ep_count) atomicAdd(&S.ep_count[t], 1u);
                }
            }
            if (big_moves) {
                __builtin_amdgcn_s_waitcnt(0);
                if (valid && get_moves(T.sw) > 255) obs[(size_t)t * kObsDim + 295] = get_moves(T.sw);
            }
            if (pend >= 0 && k == pend_k + 2) {
                // release (guide rule (2)): every sc1 store of the staged words has completed
                // before the ready flag is stored; by now two steps of block stores sit behind
                // them, so the wait also drains those
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
                flag_store(ready_flag(pend), dl.epoch << 1);
                pend = -1;
            }
            if constexpr (kDealer) {
                if (S.policy == SPL_POLICY_UNIFORM && k + 2 < K)  // step k + 2's policy word, slot b again
                    L.dl.rnd[b][lane] = uniform_draw(S.policy_seed, (uint64_t)(S.table0 + t), ply0 + (uint64_t)(k + 2));
                lds_publish(&L.dl.odone, (uint32_t)(k + 1));  // slot b is free again
            }
            if (pl.on)  // this side's progress, for the partner's decisions (a write-through store, no wait)
                flag_store(pl.line(pt_progress_line(pl.side)), pl.e << 16 | (uint32_t)(k + 1));
            WSSTAMP(3, k);
        }
        SPL_CHECK(kDealer || osync == K, BC_BARRIER);
        (void)osync;
        if (pl.on) {
            pt_close<P>(pl, ppend, ppend_k, ppend_seen, pseq, L.rows, L, S.obs, A.n, t0);
            pt_drain<P>(pl, cseq, L.rows, L, S.obs, A.n);  // then the partner's, until it is done
        }
#ifdef SPL_STAMPS
        if (g_wsend && lane == 0) g_wsend[sid * 2 + 0] = __builtin_amdgcn_s_memrealtime();
#endif
        if (dl.on && !dl.producer) {
            // consumer: the partner's staged blocks, each as soon as its ready flag shows
            const int64_t pt0 = (int64_t)(blockIdx.x + 1) * 64;
            const uint64_t limit = 200000;  // 2 ms of s_memrealtime (100 MHz) per task at most
            for (int k = 0; k < K; ++k) {
                if (!deleg_step(k, K, dl.every)) continue;
                const int j = k / dl.every;
                uint32_t f = 0;
                const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
                for (;;) {
                    f = __builtin_amdgcn_readfirstlane(flag_load(ready_flag(j)));
                    if ((f >> 1) == dl.epoch || __builtin_amdgcn_s_memrealtime() - t_start > limit) break;
                    __builtin_amdgcn_s_sleep(8);
                }
                if ((f >> 1) != dl.epoch) break;  // not seen in time: the producer stores the rest
                if (f & 1u) continue;              // the producer stored it
                flag_store(taken_flag(j), dl.epoch);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                Tab<P> T;
                unstage_state(slot_of(j), T);
                encode_row(T, L.rows, L);
                wave_lds_sync();
                store_obs_block<TPW, kRollNT>(L.rows, 64, S.obs + ((size_t)k * (size_t)A.n + pt0) * kObsDim);
                wave_lds_sync();  // the block's LDS reads are done before the next task's rows land
            }
        }
        if (dl.producer && staged) {
            // producer: every staged block whose taken flag is not visible is stored here
            for (int j = 0; j < kDelegTasks; ++j) {
                if (!((staged >> j) & 1u)) continue;
                const int k = j * dl.every + dl.every / 2 - 1;
                if (__builtin_amdgcn_readfirstlane(flag_load(taken_flag(j))) == dl.epoch) continue;
                Tab<P> T;
                unstage_state(slot_of(j), T);
                encode_row(T, L.rows, L);
                wave_lds_sync();
                store_obs_block<TPW, kRollNT>(L.rows, 64, S.obs + ((size_t)k * (size_t)A.n + t0) * kObsDim);
                wave_lds_sync();
            }
        }
#ifdef SPL_STAMPS
        if (g_wsend) {
            __builtin_amdgcn_s_waitcnt(0);  // this wave's stores have completed
            if (lane == 0) g_wsend[sid * 2 + 1] = __builtin_amdgcn_s_memrealtime();
        }
#endif
#ifdef SPL_STAMPS
        if (g_wsstamps && lane < K)
            for (int i = 0; i < kWsStamps; ++i)
                g_wsstamps[(((size_t)sid * 2 + 1) * 64 + lane) * kWsStamps + i] =
                    ((uint64_t)(uint32_t)rst_hi[i] << 32) | (uint32_t)rst_lo[i];
#endif
    }
}

// One kernel name per instantiation: a rocprofv3 --stats summary names kernels by the text before
// the template argument list when it truncates, so the per-step store (the headline), the in-place
// variant and the 32-tables-per-workgroup shapes must differ there to be separate rows.
template <int P, int TPW, bool kStore>
struct RolloutKernel;
#define SPL_ROLLOUT_KERNEL(NAME, P_, TPW_, ST_)                                                               \
    __global__ __launch_bounds__(128) void NAME(KArena A, KTables Tb, KStep S, int K, int refill, int deleg) { \
        __shared__ WsLDS<P_> L;                                                                                \
        rollout_ws<P_, TPW_, ST_>(L, A, Tb, S, K, refill, deleg);                                              \
    }                                                                                                          \
    template <>                                                                                                \
    struct RolloutKernel<P_, TPW_, ST_> {                                                                      \
        static constexpr void (*fn)(KArena, KTables, KStep, int, int, int) = NAME;                             \
    };
SPL_ROLLOUT_KERNEL(k_rollout_store_2p, 2, 64, true)
SPL_ROLLOUT_KERNEL(k_rollout_store_3p, 3, 64, true)
SPL_ROLLOUT_KERNEL(k_rollout_store_4p, 4, 64, true)
SPL_ROLLOUT_KERNEL(k_rollout_store_half_2p, 2, 32, true)
SPL_ROLLOUT_KERNEL(k_rollout_store_half_3p, 3, 32, true)
SPL_ROLLOUT_KERNEL(k_rollout_store_half_4p, 4, 32, true)
SPL_ROLLOUT_KERNEL(k_rollout_inplace_2p, 2, 64, false)
SPL_ROLLOUT_KERNEL(k_rollout_inplace_3p, 3, 64, false)
SPL_ROLLOUT_KERNEL(k_rollout_inplace_4p, 4, 64, false)
SPL_ROLLOUT_KERNEL(k_rollout_inplace_half_2p, 2, 32, false)
SPL_ROLLOUT_KERNEL(k_rollout_inplace_half_3p, 3, 32, false)
SPL_ROLLOUT_KERNEL(k_rollout_inplace_half_4p, 4, 32, false)
#undef SPL_ROLLOUT_KERNEL
// the dealer variants (three waves, 64 tables per workgroup; grids of at most two workgroups per CU)
template <int P, bool kStore>
struct RolloutDealerKernel;
#define SPL_DEALER_KERNEL(NAME, P_, ST_)                                                                       \
    __global__ __launch_bounds__(192) void NAME(KArena A, KTables Tb, KStep S, int K, int refill, int deleg) { \
        __shared__ WsDealLDS<P_> L;                                                                            \
        rollout_ws<P_, 64, ST_, true>(L, A, Tb, S, K, refill, deleg);                                          \
    }                                                                                                          \
    template <>                                                                                                \
    struct RolloutDealerKernel<P_, ST_> {                                                                      \
        static constexpr void (*fn)(KArena, KTables, KStep, int, int, int) = NAME;                             \
    };
SPL_DEALER_KERNEL(k_rollout_store_dealer_2p, 2, true)
SPL_DEALER_KERNEL(k_rollout_store_dealer_3p, 3, true)
SPL_DEALER_KERNEL(k_rollout_store_dealer_4p, 4, true)
SPL_DEALER_KERNEL(k_rollout_inplace_dealer_2p, 2, false)
SPL_DEALER_KERNEL(k_rollout_inplace_dealer_3p, 3, false)
SPL_DEALER_KERNEL(k_rollout_inplace_dealer_4p, 4, false)
#undef SPL_DEALER_KERNEL

// The six-wave dealer variant (round 4; k_rollout_*_dealer2_<P>p, 128 tables per workgroup, one
// workgroup per CU): two dealer-rollout teams (rules, output, dealer wave, 64 tables each) in ONE
// workgroup, so the roles can be given to waves by the SIMD each one landed on.  With two 3-wave
// workgroups per CU the dispatcher's placement is blind to the roles: a rules wave — the latency-bound
// critical path of the 4-player step — may share its SIMD with the other team's output or dealer
// wave, and the 4-player C4 share's stamps showed the workgroups dispatched second on their CU
// ending ~20 % after the first ones.  Here every wave reads its SIMD (HW_ID.SIMD_ID), the six are
// exchanged through LDS, and all waves make the same choice: the two rules waves go to the least
// occupied SIMDs (distinct ones), then the output waves, the dealers take the rest.  Each team is the
// dealer rollout of rollout_ws on its own LDS half; only which wave plays which part changes, so
// results are those of every other rollout shape.
template <int P>
struct __align__(16) WsDeal2LDS {
    WsDealLDS<P> team[2];
    uint32_t simd[6];
};
static_assert(sizeof(WsDeal2LDS<2>) <= 163840 && sizeof(WsDeal2LDS<3>) <= 163840 && sizeof(WsDeal2LDS<4>) <= 163840,
              "the six-wave dealer rollout needs one workgroup per CU");

// wave-uniform: (team * 3 + role) of wave w given the six waves' SIMDs.  Waves are taken in the
// order (occupancy of their SIMD, wave index); each role takes two of them, preferring SIMDs that do
// not hold a wave of that role yet: rules first, then output, then dealer.  Static indexing only.
__device__ __forceinline__ int dealer2_assign(const uint32_t (&simd)[6], int w) {
    int key[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        int occ = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) occ += simd[j] == simd[i] ? 1 : 0;
        key[i] = occ * 8 + i;
    }
    int rank[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        int r = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) r += key[j] < key[i] ? 1 : 0;
        rank[i] = r;
    }
    int code[6] = {-1, -1, -1, -1, -1, -1};
#pragma unroll
    for (int role = 0; role < 3; ++role) {
        uint32_t used = 0u;  // SIMDs that already hold a wave of this role
        int got = 0;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass)
#pragma unroll
            for (int r = 0; r < 6; ++r)
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const bool take = rank[i] == r && got < 2 && code[i] < 0 &&
                                      (pass == 1 || ((used >> (simd[i] & 3u)) & 1u) == 0u);
                    code[i] = take ? got * 3 + role : code[i];
                    used |= take ? 1u << (simd[i] & 3u) : 0u;
                    got += take ? 1 : 0;
                }
    }
    int mine = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) mine = i == w ? code[i] : mine;
    return mine;
}

template <int P, bool kStore>
__device__ __forceinline__ void rollout_dealer2(WsDeal2LDS<P> &L, KArena A, KTables Tb, KStep S, int K, int refill,
                                                int lead) {
    const int w = (int)(threadIdx.x >> 6);
    if (lane_id() == 0) L.simd[w] = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u;
    __syncthreads();
    uint32_t simd[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) simd[i] = __builtin_amdgcn_readfirstlane(L.simd[i]);
    const int code = __builtin_amdgcn_readfirstlane(dealer2_assign(simd, w));
    const int team = code / 3;
    rollout_ws<P, 64, kStore, true, WsDealLDS<P>, 2>(L.team[team], A, Tb, S, K, refill, lead,
                                                      WaveRole{code % 3, 2 * wg_block() + team});
}
template <int P, bool kStore>
struct RolloutDealer2Kernel;
#define SPL_DEALER2_KERNEL(NAME, P_, ST_)                                                                      \
    __global__ __launch_bounds__(384) void NAME(KArena A, KTables Tb, KStep S, int K, int refill, int deleg) { \
        __shared__ WsDeal2LDS<P_> L;                                                                           \
        rollout_dealer2<P_, ST_>(L, A, Tb, S, K, refill, deleg);                                               \
    }                                                                                                          \
    template <>                                                                                                \
    struct RolloutDealer2Kernel<P_, ST_> {                                                                     \
        static constexpr void (*fn)(KArena, KTables, KStep, int, int, int) = NAME;                             \
    };
SPL_DEALER2_KERNEL(k_rollout_store_dealer2_2p, 2, true)
SPL_DEALER2_KERNEL(k_rollout_store_dealer2_3p, 3, true)
SPL_DEALER2_KERNEL(k_rollout_store_dealer2_4p, 4, true)
SPL_DEALER2_KERNEL(k_rollout_inplace_dealer2_2p, 2, false)
SPL_DEALER2_KERNEL(k_rollout_inplace_dealer2_3p, 3, false)
SPL_DEALER2_KERNEL(k_rollout_inplace_dealer2_4p, 4, false)
#undef SPL_DEALER2_KERNEL

// The quad variant (round 5; k_rollout_*_quad_<P>p, 256 tables per workgroup, one workgroup per CU):
// four two-wave teams (rules + output wave, 64 tables each) in ONE 512-thread workgroup — the
// headline's 65 536 tables in 256 workgroups, all resident.  At one workgroup per CU the partner
// hand-off (PartnerLink; the rules wave polls the pair's flag words, as it did in round 4's two-wave
// kernel) is a hand-off of the guide's first measured row ("hipMalloc; one per CU", 4-byte sc1 stores
// and loads, one signalling lane per storing wave after its vmcnt(0)), which the two-wave kernel at
// four workgroups per CU was not.  Roles by SIMD as in the six-wave dealer: every
// wave reads its SIMD, and the rules waves go to distinct SIMDs (each SIMD: one rules + one output
// wave).  Each team is rollout_ws on its own LDS quarter; results are those of every other shape.
template <int P>
struct __align__(16) WsQuadLDS {
    WsLDS<P> team[4];
    uint32_t simd[8];
};
static_assert(sizeof(WsQuadLDS<2>) <= 163840 && sizeof(WsQuadLDS<3>) <= 163840 && sizeof(WsQuadLDS<4>) <= 163840,
              "the quad rollout needs one workgroup per CU");

// wave-uniform: (team * 2 + role) of wave w given the eight waves' SIMDs (dealer2_assign's rule for two
// roles of four waves each: waves in the order (occupancy of their SIMD, index), rules first on distinct
// SIMDs, then output).  Static indexing only.
__device__ __forceinline__ int quad_assign(const uint32_t (&simd)[8], int w) {
    int key[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int occ = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) occ += simd[j] == simd[i] ? 1 : 0;
        key[i] = occ * 8 + i;
    }
    int rank[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int r = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) r += key[j] < key[i] ? 1 : 0;
        rank[i] = r;
    }
    int code[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
#pragma unroll
    for (int role = 0; role < 2; ++role) {
        uint32_t used = 0u;
        int got = 0;
#pragma unroll
        for (int pass = 0; pass < 2; ++pass)
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const bool take = rank[i] == r && got < 4 && code[i] < 0 &&
                                      (pass == 1 || ((used >> (simd[i] & 3u)) & 1u) == 0u);
                    code[i] = take ? got * 2 + role : code[i];
                    used |= take ? 1u << (simd[i] & 3u) : 0u;
                    got += take ? 1 : 0;
                }
    }
    int mine = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) mine = i == w ? code[i] : mine;
    return mine;
}

template <int P, bool kStore>
__device__ __forceinline__ void rollout_quad(WsQuadLDS<P> &L, KArena A, KTables Tb, KStep S, int K, int refill, int lead) {
    const int w = (int)(threadIdx.x >> 6);
    if (lane_id() == 0) L.simd[w] = (__builtin_amdgcn_s_getreg((31 << 11) | 4) >> 4) & 3u;
    __syncthreads();
    uint32_t simd[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) simd[i] = __builtin_amdgcn_readfirstlane(L.simd[i]);
    const int code = __builtin_amdgcn_readfirstlane(quad_assign(simd, w));
    const int team = code >> 1;
    rollout_ws<P, 64, kStore, false, WsLDS<P>, 4>(L.team[team], A, Tb, S, K, refill, lead,
                                                  WaveRole{code & 1, 4 * wg_block() + team});
}
template <int P, bool kStore>
struct RolloutQuadKernel;
#define SPL_QUAD_KERNEL(NAME, P_, ST_)                                                                         \
    __global__ __launch_bounds__(512) void NAME(KArena A, KTables Tb, KStep S, int K, int refill, int deleg) { \
        __shared__ WsQuadLDS<P_> L;                                                                            \
        rollout_quad<P_, ST_>(L, A, Tb, S, K, refill, deleg);                                                  \
    }                                                                                                          \
    template <>                                                                                                \
    struct RolloutQuadKernel<P_, ST_> {                                                                        \
        static constexpr void (*fn)(KArena, KTables, KStep, int, int, int) = NAME;                             \
    };
SPL_QUAD_KERNEL(k_rollout_store_quad_2p, 2, true)
SPL_QUAD_KERNEL(k_rollout_store_quad_3p, 3, true)
SPL_QUAD_KERNEL(k_rollout_store_quad_4p, 4, true)
SPL_QUAD_KERNEL(k_rollout_inplace_quad_2p, 2, false)
SPL_QUAD_KERNEL(k_rollout_inplace_quad_3p, 3, false)
SPL_QUAD_KERNEL(k_rollout_inplace_quad_4p, 4, false)
#undef SPL_QUAD_KERNEL

// Explicit reset (SplendorEnv.reset / VectorEnv.reset), then observation + mask of all tables.
template <int P>
__global__ __launch_bounds__(64) void k_reset(KArena A, KTables Tb, const uint64_t *pcg_in, const uint8_t *mask_in,
                                              int32_t *obs, int8_t *mask_out, const uint32_t *eseed_in) {
    __shared__ BlockLDS L;
    const int lane = lane_id();
    const int t0 = blockIdx.x * 64;
    const int t = t0 + lane;
    const bool valid = t < A.n;
    const int rows = min(64, A.n - t0);
    load_tables_lds(L, Tb);
    Tab<P> T;
    if (valid) load_tab(T, A, t);
    else fresh_state(T, 0u, empty_deal());
    wave_lds_sync();
    const bool doit = valid && (mask_in == nullptr || mask_in[t] != 0);
    uint8_t *scr = &L.rows[lane * kScratchStride];
    uint32_t *const mtx = reinterpret_cast<uint32_t *>(&L.rows[64 * kScratchStride]);  // LaneMT continuation
    if (doit) {
        if (eseed_in) {  // engine/state.py:181-211 initial_state(P, seed) from an explicit engine seed
            Deal d0;     // no pool: a later reset() without a seed deals inline
            deal_into(eseed_in[t], P, slot_rec(A, t, 0), scr, d0, mtx);
            fresh_state(T, ring_bits(0, kSlotRecords - 1), d0);
        } else if (pcg_in) {  // reset(seed=...): restart this table's np_random stream, deal every record
            Pcg64 g;
            g.s_hi = pcg_in[4 * (size_t)t];
            g.s_lo = pcg_in[4 * (size_t)t + 1];
            g.inc_hi = pcg_in[4 * (size_t)t + 2];
            g.inc_lo = pcg_in[4 * (size_t)t + 3];
            g.has32 = 0;
            g.u32 = 0;
            // record 0 = this episode, records 1.. = the next episodes in stream order: the ring
            // starts full, so refills (one deal per table per call) only have to keep pace
            Deal d0, d;
            deal_into(g.engine_seed(), P, slot_rec(A, t, 0), scr, d0, mtx);
            for (int r = 1; r < kSlotRecords; ++r) {
                deal_into(g.engine_seed(), P, slot_rec(A, t, r), scr, d, mtx);
                if (r == 1) store_pool(A, t, d);
            }
            store_pcg(A, t, g);
            fresh_state(T, ring_bits(0, 0), d0);
        } else {       // reset() without a seed: continue the stream (pool deal)
            Deal d = pend_of(T.sw[SW_MISC]) < kSlotRecords - 1 ? load_pool(A, t) : empty_deal();
            uint32_t fl = 0;
            if (flip_to_pool<P>(T, A, t, d, scr, mtx, fl)) store_pool(A, t, d);
        }
    }
    wave_lds_sync();
    // env info mask, also the legal-mask cache of every stored state (reset or not)
    const uint64_t lm = (valid && !is_terminal(T.sw)) ? legal_of(T, L) : 0ull;
    if (obs || mask_out) {
        encode_row(T, L.rows, L);
        L.mask[lane] = lm;
        wave_lds_sync();
        if (obs) store_obs_block(L.rows, rows, obs + (size_t)t0 * kObsDim);
        if (mask_out) store_mask_block(L.mask, L.mbits, rows, mask_out + (size_t)t0 * 45);
    }
    if (valid) store_tab(T, A, t, lm, Tb.mtag);
}

// Pool refill: every table with consumed pool records gets ONE of them re-dealt per call, the
// earliest free one in ring order (the next episode's deal comes first in the engine-seed
// stream), so a call costs one deal per wave however many resets happened since the last one.
// The deal is one long serial chain per lane (CPython init_by_array + the shuffle's MT outputs):
// a wave's time is the same whether it carries 5 or 64 pending tables, so the scratch is padded
// to a quarter of the CU's LDS and the dispatcher spreads the waves one per SIMD.
constexpr int kRefillLds = 40 * 1024;
template <int P>
__global__ __launch_bounds__(64) void k_refill(KArena A) {
    __shared__ uint8_t scr_all[kRefillLds] __attribute__((aligned(16)));
    const int t = blockIdx.x * 64 + lane_id();
    if (t >= A.n) return;
    const size_t mi = (size_t)SW_MISC * A.n + t;
    const uint32_t misc = A.planes[mi];
    if (pend_of(misc) == 0) return;
    Deal pool;
    bool pool_dirty = false;
    A.planes[mi] = refill_table<P>(A, t, misc, &scr_all[lane_id() * kScratchStride],
                                   reinterpret_cast<uint32_t *>(&scr_all[64 * kScratchStride]), pool, pool_dirty);
    if (pool_dirty) store_pool(A, t, pool);  // it was the next pool: words to the pool planes
}

// Observation and/or mask of the current state (spl_encode / spl_legal).
template <int P>
__global__ __launch_bounds__(64) void k_observe(KArena A, KTables Tb, int32_t *obs, int8_t *mask_out) {
    __shared__ BlockLDS L;
    const int lane = lane_id();
    const int t0 = blockIdx.x * 64;
    const int t = t0 + lane;
    const bool valid = t < A.n;
    const int rows = min(64, A.n - t0);
    load_tables_lds(L, Tb);
    Tab<P> T;
    if (valid) load_tab(T, A, t);
    else fresh_state(T, 0u, empty_deal());
    wave_lds_sync();
    if (obs) encode_row(T, L.rows, L);
    L.mask[lane] = valid ? legal_of(T, L) : 0ull;  // engine legal_moves (no terminal check)
    wave_lds_sync();
    if (obs) {
        store_obs_block(L.rows, rows, obs + (size_t)t0 * kObsDim);
        if (__any(valid && get_moves(T.sw) > 255)) {
            __builtin_amdgcn_s_waitcnt(0);
            if (valid && get_moves(T.sw) > 255) obs[(size_t)t * kObsDim + 295] = get_moves(T.sw);
        }
    }
    if (mask_out) store_mask_block(L.mask, L.mbits, rows, mask_out + (size_t)t0 * 45);
}

// One wave per 64 tables: the wave's 64 x 45 mask bytes are read coalesced (64 consecutive bytes
// per instruction) into LDS, then each lane packs its table's row (a per-lane stride-45 byte
// walk would touch a new 64-byte segment per lane per byte).
__global__ __launch_bounds__(64) void k_sample(int n, const int8_t *mask, int32_t *actions, uint64_t seed, uint64_t ply,
                                               int64_t table0) {
    __shared__ uint32_t rows_w[64 * 45 / 4];
    int8_t *rows = reinterpret_cast<int8_t *>(rows_w);
    const int t0 = blockIdx.x * 64, lane = lane_id();
    const int nb = min(64, n - t0) * 45;
    const int8_t *src = mask + (size_t)t0 * 45;
    if ((reinterpret_cast<uintptr_t>(src) & 3u) == 0 && nb == 64 * 45) {  // 720 dwords, 12 per lane
        const uint32_t *s4 = reinterpret_cast<const uint32_t *>(src);
        uint32_t v[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) v[j] = lane + 64 * j < 720 ? s4[lane + 64 * j] : 0u;
#pragma unroll
        for (int j = 0; j < 12; ++j)
            if (lane + 64 * j < 720) rows_w[lane + 64 * j] = v[j];
    } else {
        for (int i = lane; i < nb; i += 64) rows[i] = src[i];
    }
    wave_lds_sync();
    const int t = t0 + lane;
    if (t >= n) return;
    uint64_t m = 0;
#pragma unroll
    for (int i = 0; i < 45; ++i) m |= (uint64_t)(rows[lane * 45 + i] != 0) << i;
    actions[t] = sample_uniform(m, seed, (uint64_t)(table0 + t), ply);
}

// spl_step_info: the per-table flags byte split into the gymnasium info planes (illegal_action,
// draw, turn_limit as 0/1 bytes, [3][n]) and a running count of the tables whose flags carry an
// error (out-of-range action, step after termination), one atomic per wave that has any
__global__ __launch_bounds__(256) void k_step_info(int n, const uint8_t *flags, uint8_t *info,
                                                   unsigned long long *errors) {
    const int t = blockIdx.x * 256 + (int)threadIdx.x;
    const uint32_t f = t < n ? flags[t] : 0u;
    if (t < n) {
        info[t] = (f & SPL_F_ILLEGAL) ? 1 : 0;
        info[(size_t)n + t] = (f & SPL_F_DRAW) ? 1 : 0;
        info[2 * (size_t)n + t] = (f & SPL_F_TURN_LIMIT) ? 1 : 0;
    }
    const uint64_t bad = __ballot((f & (SPL_F_OOB | SPL_F_AFTER_TERMINAL)) != 0);
    if (bad && lane_id() == __ffsll((unsigned long long)bad) - 1) atomicAdd(errors, (unsigned long long)__popcll(bad));
}

// host view <-> arena (splendor_table.h)
template <int P>
__global__ __launch_bounds__(64) void k_download(KArena A, int first, int count, spl_table_t *out) {
    const int i = blockIdx.x * 64 + lane_id();
    if (i >= count) return;
    const int t = first + i;
    Tab<P> T;
    load_tab(T, A, t);
    spl_table_t &v = out[i];
    const uint32_t *sw = T.sw;
    v.num_players = P;
    int bank[6];
    get_bank(sw, bank);
    for (int c = 0; c < 6; ++c) v.bank[c] = bank[c];
    const uint32_t owners = (sw[SW_NOB1] >> 8) & 0x7FFFu;
    const int nn = (int)bget(sw[SW_DECK], 3);
    for (int q = 0; q < SPL_MAX_PLAYERS; ++q) {
        spl_player_t &pv = v.players[q];
        for (int k = 0; k < 3; ++k) pv.reserved[k] = -1, pv.revealed[k] = 0;
        for (int k = 0; k < 5; ++k) pv.nobles[k] = -1;
        for (int c = 0; c < 6; ++c) pv.tokens[c] = 0;
        for (int c = 0; c < 5; ++c) pv.bonuses[c] = 0;
        pv.prestige = pv.n_reserved = pv.n_nobles = 0;
        if (q >= P) continue;
        const Pl p = unpack_pl(T.pw[q]);
        for (int c = 0; c < 6; ++c) pv.tokens[c] = p.tok[c];
        for (int c = 0; c < 5; ++c) pv.bonuses[c] = p.bon[c];
        pv.prestige = p.pres;
        pv.n_reserved = p.nres;
        for (int k = 0; k < p.nres; ++k) {
            pv.reserved[k] = p.res[k];
            pv.revealed[k] = (p.rev >> k) & 1;
        }
        int nk = 0;
        for (int s = 0; s < nn && s < 5; ++s) {
            if ((int)((owners >> (3 * s)) & 7u) == q + 1)
                pv.nobles[nk++] = s < 4 ? (int)bget(sw[SW_NOB0], s) : (int)bget(sw[SW_NOB1], 0);
        }
        pv.n_nobles = nk;
    }
    for (int k = 0; k < 12; ++k) {
        const int id = (int)bget(sw[SW_BOARD + k / 4], k % 4);
        v.board[k] = id == 0xFF ? -1 : id;
    }
    const uint8_t *rec = live_rec(A, t, sw[SW_MISC]);
    for (int tt = 0; tt < 3; ++tt) {
        const int len = (int)bget(sw[SW_DECK], tt);
        v.deck_len[tt] = len;
        for (int k = 0; k < 40; ++k) v.decks[tt][k] = k < len ? (int)rec[tier_base(tt) + k] : -1;
    }
    v.n_nobles = nn;
    for (int s = 0; s < 5; ++s) {
        const int idx = s < 4 ? (int)bget(sw[SW_NOB0], s) : (int)bget(sw[SW_NOB1], 0);
        const bool taken = ((owners >> (3 * s)) & 7u) != 0 || idx >= 10;
        v.nobles[s] = (s < nn && !taken) ? idx : -1;
    }
    v.to_play = get_to_play(sw);
    v.turn_count = get_turn(sw);
    v.move_count = get_moves(sw);
    v.game_over = (sw[SW_MISC] & ST_GAME_OVER) ? 1 : 0;
    v.winner = get_winner(sw);
    v.turn_limit_reached = (sw[SW_MISC] & ST_TURN_LIMIT) ? 1 : 0;
}

template <int P>
__global__ __launch_bounds__(64) void k_upload(KArena A, int first, int count, const spl_table_t *in) {
    const int i = blockIdx.x * 64 + lane_id();
    if (i >= count) return;
    const int t = first + i;
    const spl_table_t &v = in[i];
    Tab<P> T;
    uint32_t *sw = T.sw;
    const uint32_t old_misc = A.planes[(size_t)SW_MISC * A.n + t];
    int bank[6];
    for (int c = 0; c < 6; ++c) bank[c] = v.bank[c];
    sw[SW_BANK1] = ((uint32_t)v.to_play << 16) | ((uint32_t)v.turn_count << 24);
    put_bank(sw, bank);
    sw[SW_MISC] = ((uint32_t)v.move_count & 0xFFFFu) | (v.game_over ? ST_GAME_OVER : 0u) |
                  (v.turn_limit_reached ? ST_TURN_LIMIT : 0u) | (old_misc & (ST_ACTIVE | ST_PEND)) |
                  ((uint32_t)(v.winner + 1) << 24);
    for (int tt = 0; tt < 3; ++tt) {
        uint32_t w = 0;
        for (int s = 0; s < 4; ++s) w |= (uint32_t)(v.board[tt * 4 + s] < 0 ? 0xFF : v.board[tt * 4 + s]) << (8 * s);
        sw[SW_BOARD + tt] = w;
    }
    sw[SW_DECK] = (uint32_t)v.deck_len[0] | ((uint32_t)v.deck_len[1] << 8) | ((uint32_t)v.deck_len[2] << 16) |
                  ((uint32_t)v.n_nobles << 24);
    // visible slots keep their noble; taken slots get the players' nobles in order
    int slot_idx[5];
    uint32_t owners = 0;
    int next_taken = 0;
    for (int s = 0; s < 5; ++s) slot_idx[s] = (s < v.n_nobles && v.nobles[s] >= 0) ? v.nobles[s] : 0xFF;
    for (int s = 0; s < 5 && s < v.n_nobles; ++s)
        if (v.nobles[s] < 0) owners |= 7u << (3 * s);
    for (int q = 0; q < P; ++q) {
        for (int k = 0; k < v.players[q].n_nobles; ++k) {
            while (next_taken < v.n_nobles && !(v.nobles[next_taken] < 0)) ++next_taken;
            if (next_taken < v.n_nobles) {
                slot_idx[next_taken] = v.players[q].nobles[k];
                owners = (owners & ~(7u << (3 * next_taken))) | ((uint32_t)(q + 1) << (3 * next_taken));
                ++next_taken;
            }
        }
    }
    sw[SW_NOB0] = (uint32_t)slot_idx[0] | ((uint32_t)slot_idx[1] << 8) | ((uint32_t)slot_idx[2] << 16) |
                  ((uint32_t)slot_idx[3] << 24);
    sw[SW_NOB1] = (uint32_t)slot_idx[4] | (owners << 8);
    for (int q = 0; q < P; ++q) {
        Pl p;
        const spl_player_t &pv = v.players[q];
        for (int c = 0; c < 6; ++c) p.tok[c] = pv.tokens[c];
        for (int c = 0; c < 5; ++c) p.bon[c] = pv.bonuses[c];
        p.pres = pv.prestige;
        p.nres = pv.n_reserved;
        p.rev = 0;
        for (int k = 0; k < 3; ++k) {
            p.res[k] = k < pv.n_reserved ? pv.reserved[k] : 0xFF;
            p.rev |= (k < pv.n_reserved && pv.revealed[k]) ? (1 << k) : 0;
        }
        pack_pl(p, T.pw[q]);
    }
    store_tab(T, A, t, 0ull, 0u);  // a crafted state: its legal mask is unknown until a step evaluates it
    uint8_t *rec = slot_rec(A, t, active_of(old_misc));
    for (int tt = 0; tt < 3; ++tt)
        for (int k = 0; k < tier_size(tt); ++k) rec[tier_base(tt) + k] = (uint8_t)(k < v.deck_len[tt] ? v.decks[tt][k] : 0xFF);
}

}  // namespace spl

// ==========================================================================================
// host side: C-ABI
// ==========================================================================================
using namespace spl;

struct spl_ctx_s {
    int device;
    uint4 *cards;
    uint2 *nobles;
    uint4 *lut;
    int refill_period;
    int refill_fused;  // spl_rollout: refill inside the rollout launch (default) or as a k_refill launch after it
    int pipeline;      // spl_rollout: 0 one wave per 64 tables, 1 two-wave (auto tables per workgroup), 2 / 3 two-wave at 64 / 32
    int ws_resident[5];  // k_rollout_store_<P>p: workgroups resident per device (occupancy x CUs), index P
    int dealer_resident[5];  // k_rollout_store_dealer_<P>p: the same for the three-wave dealer variant
    int dealer2_resident[5]; // k_rollout_store_dealer2_<P>p: the same for the six-wave dealer variant
    int quad_resident[5];    // k_rollout_store_quad_<P>p: the same for the quad variant
    int deleg_every;     // spl_rollout per-step store: rollout-store delegation every n-th step (0 = off)
    int partner_lead;    // per-step store partner hand-off lead in steps (0 off, < 0 forced)
    uint32_t mtag;         // legal-mask cache tag of this context's card table (card_table_tag), 1..65535, or 0
    int step_tail;         // spl_step shape: -1 auto (the tail wave up to step_tail_blocks workgroups), 0 two waves, 1 three
    int64_t step_tail_blocks;
    uint64_t *fault_host;  // host-mapped, fine-grained: the serial of a launch that faulted (0 = none), spl_ctx_faults
    uint64_t *fault_dev;   // its device address (KStep::fault)
    uint64_t launches;     // launch serial (KStep::fault_tag)
    void *stage;
    size_t stage_bytes;
};

static thread_local std::string g_err;

// shared with spl_policy.hip
int spl_fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}
static inline int fail(int code, const std::string &msg) { return spl_fail(code, msg); }

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) return fail(SPL_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

static KTables ktables(const spl_ctx_t *c) { return KTables{c->cards, c->nobles, c->lut, c->mtag}; }

static int check_arena(const spl_ctx_t *ctx, const spl_arena_t *a) {
    if (!ctx) return fail(SPL_E_ARG, "null context");
    if (!a || !a->base) return fail(SPL_E_ARG, "null arena");
    if (a->players < 2 || a->players > 4) return fail(SPL_E_ARG, "players must be 2..4");
    if (a->n <= 0) return fail(SPL_E_ARG, "arena must hold at least one table");
    if (((uintptr_t)a->base & 255u) != 0) return fail(SPL_E_ARG, "arena base must be 256-byte aligned");
    if (a->bytes < spl_arena_bytes(a->n, a->players)) return fail(SPL_E_ARG, "arena too small");
    return SPL_OK;
}

static KArena karena(const spl_arena_t *a) {
    const ArenaLayout L = arena_layout(a->n, a->players);
    uint8_t *b = static_cast<uint8_t *>(a->base);
    return KArena{reinterpret_cast<uint32_t *>(b + L.planes), reinterpret_cast<uint32_t *>(b + L.pool), b + L.slots,
                  b + L.pcg, a->n, b + L.deleg, reinterpret_cast<uint32_t *>(b + L.dflags),
                  reinterpret_cast<uint32_t *>(b + L.legal)};
}

static int launch_check() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SPL_E_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return SPL_OK;
}

static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 63) / 64); }
#ifndef SPL_STEP_WAVES
#define SPL_STEP_WAVES 1
#endif
constexpr int kStepWaves = SPL_STEP_WAVES;  // k_step waves per workgroup
#ifndef SPL_STEP_WS
#define SPL_STEP_WS 1
#endif
constexpr bool kStepWs = SPL_STEP_WS != 0;  // spl_step: two-wave k_step_ws_<P>p (else k_step)

extern "C" {

int spl_abi_version(void) { return SPL_ABI_VERSION; }

#ifdef SPL_STAMPS
int spl_debug_set_stamps(void *buf) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &buf, sizeof(buf)));
    return SPL_OK;
}
int spl_debug_set_ws_clk(void *buf) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wsclk), &buf, sizeof(buf)));
    return SPL_OK;
}
int spl_debug_set_ws_end(void *buf) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wsend), &buf, sizeof(buf)));
    return SPL_OK;
}
int spl_debug_set_ws_hwid(void *buf) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wshwid), &buf, sizeof(buf)));
    return SPL_OK;
}
int spl_debug_set_ws_stamps(void *buf) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_wsstamps), &buf, sizeof(buf)));
    return SPL_OK;
}
int spl_debug_set_rollout_stamps(void *buf) {
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_rstamps), &buf, sizeof(buf)));
    return SPL_OK;
}
#endif

int spl_debug_bounds_flags(uint32_t *flags, int clear) {
#ifdef SPL_BOUNDS_CHECK
    if (!flags) return fail(SPL_E_ARG, "null flags");
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(flags, HIP_SYMBOL(g_bounds_flags), sizeof(uint32_t)));
    if (clear) {
        const uint32_t z = 0;
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_flags), &z, sizeof(z)));
    }
    return SPL_OK;
#else
    (void)flags;
    (void)clear;
    return fail(SPL_E_ARG, "not a bounds-check build (-DSPL_BOUNDS_CHECK)");
#endif
}

int spl_debug_set_stream_limit(int outputs) {
    if (outputs < 1 || outputs > MTStream::kMaxOut) return fail(SPL_E_ARG, "stream limit must be 1..454");
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_stream_limit), &outputs, sizeof(outputs)));
    return SPL_OK;
}

int spl_debug_set_spin_limit(int64_t polls) {
    if (polls > (int64_t)kSpinLimit) return fail(SPL_E_ARG, "spin limit must be <= 2^22 (negative = default)");
    const uint32_t v = polls < 0 ? kSpinLimit : (uint32_t)polls;
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_spin_limit), &v, sizeof(v)));
    return SPL_OK;
}

const char *spl_last_error(void) { return g_err.c_str(); }

int64_t spl_arena_bytes(int32_t n, int32_t players) {
    if (n <= 0 || players < 2 || players > 4) return -1;
    return arena_layout(n, players).total;
}

// The legal-mask cache tag of a card table (the 90 card and 10 noble records the kernels read; legal_moves
// depends on the state and the card costs only): one tag per DISTINCT table in this process, never
// recycled, so an arena stepped under two contexts reuses masks exactly when their tables are equal (an
// edited table gets a tag of its own; contexts of the canonical table share one).  Past 65 535 distinct
// tables a context gets tag 0: it neither trusts a cached mask nor publishes one (LegalCache::known).
static uint32_t card_table_tag(const std::vector<uint4> &crec, const std::vector<uint2> &nrec) {
    static std::mutex mu;
    static std::map<std::string, uint32_t> tags;
    std::string key(reinterpret_cast<const char *>(crec.data()), crec.size() * sizeof(uint4));
    key.append(reinterpret_cast<const char *>(nrec.data()), nrec.size() * sizeof(uint2));
    std::lock_guard<std::mutex> g(mu);
    const auto it = tags.find(key);
    if (it != tags.end()) return it->second;
    if (tags.size() >= kLegalTagMax) return 0u;
    const uint32_t tag = (uint32_t)tags.size() + 1u;
    tags.emplace(std::move(key), tag);
    return tag;
}

int spl_ctx_create(int device, const int32_t *cards, const int32_t *nobles, spl_ctx_t **out) {
    if (!cards || !nobles || !out) return fail(SPL_E_ARG, "null argument");
    *out = nullptr;
    // constant records: observation-ready card bytes (engine/encode.py:77-96) + costs
    std::vector<uint4> crec(90);
    for (int i = 0; i < 90; ++i) {
        const int32_t *c = cards + 8 * i;
        if (c[0] < 1 || c[0] > 3 || c[1] < 0 || c[1] > 4 || c[2] < 0 || c[2] > 255)
            return fail(SPL_E_ARG, "bad card table row " + std::to_string(i));
        uint8_t b[16] = {0};
        b[0] = 1;
        b[1] = (uint8_t)c[0];
        b[2] = (uint8_t)c[2];
        b[3 + c[1]] = 1;
        for (int k = 0; k < 5; ++k) {
            if (c[3 + k] < 0 || c[3 + k] > 255) return fail(SPL_E_ARG, "bad card cost");
            b[8 + k] = (uint8_t)c[3 + k];
        }
        b[13] = (uint8_t)c[1];
        memcpy(&crec[i], b, 16);
    }
    std::vector<uint2> nrec(10);
    for (int i = 0; i < 10; ++i) {
        const int32_t *n = nobles + 6 * i;
        uint8_t b[8] = {0};
        b[0] = 1;
        for (int k = 0; k < 5; ++k) {
            if (n[k] < 0 || n[k] > 255) return fail(SPL_E_ARG, "bad noble table");
            b[1 + k] = (uint8_t)n[k];
        }
        b[6] = (uint8_t)n[5];
        memcpy(&nrec[i], b, 8);
    }
    HIP_TRY(hipSetDevice(device));
    int ws_resident[5], dealer_resident[5], dealer2_resident[5], quad_resident[5];
    {
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        int occ[5] = {0, 0, 0, 0, 0};
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[2], RolloutKernel<2, 64, true>::fn, 128, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[3], RolloutKernel<3, 64, true>::fn, 128, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[4], RolloutKernel<4, 64, true>::fn, 128, 0));
        for (int q = 0; q < 5; ++q) ws_resident[q] = occ[q] * cus;
        int docc[5] = {0, 0, 0, 0, 0};
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&docc[2], RolloutDealerKernel<2, true>::fn, 192, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&docc[3], RolloutDealerKernel<3, true>::fn, 192, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&docc[4], RolloutDealerKernel<4, true>::fn, 192, 0));
        for (int q = 0; q < 5; ++q) dealer_resident[q] = docc[q] * cus;
        int d2occ[5] = {0, 0, 0, 0, 0};
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&d2occ[2], RolloutDealer2Kernel<2, true>::fn, 384, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&d2occ[3], RolloutDealer2Kernel<3, true>::fn, 384, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&d2occ[4], RolloutDealer2Kernel<4, true>::fn, 384, 0));
        for (int q = 0; q < 5; ++q) dealer2_resident[q] = d2occ[q] * cus;
        int qocc[5] = {0, 0, 0, 0, 0};
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&qocc[2], RolloutQuadKernel<2, true>::fn, 512, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&qocc[3], RolloutQuadKernel<3, true>::fn, 512, 0));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&qocc[4], RolloutQuadKernel<4, true>::fn, 512, 0));
        for (int q = 0; q < 5; ++q) quad_resident[q] = qocc[q] * cus;
    }
    spl_ctx_t *c = new spl_ctx_t();
    c->device = device;
    c->mtag = card_table_tag(crec, nrec);
    c->refill_period = 64;
    c->refill_fused = 1;
    c->deleg_every = SPL_DELEG_EVERY;
    c->partner_lead = SPL_PARTNER_LEAD;
    c->step_tail = -1;
    {
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        // up to three workgroups per CU (49 152 tables on 256 CUs): per step 20.0 against 20.45 us there,
        // 24.2 against 22.35 us at four (profiles/r06/step_shape_48k_64k_r06al.txt)
        c->step_tail_blocks = 3 * (int64_t)cus;
    }
    c->pipeline = 1;
    memcpy(c->ws_resident, ws_resident, sizeof(ws_resident));
    memcpy(c->dealer_resident, dealer_resident, sizeof(dealer_resident));
    memcpy(c->dealer2_resident, dealer2_resident, sizeof(dealer2_resident));
    memcpy(c->quad_resident, quad_resident, sizeof(quad_resident));
    if (hipMalloc(&c->cards, sizeof(uint4) * 90) != hipSuccess || hipMalloc(&c->nobles, sizeof(uint2) * 10) != hipSuccess ||
        hipMalloc(&c->lut, sizeof(uint4) * kLutEntries) != hipSuccess) {
        spl_ctx_destroy(c);
        return fail(SPL_E_HIP, "hipMalloc of constant tables failed");
    }
    // the fault word: host memory the kernels write through to (fine-grained), so the host reads a
    // launch's fault without synchronising the stream
    if (hipHostMalloc(reinterpret_cast<void **>(&c->fault_host), sizeof(uint64_t),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void **>(&c->fault_dev), c->fault_host, 0) != hipSuccess) {
        spl_ctx_destroy(c);
        return fail(SPL_E_HIP, "hipHostMalloc of the fault word failed");
    }
    *c->fault_host = 0;
    HIP_TRY(hipMemcpy(c->cards, crec.data(), sizeof(uint4) * 90, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->nobles, nrec.data(), sizeof(uint2) * 10, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_build_lut, dim3(blocks_for(kLutEntries)), dim3(64), 0, 0, c->lut);
    if (int r = launch_check()) {
        spl_ctx_destroy(c);
        return r;
    }
    HIP_TRY(hipDeviceSynchronize());
    *out = c;
    return SPL_OK;
}

int spl_ctx_destroy(spl_ctx_t *ctx) {
    if (!ctx) return SPL_OK;
    if (ctx->cards) (void)hipFree(ctx->cards);
    if (ctx->nobles) (void)hipFree(ctx->nobles);
    if (ctx->lut) (void)hipFree(ctx->lut);
    if (ctx->stage) (void)hipFree(ctx->stage);
    if (ctx->fault_host) (void)hipHostFree(ctx->fault_host);
    delete ctx;
    return SPL_OK;
}

int spl_ctx_faults(spl_ctx_t *ctx, uint64_t *launch, int clear) {
    if (!ctx || !launch) return fail(SPL_E_ARG, "null argument");
    volatile uint64_t *w = ctx->fault_host;
    *launch = *w;
    if (clear) *w = 0;
    return SPL_OK;
}

const volatile uint64_t *spl_ctx_fault_word(spl_ctx_t *ctx) {
    if (!ctx) {
        fail(SPL_E_ARG, "null ctx");
        return nullptr;
    }
    return ctx->fault_host;
}

uint64_t spl_ctx_launches(spl_ctx_t *ctx) { return ctx ? ctx->launches : 0; }

int spl_host_mapped(const void *host, int32_t *same_address) {
    if (!host || !same_address) return fail(SPL_E_ARG, "null argument");
    void *dev = nullptr;
    const hipError_t e = hipHostGetDevicePointer(&dev, const_cast<void *>(host), 0);
    *same_address = (e == hipSuccess && dev == host) ? 1 : 0;
    if (e != hipSuccess) (void)hipGetLastError();  // not page-locked by HIP: not an error of this call
    return SPL_OK;
}

int spl_ctx_set_refill_period(spl_ctx_t *ctx, int period) {
    if (!ctx || period < 0) return fail(SPL_E_ARG, "bad refill period");
    ctx->refill_period = period;
    return SPL_OK;
}

int spl_ctx_set_rollout_pipeline(spl_ctx_t *ctx, int on) {
    if (!ctx) return fail(SPL_E_ARG, "null ctx");
    if (on < 0 || on > 6) return fail(SPL_E_ARG, "rollout pipeline must be 0..6");
    ctx->pipeline = on;
    return SPL_OK;
}

int spl_ctx_set_step_tail(spl_ctx_t *ctx, int mode) {
    if (!ctx || mode < -1 || mode > 2) return fail(SPL_E_ARG, "step shape must be -1 (auto), 0, 1 or 2");
    ctx->step_tail = mode;
    return SPL_OK;
}

int spl_ctx_set_partner_lead(spl_ctx_t *ctx, int lead) {
    if (!ctx || lead < -1 || lead > 64) return fail(SPL_E_ARG, "partner lead must be in [-1, 64]");
    ctx->partner_lead = lead;
    return SPL_OK;
}

int spl_debug_partner_stats(uint64_t *stats, int clear) {
    if (!stats) return fail(SPL_E_ARG, "stats must be non-null");
    unsigned long long v[2] = {0ull, 0ull};
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(v, HIP_SYMBOL(g_partner_stats), sizeof(v)));
    stats[0] = v[0];
    stats[1] = v[1];
    if (clear) {
        const unsigned long long z[2] = {0ull, 0ull};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_partner_stats), z, sizeof(z)));
    }
    return SPL_OK;
}

int spl_ctx_set_rollout_delegation(spl_ctx_t *ctx, int every) {
    if (!ctx || every < 0 || (every > 0 && every < 4)) return fail(SPL_E_ARG, "delegation period must be 0 or >= 4");
    ctx->deleg_every = every;
    return SPL_OK;
}

int spl_ctx_set_refill_fused(spl_ctx_t *ctx, int fused) {
    if (!ctx) return fail(SPL_E_ARG, "null ctx");
    ctx->refill_fused = fused != 0;
    return SPL_OK;
}

int64_t spl_ctx_token_lut(spl_ctx_t *ctx, uint32_t *out, int64_t words) {
    const int64_t need = (int64_t)kLutEntries * 4;
    if (!ctx) return fail(SPL_E_ARG, "null context");
    if (!out) return need;
    if (words < need) return fail(SPL_E_ARG, "output too small");
    HIP_TRY(hipMemcpy(out, ctx->lut, need * 4, hipMemcpyDeviceToHost));
    return need;
}

#define DISPATCH_P(P_, call)                        \
    switch (P_) {                                   \
        case 2: { constexpr int PP = 2; call; } break; \
        case 3: { constexpr int PP = 3; call; } break; \
        case 4: { constexpr int PP = 4; call; } break; \
        default: return fail(SPL_E_ARG, "players must be 2..4"); \
    }

int spl_reset(spl_ctx_t *ctx, spl_arena_t *arena, const uint64_t *pcg, const uint8_t *reset_mask, int32_t *obs,
              int8_t *mask, void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (obs && ((uintptr_t)obs & 15u)) return fail(SPL_E_ARG, "obs must be 16-byte aligned");
    if (mask && ((uintptr_t)mask & 3u)) return fail(SPL_E_ARG, "mask must be 4-byte aligned");
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    DISPATCH_P(arena->players, hipLaunchKernelGGL(k_reset<PP>, dim3(blocks_for(arena->n)), dim3(64), 0, s, A,
                                                  ktables(ctx), pcg, reset_mask, obs, mask, (const uint32_t *)nullptr));
    if (int r = launch_check()) return r;
    arena->steps = 0;
    return SPL_OK;
}

int spl_deal(spl_ctx_t *ctx, spl_arena_t *arena, const uint32_t *engine_seeds, const uint8_t *deal_mask,
             int32_t *obs, int8_t *mask, void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (!engine_seeds) return fail(SPL_E_ARG, "engine_seeds is required");
    if (obs && ((uintptr_t)obs & 15u)) return fail(SPL_E_ARG, "obs must be 16-byte aligned");
    if (mask && ((uintptr_t)mask & 3u)) return fail(SPL_E_ARG, "mask must be 4-byte aligned");
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    DISPATCH_P(arena->players, hipLaunchKernelGGL(k_reset<PP>, dim3(blocks_for(arena->n)), dim3(64), 0, s, A,
                                                  ktables(ctx), (const uint64_t *)nullptr, deal_mask, obs, mask,
                                                  engine_seeds));
    return launch_check();
}

int spl_arena_init(spl_ctx_t *ctx, spl_arena_t *arena, void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIP_TRY(hipMemsetAsync(arena->base, 0, (size_t)spl_arena_bytes(arena->n, arena->players), s));
    // no pool deal yet: a reset() without seed deals inline, the refill kernel deals it
    const KArena A = karena(arena);
    HIP_TRY(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(A.planes + (size_t)SW_MISC * arena->n),
                              (int)((uint32_t)(kSlotRecords - 1) << ST_PEND_SHIFT),
                              (size_t)arena->n, s));
    arena->steps = 0;
    arena->epoch = 0;
    return SPL_OK;
}

int spl_refill(spl_ctx_t *ctx, spl_arena_t *arena, void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    DISPATCH_P(arena->players, hipLaunchKernelGGL(k_refill<PP>, dim3(blocks_for(arena->n)), dim3(64), 0, s, A));
    if (int r = launch_check()) return r;
    arena->epoch += 1;
    return SPL_OK;
}

static int check_step_args(const spl_step_args_t *a) {
    if (!a || !a->actions || !(a->obs || a->obs_u8) || !a->mask || !a->reward || !a->terminated || !a->flags)
        return fail(SPL_E_ARG, "actions/obs/mask/reward/terminated/flags are required");
    if ((uintptr_t)a->obs_u8 & 15u) return fail(SPL_E_ARG, "obs_u8 must be 16-byte aligned");
    if (!a->gate_terminated != !a->gate_flags) return fail(SPL_E_ARG, "gate_terminated and gate_flags go together");
    if (a->autoreset < 0 || a->autoreset > 2) return fail(SPL_E_ARG, "autoreset must be 0, 1 or 2");
    if (a->policy < SPL_POLICY_UNIFORM || a->policy > SPL_POLICY_BASIC_PRIORITY) return fail(SPL_E_ARG, "unknown policy");
    if (((uintptr_t)a->obs & 15u) || (a->final_obs && ((uintptr_t)a->final_obs & 3u)))
        return fail(SPL_E_ARG, "obs must be 16-byte aligned");
    if ((uintptr_t)a->mask & 3u) return fail(SPL_E_ARG, "mask must be 4-byte aligned");
    return SPL_OK;
}

static KStep kstep(spl_ctx_t *ctx, const spl_step_args_t *a) {
    KStep S;
    S.fault = ctx->fault_dev;
    S.fault_tag = ++ctx->launches;
    S.actions = a->actions;
    S.obs = a->obs;
    S.mask = a->mask;
    S.reward = a->reward;
    S.terminated = a->terminated;
    S.flags = a->flags;
    S.winner = a->winner;
    S.final_obs = a->final_obs;
    S.next_actions = a->next_actions;
    S.ep_return = a->ep_return;
    S.ep_count = a->ep_count;
    S.info = a->info;
    S.obs_u8 = a->obs_u8;
    S.gate_terminated = a->gate_terminated;
    S.gate_flags = a->gate_flags;
    S.errors = reinterpret_cast<unsigned long long *>(a->errors);
    S.ply_base = a->ply_base;
    S.policy_seed = a->policy_seed;
    S.ply = a->ply;
    S.table0 = a->table0;
    S.autoreset = a->autoreset;
    S.policy = a->policy;
    return S;
}

int spl_step(spl_ctx_t *ctx, spl_arena_t *arena, const spl_step_args_t *a, void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (int r = check_step_args(a)) return r;
    if (a->obs_u8 && !kStepWs) return fail(SPL_E_ARG, "obs_u8 needs the two-wave step kernel");
    const KStep S = kstep(ctx, a);
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (kStepWs) {
        const unsigned blocks = blocks_for(arena->n);
        // auto: the tail wave up to three workgroups per CU, and for compact-only outputs (obs_u8 without the
        // int32 rows: a quarter of the row stores, so the rules wave's tail is the longer one)
        const int shape = ctx->step_tail >= 0 ? ctx->step_tail
                                              : (((int64_t)blocks <= ctx->step_tail_blocks || a->obs == nullptr) ? 1 : 0);
        if (shape == 1)
            DISPATCH_P(arena->players, hipLaunchKernelGGL((StepWsKernel<PP, 1>::fn), dim3(blocks), dim3(192), 0, s, A,
                                                          ktables(ctx), S))
        else if (shape == 2)
            DISPATCH_P(arena->players, hipLaunchKernelGGL((StepWsKernel<PP, 2>::fn), dim3(blocks), dim3(128), 0, s, A,
                                                          ktables(ctx), S))
        else
            DISPATCH_P(arena->players, hipLaunchKernelGGL((StepWsKernel<PP, 0>::fn), dim3(blocks), dim3(128), 0, s, A,
                                                          ktables(ctx), S))
    } else {
        DISPATCH_P(arena->players,
                   hipLaunchKernelGGL((k_step<PP, kStepWaves>), dim3((unsigned)((arena->n + 64 * kStepWaves - 1) / (64 * kStepWaves))),
                                      dim3(64 * kStepWaves), 0, s, A, ktables(ctx), S));
    }
    if (int r = launch_check()) return r;
    arena->steps += 1;
    if (a->autoreset && ctx->refill_period > 0 && arena->steps % ctx->refill_period == 0)
        return spl_refill(ctx, arena, stream);
    return SPL_OK;
}

// The rollout kernel shape: tables per workgroup of the two-wave rollout (0 = the one-wave
// k_rollout), or kDealerShape / kDealer2Shape for the three- / six-wave dealer variants.  Auto
// (pipeline 1): the six-wave dealer variant when every 128-table workgroup is resident at once (one
// per CU, e.g. C4's 32 768 tables per GPU: 1 120-1 137 against 1 166-1 172 us per 128-step launch
// for the three-wave one, alternating on one box, profiles/r04/c4ab_r04b.txt), else the three-wave
// one when it fits, else (2 players) the quad kernel when every 256-table workgroup is resident, else
// two waves at 64 tables per workgroup.
constexpr int kDealerShape = -1, kDealer2Shape = -2, kQuadShape = -3;
static int rollout_tpw(const spl_ctx_t *ctx, int32_t n, int32_t players) {
    if (ctx->pipeline == 2) return 64;
    if (ctx->pipeline == 3) return 32;
    if (ctx->pipeline == 4) return kDealerShape;
    if (ctx->pipeline == 5) return kDealer2Shape;
    if (ctx->pipeline == 6) return kQuadShape;
    if (ctx->pipeline == 1) {  // auto: the six-wave dealer (SIMD-aware roles, -3.5 % on C4's share), else three-wave
        if ((int64_t)((n + 127) / 128) <= ctx->dealer2_resident[players]) return kDealer2Shape;
        if ((int64_t)blocks_for(n) <= ctx->dealer_resident[players]) return kDealerShape;
        // 2 players up to one quad workgroup per CU (the headline's 65 536 tables): the quad kernel with its
        // partner hand-off, 1 959-1 983 against 2 008-2 031 us per 128-step launch for the two-wave kernel,
        // alternating on one box (profiles/r05/headline_quad_ab_r05h.txt); 3-4 players keep the two-wave
        if (players == 2 && (int64_t)((n + 255) / 256) <= ctx->quad_resident[players]) return kQuadShape;
        return 64;
    }
    return 0;
}

const char *spl_rollout_kernel_name(spl_ctx_t *ctx, int32_t n, int32_t players, int32_t per_step_outputs) {
    static const char *const names[2][2][3] = {
        {{"k_rollout_inplace_2p", "k_rollout_inplace_3p", "k_rollout_inplace_4p"},
         {"k_rollout_inplace_half_2p", "k_rollout_inplace_half_3p", "k_rollout_inplace_half_4p"}},
        {{"k_rollout_store_2p", "k_rollout_store_3p", "k_rollout_store_4p"},
         {"k_rollout_store_half_2p", "k_rollout_store_half_3p", "k_rollout_store_half_4p"}}};
    static const char *const one_wave[3] = {"k_rollout<2>", "k_rollout<3>", "k_rollout<4>"};
    static const char *const dealer[2][3] = {
        {"k_rollout_inplace_dealer_2p", "k_rollout_inplace_dealer_3p", "k_rollout_inplace_dealer_4p"},
        {"k_rollout_store_dealer_2p", "k_rollout_store_dealer_3p", "k_rollout_store_dealer_4p"}};
    static const char *const dealer2[2][3] = {
        {"k_rollout_inplace_dealer2_2p", "k_rollout_inplace_dealer2_3p", "k_rollout_inplace_dealer2_4p"},
        {"k_rollout_store_dealer2_2p", "k_rollout_store_dealer2_3p", "k_rollout_store_dealer2_4p"}};
    static const char *const quad[2][3] = {
        {"k_rollout_inplace_quad_2p", "k_rollout_inplace_quad_3p", "k_rollout_inplace_quad_4p"},
        {"k_rollout_store_quad_2p", "k_rollout_store_quad_3p", "k_rollout_store_quad_4p"}};
    if (!ctx || n <= 0 || players < 2 || players > 4) {
        fail(SPL_E_ARG, "spl_rollout_kernel_name: bad arguments");
        return nullptr;
    }
    const int tpw = rollout_tpw(ctx, n, players);
    if (tpw == 0) return one_wave[players - 2];
    if (tpw == kDealerShape) return dealer[per_step_outputs ? 1 : 0][players - 2];
    if (tpw == kDealer2Shape) return dealer2[per_step_outputs ? 1 : 0][players - 2];
    if (tpw == kQuadShape) return quad[per_step_outputs ? 1 : 0][players - 2];
    return names[per_step_outputs ? 1 : 0][tpw == 32 ? 1 : 0][players - 2];
}

int spl_rollout(spl_ctx_t *ctx, spl_arena_t *arena, const spl_step_args_t *a, int32_t steps, int32_t per_step_outputs,
                void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (int r = check_step_args(a)) return r;
    if (!a->obs) return fail(SPL_E_ARG, "spl_rollout writes int32 obs (obs_u8 is spl_step only)");
    if (a->gate_terminated || a->gate_flags) return fail(SPL_E_ARG, "the gate is spl_step only");
    if (steps < 1) return fail(SPL_E_ARG, "spl_rollout: steps must be >= 1");
    if (per_step_outputs && (arena->n & 3))
        return fail(SPL_E_ARG, "spl_rollout: per-step outputs need a table count divisible by 4 (16-byte obs blocks)");
    const KStep S = kstep(ctx, a);
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t before = arena->steps;
    const bool due = a->autoreset && ctx->refill_period > 0 &&
                     (before + steps) / ctx->refill_period != before / ctx->refill_period;
    // fused: every refill the launch is due (one per refill period it crosses) runs inside it
    const int fused = (due && ctx->refill_fused)
                          ? (int)std::min<int64_t>(steps, (before + steps) / ctx->refill_period - before / ctx->refill_period)
                          : 0;
    // two-wave kernel (WsLDS<P> fits four workgroups per CU at every player count)
    // (pipeline 1 = auto, 2 = two-wave at 64 tables per workgroup, 3 = two-wave at 32)
    const int64_t resident = ctx->ws_resident[arena->players];
    const int tpw = rollout_tpw(ctx, arena->n, arena->players);
    const bool p_out = per_step_outputs != 0;
    // delegation / partner pairs must run at the same time: off when the grid exceeds what is resident
    // at once.  The two-wave kernel's `deleg`: the static delegation period (>= 4) or 0 (round 5: the
    // partner hand-off is the six-wave dealer's only)
    const int deleg = ((int64_t)blocks_for(arena->n) <= resident && ctx->deleg_every > 0) ? ctx->deleg_every : 0;
    // the six-wave dealer's partner lead, likewise 0 unless every workgroup is resident (ADVICE r04:
    // pipeline "dealer2" forced on a larger grid)
    const int lead2 = (int64_t)((arena->n + 127) / 128) <= ctx->dealer2_resident[arena->players] ? ctx->partner_lead : 0;
    const int lead4 = (int64_t)((arena->n + 255) / 256) <= ctx->quad_resident[arena->players] ? ctx->partner_lead : 0;
#define SPL_LAUNCH_WS(TPW, BLOCKS)                                                                           \
    DISPATCH_P(arena->players, if (p_out) {                                                                  \
        hipLaunchKernelGGL((RolloutKernel<PP, TPW, true>::fn), dim3(BLOCKS), dim3(128), 0, s, A, ktables(ctx), S, \
                           (int)steps, fused, deleg);                                                        \
    } else {                                                                                                 \
        hipLaunchKernelGGL((RolloutKernel<PP, TPW, false>::fn), dim3(BLOCKS), dim3(128), 0, s, A, ktables(ctx), S, \
                           (int)steps, fused, 0);                                                            \
    })
    if (tpw == kQuadShape) {
        const unsigned blocks = (unsigned)((arena->n + 255) / 256);
        DISPATCH_P(arena->players, if (p_out) {
            hipLaunchKernelGGL((RolloutQuadKernel<PP, true>::fn), dim3(blocks), dim3(512), 0, s, A, ktables(ctx), S,
                               (int)steps, fused, lead4);
        } else {
            hipLaunchKernelGGL((RolloutQuadKernel<PP, false>::fn), dim3(blocks), dim3(512), 0, s, A, ktables(ctx), S,
                               (int)steps, fused, 0);
        })
    } else if (tpw == kDealer2Shape) {
        const unsigned blocks = (unsigned)((arena->n + 127) / 128);
        DISPATCH_P(arena->players, if (p_out) {
            hipLaunchKernelGGL((RolloutDealer2Kernel<PP, true>::fn), dim3(blocks), dim3(384), 0, s, A, ktables(ctx), S,
                               (int)steps, fused, lead2);
        } else {
            hipLaunchKernelGGL((RolloutDealer2Kernel<PP, false>::fn), dim3(blocks), dim3(384), 0, s, A, ktables(ctx), S,
                               (int)steps, fused, 0);
        })
    } else if (tpw == kDealerShape) {
        DISPATCH_P(arena->players, if (p_out) {
            hipLaunchKernelGGL((RolloutDealerKernel<PP, true>::fn), dim3(blocks_for(arena->n)), dim3(192), 0, s, A,
                               ktables(ctx), S, (int)steps, fused, 0);
        } else {
            hipLaunchKernelGGL((RolloutDealerKernel<PP, false>::fn), dim3(blocks_for(arena->n)), dim3(192), 0, s, A,
                               ktables(ctx), S, (int)steps, fused, 0);
        })
    } else if (tpw == 64) {
        SPL_LAUNCH_WS(64, blocks_for(arena->n));
    } else if (tpw == 32) {
        SPL_LAUNCH_WS(32, (unsigned)((arena->n + 31) / 32));
    } else {
        DISPATCH_P(arena->players, hipLaunchKernelGGL(k_rollout<PP>, dim3(blocks_for(arena->n)), dim3(64), 0, s, A,
                                                      ktables(ctx), S, (int)steps, (int)(per_step_outputs != 0), fused));
    }
#undef SPL_LAUNCH_WS
    if (int r = launch_check()) return r;
    arena->steps += steps;
    if (fused) arena->epoch += fused;
    else if (due) return spl_refill(ctx, arena, stream);
    return SPL_OK;
}

int spl_encode(spl_ctx_t *ctx, spl_arena_t *arena, int32_t *obs, void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (!obs || ((uintptr_t)obs & 15u)) return fail(SPL_E_ARG, "obs must be non-null and 16-byte aligned");
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    DISPATCH_P(arena->players, hipLaunchKernelGGL(k_observe<PP>, dim3(blocks_for(arena->n)), dim3(64), 0, s, A,
                                                  ktables(ctx), obs, (int8_t *)nullptr));
    return launch_check();
}

int spl_legal(spl_ctx_t *ctx, spl_arena_t *arena, int8_t *mask, void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (!mask || ((uintptr_t)mask & 3u)) return fail(SPL_E_ARG, "mask must be non-null and 4-byte aligned");
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    DISPATCH_P(arena->players, hipLaunchKernelGGL(k_observe<PP>, dim3(blocks_for(arena->n)), dim3(64), 0, s, A,
                                                  ktables(ctx), (int32_t *)nullptr, mask));
    return launch_check();
}

int spl_sample_uniform(spl_ctx_t *ctx, int32_t n, const int8_t *mask, int32_t *actions, uint64_t seed, uint64_t ply,
                       int64_t table0, void *stream) {
    if (!ctx || n <= 0 || !mask || !actions) return fail(SPL_E_ARG, "bad sample arguments");
    hipLaunchKernelGGL(k_sample, dim3(blocks_for(n)), dim3(64), 0, static_cast<hipStream_t>(stream), n, mask, actions,
                       seed, ply, table0);
    return launch_check();
}

int spl_step_info(int32_t n, const uint8_t *flags, uint8_t *info, uint64_t *errors, void *stream) {
    if (n <= 0 || !flags || !info || !errors || ((uintptr_t)errors & 7u)) return fail(SPL_E_ARG, "bad step-info arguments");
    hipLaunchKernelGGL(k_step_info, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream), n,
                       flags, info, reinterpret_cast<unsigned long long *>(errors));
    return launch_check();
}

static int ensure_stage(spl_ctx_t *ctx, size_t bytes) {
    if (ctx->stage_bytes >= bytes) return SPL_OK;
    if (ctx->stage) (void)hipFree(ctx->stage);
    ctx->stage = nullptr;
    ctx->stage_bytes = 0;
    HIP_TRY(hipMalloc(&ctx->stage, bytes));
    ctx->stage_bytes = bytes;
    return SPL_OK;
}

int spl_table_download(spl_ctx_t *ctx, spl_arena_t *arena, int32_t first, int32_t count, spl_table_t *host,
                       void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (!host || first < 0 || count <= 0 || first + count > arena->n) return fail(SPL_E_ARG, "bad download range");
    if (int r = ensure_stage(ctx, sizeof(spl_table_t) * (size_t)count)) return r;
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    spl_table_t *st = static_cast<spl_table_t *>(ctx->stage);
    DISPATCH_P(arena->players, hipLaunchKernelGGL(k_download<PP>, dim3(blocks_for(count)), dim3(64), 0, s, A, first, count, st));
    if (int r = launch_check()) return r;
    HIP_TRY(hipMemcpyAsync(host, st, sizeof(spl_table_t) * (size_t)count, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return SPL_OK;
}

static int validate_view(const spl_table_t &v, int P) {
    if (v.num_players != P) return fail(SPL_E_RANGE, "num_players does not match the arena");
    for (int c = 0; c < 6; ++c)
        if (v.bank[c] < 0 || v.bank[c] > 255) return fail(SPL_E_RANGE, "bank out of range");
    int owned = 0;
    for (int q = 0; q < P; ++q) {
        const spl_player_t &p = v.players[q];
        for (int c = 0; c < 6; ++c)
            if (p.tokens[c] < 0 || p.tokens[c] > 255) return fail(SPL_E_RANGE, "tokens out of range");
        for (int c = 0; c < 5; ++c)
            if (p.bonuses[c] < 0 || p.bonuses[c] > 255) return fail(SPL_E_RANGE, "bonuses out of range");
        if (p.prestige < 0 || p.prestige > 255) return fail(SPL_E_RANGE, "prestige out of range");
        if (p.n_reserved < 0 || p.n_reserved > 3) return fail(SPL_E_RANGE, "n_reserved out of range");
        for (int k = 0; k < p.n_reserved; ++k)
            if (p.reserved[k] < 0 || p.reserved[k] >= 90) return fail(SPL_E_RANGE, "reserved card id out of range");
        if (p.n_nobles < 0 || p.n_nobles > 5) return fail(SPL_E_RANGE, "player nobles out of range");
        for (int k = 0; k < p.n_nobles; ++k)
            if (p.nobles[k] < 0 || p.nobles[k] >= 10) return fail(SPL_E_RANGE, "player noble id out of range");
        owned += p.n_nobles;
    }
    for (int k = 0; k < 12; ++k)
        if (v.board[k] < -1 || v.board[k] >= 90) return fail(SPL_E_RANGE, "board card id out of range");
    for (int t = 0; t < 3; ++t) {
        if (v.deck_len[t] < 0 || v.deck_len[t] > tier_size(t)) return fail(SPL_E_RANGE, "deck too long for its record");
        for (int k = 0; k < v.deck_len[t]; ++k)
            if (v.decks[t][k] < 0 || v.decks[t][k] >= 90) return fail(SPL_E_RANGE, "deck card id out of range");
    }
    if (v.n_nobles < 0 || v.n_nobles > 5) return fail(SPL_E_RANGE, "visible noble slots out of range");
    int taken = 0;
    for (int s = 0; s < v.n_nobles; ++s) {
        if (v.nobles[s] >= 10 || v.nobles[s] < -1) return fail(SPL_E_RANGE, "noble id out of range");
        taken += v.nobles[s] < 0;
    }
    if (owned > taken) return fail(SPL_E_RANGE, "players hold more nobles than taken slots");
    if (v.to_play < 0 || v.to_play >= P) return fail(SPL_E_RANGE, "to_play out of range");
    if (v.turn_count < 0 || v.turn_count > 255) return fail(SPL_E_RANGE, "turn_count out of range");
    if (v.move_count < 0 || v.move_count > 508) return fail(SPL_E_RANGE, "move_count out of range (<= 508)");
    if (v.winner < -1 || v.winner >= P) return fail(SPL_E_RANGE, "winner out of range");
    return SPL_OK;
}

int spl_table_upload(spl_ctx_t *ctx, spl_arena_t *arena, int32_t first, int32_t count, const spl_table_t *host,
                     void *stream) {
    if (int r = check_arena(ctx, arena)) return r;
    if (!host || first < 0 || count <= 0 || first + count > arena->n) return fail(SPL_E_ARG, "bad upload range");
    for (int i = 0; i < count; ++i)
        if (int r = validate_view(host[i], arena->players)) return r;
    if (int r = ensure_stage(ctx, sizeof(spl_table_t) * (size_t)count)) return r;
    const KArena A = karena(arena);
    hipStream_t s = static_cast<hipStream_t>(stream);
    spl_table_t *st = static_cast<spl_table_t *>(ctx->stage);
    HIP_TRY(hipMemcpyAsync(st, host, sizeof(spl_table_t) * (size_t)count, hipMemcpyHostToDevice, s));
    DISPATCH_P(arena->players, hipLaunchKernelGGL(k_upload<PP>, dim3(blocks_for(count)), dim3(64), 0, s, A, first, count, st));
    if (int r = launch_check()) return r;
    HIP_TRY(hipStreamSynchronize(s));
    return SPL_OK;
}

}  // extern "C"

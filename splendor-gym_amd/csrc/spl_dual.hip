// spl_dual.hip — glue of the batched dual step (include/splendor_dual.h): the per-table branches
// of wrappers/dual_step_native.py:90-193 as two elementwise kernels, so a dual step is four or
// five launches instead of a chain of ~30 tensor ops.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/splendor_amd.h"
#include "../../include/splendor_dual.h"
#include "spl_rng.h"

int spl_fail(int code, const std::string &msg);  // spl_engine.hip

namespace spld {

__global__ __launch_bounds__(256) void k_dual_gate(int n, const uint8_t *__restrict__ ta, const uint8_t *__restrict__ fa,
                                                   int32_t *__restrict__ opp) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const bool passed = ta[i] == 0 && (fa[i] & (SPL_F_ILLEGAL | SPL_F_OOB)) == 0;
    if (!passed) opp[i] = -1;
}

// ppo_splendor.py:137-143 opponent_supplier for table i starting an episode
__device__ __forceinline__ void draw_one(int i, uint32_t *__restrict__ episode, int32_t *__restrict__ group_of,
                                         const int32_t *__restrict__ pool_slots, int pool_len, float p_current,
                                         uint64_t seed, int64_t table0) {
    const uint32_t ep = episode[i];
    episode[i] = ep + 1;
    const uint64_t t = (uint64_t)(table0 + i);
    const uint4 r = spl::philox4x32(make_uint4((uint32_t)t, (uint32_t)(t >> 32), ep, 0x6F70706Fu),
                                    make_uint2((uint32_t)seed, (uint32_t)(seed >> 32)));
    const float u = (float)(r.x >> 8) * (1.f / 16777216.f);
    group_of[i] = (pool_len <= 0 || u < p_current) ? 0 : pool_slots[(uint32_t)(((uint64_t)r.y * (uint32_t)pool_len) >> 32)];
}

__global__ __launch_bounds__(256) void k_draw_opponents(int n, const uint8_t *__restrict__ draw,
                                                        uint32_t *__restrict__ episode, int32_t *__restrict__ group_of,
                                                        const int32_t *__restrict__ pool_slots, int pool_len,
                                                        float p_current, uint64_t seed, int64_t table0) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || (draw && draw[i] == 0)) return;
    draw_one(i, episode, group_of, pool_slots, pool_len, p_current, seed, table0);
}

struct Draw {
    uint32_t *episode;
    int32_t *group_of, *group_prev;
    const int32_t *pool_slots;
    int pool_len;
    float p_current;
    uint64_t seed;
    int64_t table0;
};

// final_rewards[player] of a finished game (envs/splendor_env.py:92-115): +-1 for the winner /
// loser; without a winner -0.1 after the turn limit, else 0 (the no-legal-move draw reports none)
__device__ __forceinline__ float final_reward(int player, int winner, uint8_t flags) {
    if (winner < 0) return (flags & SPL_F_TURN_LIMIT) ? -0.1f : 0.f;
    return winner == player ? 1.f : -1.f;
}

struct Io {
    const float *ra, *rb;
    const uint8_t *ta, *tb, *fa, *fb;
    const int8_t *wa, *wb;
    float *agent_reward, *opp_reward;
    uint8_t *done;
    int8_t *ended_on;
    uint8_t *info;
    int64_t *step_counter;
};

template <bool kDraw>
__global__ __launch_bounds__(256) void k_dual_finish(int n, Io io, Draw d) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (i == 0 && io.step_counter) *io.step_counter += 1;  // read by the next step's launches only
    const uint8_t ta = io.ta[i], fa = io.fa[i], fb = io.fb[i];
    const bool ended_a = ta != 0, ended_b = !ended_a && io.tb[i] != 0;
    const bool passed = !ended_a && (fa & (SPL_F_ILLEGAL | SPL_F_OOB)) == 0;
    io.agent_reward[i] = ended_a ? io.ra[i] : ended_b ? final_reward(0, io.wb[i], fb) : 0.f;
    io.opp_reward[i] = ended_a ? final_reward(1, io.wa[i], fa) : passed ? io.rb[i] : 0.f;
    io.done[i] = ended_a || ended_b;
    io.ended_on[i] = ended_a ? 1 : ended_b ? 2 : 0;
    io.info[i] = ((fa & SPL_F_ILLEGAL) ? SPL_DUAL_ILLEGAL : 0) | (((fa | fb) & SPL_F_DRAW) ? SPL_DUAL_DRAW : 0) |
                 (((fa | fb) & SPL_F_TURN_LIMIT) ? SPL_DUAL_TURN_LIMIT : 0);
    if constexpr (kDraw) {
        if (d.group_prev) d.group_prev[i] = d.group_of[i];
        if (ended_a || ended_b) draw_one(i, d.episode, d.group_of, d.pool_slots, d.pool_len, d.p_current, d.seed, d.table0);
    }
}

// opponent_obs = done ? final_obs : obs, 16 bytes per thread (rows are 297 int32: a 16-byte
// piece may straddle two tables, so each int picks by its own table)
__global__ __launch_bounds__(256) void k_dual_opp_obs(int n, const uint8_t *__restrict__ ta, const uint8_t *__restrict__ tb,
                                                      const int4 *__restrict__ obs, const int4 *__restrict__ fin,
                                                      int4 *__restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, total = (int64_t)n * 297;
    if (4 * q >= total) return;
    if (4 * q + 3 < total) {
        const int4 o = obs[q], f = fin[q];
        int v[4] = {o.x, o.y, o.z, o.w};
        const int w[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int64_t t = (4 * q + k) / 297;
            if (ta[t] != 0 || tb[t] != 0) v[k] = w[k];
        }
        out[q] = make_int4(v[0], v[1], v[2], v[3]);
    } else {
        const int32_t *o = reinterpret_cast<const int32_t *>(obs), *f = reinterpret_cast<const int32_t *>(fin);
        int32_t *d = reinterpret_cast<int32_t *>(out);
        for (int64_t e = 4 * q; e < total; ++e) {
            const int64_t t = e / 297;
            d[e] = (ta[t] != 0 || tb[t] != 0) ? f[e] : o[e];
        }
    }
}



}  // namespace spld

using namespace spld;

extern "C" {

int spl_dual_gate(int32_t n, const uint8_t *terminated_a, const uint8_t *flags_a, int32_t *opp_action, void *stream) {
    if (n <= 0) return spl_fail(SPL_E_ARG, "n must be positive");
    if (!terminated_a || !flags_a || !opp_action) return spl_fail(SPL_E_ARG, "null buffer");
    hipLaunchKernelGGL(k_dual_gate, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, terminated_a, flags_a,
                       opp_action);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SPL_OK : spl_fail(SPL_E_HIP, std::string("k_dual_gate: ") + hipGetErrorString(e));
}

static int dual_finish(int32_t n, const spl_dual_io_t *io, const spl_dual_draw_t *draw, void *stream) {
    if (n <= 0) return spl_fail(SPL_E_ARG, "n must be positive");
    if (draw && (!draw->episode || !draw->group_of || (draw->pool_len > 0 && !draw->pool_slots)))
        return spl_fail(SPL_E_ARG, "null buffer");
    if (draw && !(draw->p_current >= 0.f && draw->p_current <= 1.f)) return spl_fail(SPL_E_ARG, "p_current must be in [0, 1]");
    if (!io || !io->reward_a || !io->reward_b || !io->terminated_a || !io->terminated_b || !io->flags_a ||
        !io->flags_b || !io->winner_a || !io->winner_b || !io->agent_reward || !io->opp_reward || !io->done ||
        !io->game_ended_on || !io->info_flags)
        return spl_fail(SPL_E_ARG, "null buffer");
    if (io->opp_obs && (!io->obs || !io->final_obs)) return spl_fail(SPL_E_ARG, "opp_obs needs obs and final_obs");
    if (io->opp_obs && (((uintptr_t)io->obs | (uintptr_t)io->final_obs | (uintptr_t)io->opp_obs) & 15u))
        return spl_fail(SPL_E_ARG, "observation buffers must be 16-byte aligned");
    const hipStream_t s = (hipStream_t)stream;
    const Io k{io->reward_a, io->reward_b, io->terminated_a, io->terminated_b, io->flags_a, io->flags_b, io->winner_a,
               io->winner_b, io->agent_reward, io->opp_reward, io->done, io->game_ended_on, io->info_flags,
               io->step_counter};
    if (draw) {
        const Draw d{draw->episode, draw->group_of, draw->group_prev, draw->pool_slots, draw->pool_len, draw->p_current,
                     draw->seed, draw->table0};
        hipLaunchKernelGGL(k_dual_finish<true>, dim3((n + 255) / 256), dim3(256), 0, s, n, k, d);
    } else {
        hipLaunchKernelGGL(k_dual_finish<false>, dim3((n + 255) / 256), dim3(256), 0, s, n, k, Draw{});
    }
    if (io->opp_obs) {
        const int64_t quads = ((int64_t)n * 297 + 3) / 4;
        hipLaunchKernelGGL(k_dual_opp_obs, dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, s, n, io->terminated_a,
                           io->terminated_b, reinterpret_cast<const int4 *>(io->obs),
                           reinterpret_cast<const int4 *>(io->final_obs), reinterpret_cast<int4 *>(io->opp_obs));
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SPL_OK : spl_fail(SPL_E_HIP, std::string("k_dual_finish: ") + hipGetErrorString(e));
}

int spl_dual_finish(int32_t n, const spl_dual_io_t *io, void *stream) { return dual_finish(n, io, nullptr, stream); }

int spl_dual_finish_draw(int32_t n, const spl_dual_io_t *io, const spl_dual_draw_t *draw, void *stream) {
    if (!draw) return spl_fail(SPL_E_ARG, "null draw arguments");
    return dual_finish(n, io, draw, stream);
}

int spl_dual_draw_opponents(int32_t n, const uint8_t *draw, uint32_t *episode, int32_t *group_of,
                            const int32_t *pool_slots, int32_t pool_len, float p_current, uint64_t seed, int64_t table0,
                            void *stream) {
    if (n <= 0) return spl_fail(SPL_E_ARG, "n must be positive");
    if (!episode || !group_of || (pool_len > 0 && !pool_slots)) return spl_fail(SPL_E_ARG, "null buffer");
    if (!(p_current >= 0.f && p_current <= 1.f)) return spl_fail(SPL_E_ARG, "p_current must be in [0, 1]");
    hipLaunchKernelGGL(k_draw_opponents, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, draw, episode,
                       group_of, pool_slots, pool_len, p_current, seed, table0);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SPL_OK : spl_fail(SPL_E_HIP, std::string("k_draw_opponents: ") + hipGetErrorString(e));
}

}  // extern "C"

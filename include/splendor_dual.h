/*
 * splendor_dual.h — C-ABI of the batched dual step's glue (wrappers/dual_step_native.py:90-193).
 *
 * A batched DualStepNativeWrapper.dual_step is: spl_step(agent moves, no autoreset) -> the
 * opponent's actions (device policy, or spl_policy_act GREEDY) -> spl_dual_gate -> spl_step(
 * opponent moves, autoreset 2) -> spl_dual_finish.  These two kernels replace the per-table
 * Python branches of the reference wrapper:
 *
 *   spl_dual_gate    the opponent moves only where the agent's move was applied and did not end
 *                    the game (dual_step_native.py:120-140); elsewhere its action becomes -1,
 *                    which spl_step reports as out-of-range and leaves the table unchanged
 *   spl_dual_finish  agent/opponent rewards (final_rewards of the finished game, the step
 *                    reward of the mover: dual_step_native.py:141-193, envs/splendor_env.py:
 *                    92-115), done and the info vectors; optionally the reference's opponent_obs
 *                    (the final observation on finished tables)
 *
 * Conventions as in splendor_amd.h.  The dual glue has no version of its own: it changes with
 * SPL_ABI_VERSION (splendor_amd.h).  ABI 8 appended spl_dual_io_t.step_counter; a caller must
 * zero-initialise every spl_dual_io_t (`spl_dual_io_t io = {0};` / ctypes Structure()) so that a
 * member it does not set is NULL = skip.
 */
#ifndef SPLENDOR_DUAL_H
#define SPLENDOR_DUAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    /* phase A = the agent's move (spl_step outputs), phase B = the opponent's move */
    const float *reward_a, *reward_b;
    const uint8_t *terminated_a, *terminated_b;
    const uint8_t *flags_a, *flags_b;
    const int8_t *winner_a, *winner_b;
    /* outputs [n] */
    float *agent_reward; /* ended on A: A's step reward; ended on B: final_rewards[0]; else 0      */
    float *opp_reward;   /* ended on A: final_rewards[1]; opponent moved: its step reward; else 0 */
    uint8_t *done;
    int8_t *game_ended_on; /* 0 running, 1 on the agent's move, 2 on the opponent's            */
    uint8_t *info_flags;   /* bit 0 illegal agent action, bit 1 draw, bit 2 turn limit          */
    /* optional opponent_obs: done ? final_obs : obs, int32 [n][297] (NULL = skip) */
    const int32_t *obs, *final_obs;
    int32_t *opp_obs;
    /* optional: incremented by one after the dual step (one device thread; NULL = skip).  A
     * graph-captured rollout loop passes it as the next step's policy ply_base (spl_act_args_t),
     * so every replay draws fresh actions without a separate counter launch. */
    int64_t *step_counter;
} spl_dual_io_t;

#define SPL_DUAL_ILLEGAL 0x01
#define SPL_DUAL_DRAW 0x02
#define SPL_DUAL_TURN_LIMIT 0x04

/* opp_action[i] = -1 unless the agent's move on table i was applied and left the game running */
int spl_dual_gate(int32_t n, const uint8_t *terminated_a, const uint8_t *flags_a, int32_t *opp_action,
                  void *stream);
int spl_dual_finish(int32_t n, const spl_dual_io_t *io, void *stream);

/* ppo_splendor.py:137-143 opponent_supplier, per table: every table with draw[t] != 0 (draw NULL = all)
 * starts an episode against group_of[t] = 0 (the current policy) with probability p_current or when
 * pool_len == 0, else pool_slots[i] for i uniform in 0..pool_len-1 (one of the <= pool_size frozen
 * snapshots, ppo_splendor.py:366-370).  Draws come from a Philox stream keyed by (seed; table0 + t,
 * episode[t]) and episode[t] is incremented, so results do not depend on sharding or batching. */
int spl_dual_draw_opponents(int32_t n, const uint8_t *draw, uint32_t *episode, int32_t *group_of,
                            const int32_t *pool_slots, int32_t pool_len, float p_current, uint64_t seed, int64_t table0,
                            void *stream);
/* spl_dual_finish, then in the same launch spl_dual_draw_opponents with draw = io->done (the tables
 * re-dealt in this dual step), group_prev[t] = group_of[t] before the draw (the opponent that played
 * the finished episode; NULL = skip): one launch instead of three (finish, copy, draw). */
typedef struct {
    uint32_t *episode;
    int32_t *group_of;
    int32_t *group_prev;
    const int32_t *pool_slots;
    int32_t pool_len;
    float p_current;
    uint64_t seed;
    int64_t table0;
} spl_dual_draw_t;
int spl_dual_finish_draw(int32_t n, const spl_dual_io_t *io, const spl_dual_draw_t *draw, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SPLENDOR_DUAL_H */

/*
 * splendor_amd.h — C-ABI of the MI355X (gfx950) Splendor rollout engine.
 *
 * The reference has no FFI: its hot path is the Python functions below, called per table.
 * Each entry point here replaces one of them for a whole batch of tables living in HBM:
 *
 *   spl_ctx_create     engine/state.py:113-178 (_load_cards_from_json/_load_nobles_from_json,
 *                      re-parsed on every reset in the reference) -> constant tables uploaded
 *                      once; also builds the token-return RNG table (engine/rules.py:170-176)
 *   spl_reset          envs/splendor_env.py:41-48 SplendorEnv.reset -> engine/state.py:181-211
 *                      initial_state (CPython MT19937 shuffles on device)
 *   spl_deal           engine/rules.py:33-34 initial_state(num_players, seed) with the engine seed
 *                      given directly (the functional engine API)
 *   spl_step           envs/splendor_env.py:51-90 SplendorEnv.step = rules.py:40-93 legal_moves,
 *                      :196-287 apply_action, encode.py:124-187 encode_observation, reward /
 *                      termination, plus gymnasium-0.29 SyncVectorEnv same-step autoreset
 *   spl_rollout        K x spl_step under the device uniform-random policy in one launch
 *                      (splendor_gym/scripts/random_rollout.py:15-26 loop, batched)
 *   spl_encode         engine/encode.py:124-187 encode_observation (current state)
 *   spl_legal          engine/rules.py:40-93 legal_moves (current state)
 *   spl_sample_uniform scripts/random_rollout.py:23 / wrappers/dual_step_native.py:215-223
 *                      random_opponent (uniform over legal; Philox stream, not numpy's)
 *   spl_table_download / spl_table_upload
 *                      the reference's direct `env.state` access (tests/utils.py:25-53 mutate
 *                      it in place) -> host view spl_table_t (splendor_table.h)
 *
 * Conventions
 *  - Every buffer is caller-owned device memory (e.g. a PyTorch-ROCm tensor) passed as a raw
 *    pointer; the library owns only the constant tables inside spl_ctx_t.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).  Calls are asynchronous
 *    on that stream except spl_ctx_create/destroy and the table download/upload helpers.
 *  - Return value: 0 on success, negative SPL_E_* on a host-side argument error (nothing was
 *    launched); spl_last_error() describes it.  Per-table conditions are reported in `flags`.
 *  - Not re-entrant per arena: one host thread drives one arena.
 */
#ifndef SPLENDOR_AMD_H
#define SPLENDOR_AMD_H

#include <stdint.h>

#include "splendor_table.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SPL_ABI_VERSION 9  /* 9: the arena holds a legal-mask cache ([2][n] u32 after the delegation flags,
                                 spl_arena_bytes grows by 8 B per table; spl_step reads it), spl_host_mapped,
                                 spl_ctx_set_step_tail;
                              8: spl_step with both obs and obs_u8 writes both (the compact rows as a copy);
                                 splendor_dual.h spl_dual_io_t gained a trailing step_counter (zero-initialise);
                              7: spl_ctx_set_partner_lead, spl_debug_partner_stats (rollout-store partner hand-off);
                              6: SPL_F_FAULT + spl_ctx_faults (a lost hand-off in a rollout launch is reported);
                              5: spl_step_args_t.obs_u8 (compact observation), gate_terminated / gate_flags */

/* ---- per-table flag bits (uint8) --------------------------------------------------- */
#define SPL_F_ILLEGAL 0x01        /* info["illegal_action"]      envs/splendor_env.py:64-66 */
#define SPL_F_DRAW 0x02           /* info["draw"] (no legal move) envs/splendor_env.py:56-61 */
#define SPL_F_TURN_LIMIT 0x04     /* info["turn_limit"]          envs/splendor_env.py:82-83 */
#define SPL_F_AFTER_TERMINAL 0x08 /* reference raises RuntimeError envs/splendor_env.py:53-54 */
#define SPL_F_OOB 0x10            /* reference raises ValueError  envs/splendor_env.py:62-63 */
#define SPL_F_RESET 0x20          /* autoreset: obs/mask describe the freshly dealt table   */
#define SPL_F_RNG_LIMIT 0x40      /* reserved (ABI 2 raised it when a deal or token return   */
                                  /* outran the MT stream; ABI 3 continues the stream instead) */
#define SPL_F_FAULT 0x80          /* the launch faulted (a lost internal hand-off, spl_ctx_faults):  */
                                  /* this step's outputs of the table were NOT written (stale rows) */

/* ---- device policies for next_actions (scripts/eval_suite.py opponents) --------------- */
#define SPL_POLICY_UNIFORM 0         /* uniform over legal (wrappers/selfplay.py:66-73 random_opponent) */
#define SPL_POLICY_GREEDY_V1 1       /* eval_suite.py:9-29 greedy_opponent_v1 (deterministic)        */
#define SPL_POLICY_BASIC_PRIORITY 2  /* eval_suite.py:32-78 basic_priority_opponent                  */

/* ---- error codes -------------------------------------------------------------------- */
#define SPL_OK 0
#define SPL_E_ARG -1      /* bad argument (null pointer, size, player count) */
#define SPL_E_HIP -2      /* HIP runtime error */
#define SPL_E_RANGE -3    /* host view out of the device's representable range */

typedef struct spl_ctx_s spl_ctx_t;

/* Device arena descriptor (host memory, owned by the caller).  `base` points at caller-owned
 * device memory of at least spl_arena_bytes(n, players) bytes, 256-byte aligned. */
typedef struct spl_arena_s {
    void *base;
    int64_t bytes;
    int32_t n;            /* tables */
    int32_t players;      /* 2..4 */
    int64_t steps;        /* maintained by the library: spl_step calls since the last reset */
    int64_t epoch;        /* maintained by the library: pool refills launched so far */
} spl_arena_t;

/* Batched step arguments (all device pointers; [n] = one entry per table). */
typedef struct spl_step_args_s {
    const int32_t *actions;  /* [n] action per table (0..44 legal range)                    */
    int32_t *obs;            /* [n][297] observation after the step (reset obs on SPL_F_RESET) */
    int8_t *mask;            /* [n][45]  action mask after the step                          */
    float *reward;           /* [n]      reward of the mover                                 */
    uint8_t *terminated;     /* [n]                                                          */
    uint8_t *flags;          /* [n]      SPL_F_* bits                                        */
    int8_t *winner;          /* [n] or NULL: winner of the state the step produced (−1 None) */
    int32_t *final_obs;      /* [n][297] or NULL: terminal obs, written on SPL_F_RESET rows  */
    int32_t autoreset;       /* 1: terminated tables are re-dealt in the same step; 2: also the
                                tables already terminal when the step starts (no move applied:
                                SPL_F_RESET, reward 0, final_obs row = that terminal obs)        */
    int32_t policy;          /* next_actions policy: SPL_POLICY_* (0 = uniform random)       */
    int32_t *next_actions;   /* [n] or NULL: fused policy's action over the new state / mask */
    const uint64_t *ply_base; /* device, nullable: added to `ply` (lets a captured graph replay) */
    uint64_t policy_seed;    /* Philox key for next_actions                                  */
    uint64_t ply;            /* Philox counter for next_actions                              */
    int64_t table0;          /* global id of table 0 (sharding: streams keyed by global id) */
    float *ep_return;        /* [n] or NULL: += final reward of player 0 on termination      */
    uint32_t *ep_count;      /* [n] or NULL: += 1 on termination                             */
    uint8_t *info;           /* [4][n] or NULL (spl_step only): 0/1 bytes of the gymnasium info
                                planes illegal_action, draw, turn_limit (the SPL_F_ILLEGAL / DRAW /
                                TURN_LIMIT bits of `flags`), then the step's `truncated` (always 0:
                                SplendorEnv.step never truncates, envs/splendor_env.py:61-90)   */
    uint64_t *errors;        /* [1] or NULL (spl_step only): += the number of tables whose flags
                                carry SPL_F_OOB or SPL_F_AFTER_TERMINAL (the reference's
                                ValueError / RuntimeError cases, envs/splendor_env.py:53-63)   */
    uint8_t *obs_u8;         /* [n][300] or NULL (spl_step only): the observation as bytes for a
                                device consumer (spl_act_args_t.obs_u8), a quarter of obs's bytes:
                                bytes 0..296 = obs (every value < 256 but move_count, byte 295 =
                                move_count mod 256), byte 297 = move_count >> 8, 298-299 = 0.
                                With obs NULL only the bytes are written; with obs set too (ABI 8)
                                both are, the bytes a copy of the rows (a fused actor's input
                                beside the int32 observation the caller keeps)                   */
    const uint8_t *gate_terminated; /* [n] or NULL (spl_step only, with gate_flags): the dual step's
                                gate fused into the opponent's move — where gate_terminated[t] != 0
                                or gate_flags[t] has SPL_F_ILLEGAL / SPL_F_OOB (the agent's move
                                ended the game or was not applied) actions[t] becomes -1 (written
                                back) and the table is not moved (spl_dual_gate + spl_step) */
    const uint8_t *gate_flags;
} spl_step_args_t;

int spl_abi_version(void);
const char *spl_last_error(void);

/* cards: 90 x 8 int32 [tier, bonus colour, points, cost w,b,g,r,k];
 * nobles: 10 x 6 int32 [req w,b,g,r,k, points]   (splendor_gym/engine/data/tables.json) */
int spl_ctx_create(int device, const int32_t *cards, const int32_t *nobles, spl_ctx_t **out);
int spl_ctx_destroy(spl_ctx_t *ctx);
/* Pool refill period in steps (default 64; three pool deals per table cover three resets in between);
 * 0 disables automatic refills (inline deals). */
int spl_ctx_set_refill_period(spl_ctx_t *ctx, int period);
/* spl_rollout only: 1 (default) = a due refill runs inside the rollout launch, each wave at a step
 * of its own while other waves' stores keep HBM busy; 0 = a separate spl_refill launch after it.
 * Results are identical either way. */
int spl_ctx_set_refill_fused(spl_ctx_t *ctx, int fused);
/* spl_rollout only: the two-wave pipelined kernel (one wave steps the tables, the other encodes
 * and stores the step's outputs) vs one wave per 64 tables (0).  1 (default) = auto: the six-wave
 * dealer variant (5) when every 128-table workgroup of it is resident at once (one per CU, e.g.
 * 32 768 tables), else the three-wave dealer variant (4: a third wave deals the pool refills beside the
 * other two) when it fits, else at 2 players the quad variant (6) when every 256-table workgroup of it
 * is resident at once (e.g. the headline's 65 536 tables), else two-wave at 64 tables per workgroup;
 * 2 = two-wave at 64; 3 = two-wave
 * at 32; 4 = the three-wave dealer variant; 5 = the six-wave dealer variant (two dealer teams per
 * 128-table workgroup, roles given to waves by the SIMD they run on); 6 = the quad variant (four
 * two-wave teams per 256-table workgroup, one workgroup per CU, roles by SIMD; the partner hand-off
 * of spl_ctx_set_partner_lead runs in it).
 * Results are identical in every mode. */
int spl_ctx_set_rollout_pipeline(spl_ctx_t *ctx, int on);
/* spl_rollout with per_step_outputs at 64 tables per workgroup only: rollout-store delegation.  On
 * every `every`-th step (every >= 4; 0 = off) each workgroup on an odd XCC skips that step's encode
 * and stages its 64 tables' state words after the step (64 x num_words(P) u32, 4.3 KB at 2 players,
 * sc1 stores, released by s_waitcnt vmcnt(0) before an sc1 ready flag) for its partner on the
 * neighbouring even XCC, which encodes the rows and stores them into the rollout store after its
 * own steps: MI355X's odd XCCs drain stores ~20 % slower, and the slowest sets the launch time.
 * Turned off for grids larger than the resident workgroup capacity (pairs might not run together).
 * Default: SPL_DELEG_EVERY (DESIGN.md §2 gives the measured A/B).  Results are identical either way. */
int spl_ctx_set_rollout_delegation(spl_ctx_t *ctx, int every);
/* Partner hand-off of the rollout store in the kernels that run one workgroup per CU with the grid
 * resident at once: the six-wave dealer (k_rollout_store_dealer2_<P>p, 384 threads) and the quad
 * variant (k_rollout_store_quad_<P>p, 512 threads); the two-wave kernels (several workgroups per CU)
 * have none since the round-5 library: a 64-table team that falls `lead` or more steps behind the same team of the
 * workgroup on the neighbouring XCC hands whole steps of observation rows (its state words, ~6 KB) to
 * that team's output wave, which encodes and stores them between its own steps (the XCCs drain the
 * rollout store at different rates under load).  0 = off, -1 = hand off whenever a slot
 * is free (tests).  Other kernels ignore it.  Default 0 = off (round 6: with the sc0 nt sc1 row stores
 * the teams lag little and the hand-off no longer pays; DESIGN.md §4.1 gives the measured A/B).
 * Results are identical either way. */
int spl_ctx_set_partner_lead(spl_ctx_t *ctx, int lead);
/* spl_step's kernel shape (round 6): 0 = two waves (k_step_ws_<P>p: the rules wave evaluates the new
 * state's legal mask after the row halves), 1 = three waves per 64 tables (k_step_wst_<P>p: a TAIL wave
 * takes the new state's legal mask, the mask block, the fused policy's action and the legal-mask cache off
 * the rules wave), 2 = two waves with the OUTPUT wave evaluating the mask between the halves of its row
 * stores (k_step_wso_<P>p); -1 = auto (default, by grid size: DESIGN.md §4.3).  Results are identical. */
int spl_ctx_set_step_tail(spl_ctx_t *ctx, int mode);
/* The name of the kernel spl_rollout launches for n tables of `players` players under the context's
 * settings (e.g. "k_rollout_store_2p", "k_rollout_inplace_half_4p"): every instantiation has a name
 * of its own, so a rocprofv3 summary row maps to one variant.  NULL (spl_last_error) on bad input. */
const char *spl_rollout_kernel_name(spl_ctx_t *ctx, int32_t n, int32_t players, int32_t per_step_outputs);

/* Launch faults.  A spl_rollout launch of the three-wave dealer variant whose waves hand off through
 * LDS counters bounds every wait; a wait that runs out (a lost hand-off: never in a correct run) stops
 * that workgroup — it stores no more steps and leaves its tables' state as it was, marks SPL_F_FAULT in
 * the flags of every step it did not store — and writes the launch's serial (spl_ctx_launches at the
 * time of the call) into the context's fault word.  The word lives in host-mapped memory the kernel
 * writes through to, so reading it needs no synchronisation: it shows the faults of every launch that
 * has finished (and of running ones as they happen).  After a fault the tables must be reset.
 * spl_ctx_faults: *launch = the word (0 = no fault since the last clear); `clear` zeroes it.
 * spl_ctx_fault_word: the word's host address, for polling without a call (valid until destroy).
 * spl_ctx_launches: kernel launches through this context so far (spl_step / spl_rollout serials). */
int spl_ctx_faults(spl_ctx_t *ctx, uint64_t *launch, int clear);
const volatile uint64_t *spl_ctx_fault_word(spl_ctx_t *ctx);
uint64_t spl_ctx_launches(spl_ctx_t *ctx);
/* Whether host memory `host` is page-locked by HIP and mapped into the device at the SAME address
 * (*same_address = 1), so a kernel may be handed the host pointer itself (SplendorEnv's pinned I/O
 * block); 0 otherwise (e.g. registered rather than allocated pinned memory): the caller must then
 * use device memory and copy.  Not part of the reference; host-side check only (hipHostGetDevicePointer). */
int spl_host_mapped(const void *host, int32_t *same_address);

int64_t spl_arena_bytes(int32_t n, int32_t players);
/* Zero the arena and mark every table's pool as not dealt (must precede the first spl_reset
 * of a fresh allocation).  A table that was never reset with a seed has no engine-seed stream:
 * an unseeded reset or a refill deals it from engine seed 0. */
int spl_arena_init(spl_ctx_t *ctx, spl_arena_t *arena, void *stream);

/* Reset tables.  pcg (device, nullable): 4 x uint64 per table = numpy PCG64 state
 * (state_hi, state_lo, inc_hi, inc_lo) of the table's gymnasium np_random after seeding; when
 * given, the table's engine-seed stream restarts from it (reset(seed=...)); when NULL the
 * stream continues (reset() without a seed).  reset_mask (device, nullable): tables with a
 * non-zero byte are reset, NULL = all.  obs/mask (nullable) receive every table's current
 * observation / action mask after the reset. */
int spl_reset(spl_ctx_t *ctx, spl_arena_t *arena, const uint64_t *pcg, const uint8_t *reset_mask,
              int32_t *obs, int8_t *mask, void *stream);

/* engine/state.py:181-211 initial_state(players, seed) (engine/rules.py:33-34) from an explicit engine
 * seed per table (device [n] uint32; CPython seeds abs(seed) < 2^32), for tables with a non-zero
 * deal_mask byte (NULL = all).  Unlike spl_reset it does not touch the table's engine-seed stream and
 * deals no pool records.  obs/mask (nullable) as in spl_reset.  The functional engine API
 * (splendor_gym.engine.initial_state) runs on this. */
int spl_deal(spl_ctx_t *ctx, spl_arena_t *arena, const uint32_t *engine_seeds, const uint8_t *deal_mask,
             int32_t *obs, int8_t *mask, void *stream);

int spl_step(spl_ctx_t *ctx, spl_arena_t *arena, const spl_step_args_t *args, void *stream);

/* `steps` consecutive SplendorEnv.step calls of every table under the device uniform-random
 * policy (splendor_gym/scripts/random_rollout.py:15-26 batched): identical to `steps` spl_step calls in which
 * next_actions of one call is the next call's actions and ply runs ply, ply+1, ...  args.actions
 * holds the first step's actions; args.next_actions (nullable) receives the action sampled after
 * the last step.  With per_step_outputs != 0, step k writes block k of every output array (obs
 * [steps][n][297], mask [steps][n][45], reward/terminated/flags/winner [steps][n], final_obs
 * [steps][n][297]; n divisible by 4); otherwise every step overwrites block 0.  A pool refill
 * is due when the step counter crosses a multiple of the refill period (keep steps <= period);
 * it runs inside the launch (spl_ctx_set_refill_fused) or as a spl_refill launch after it. */
int spl_rollout(spl_ctx_t *ctx, spl_arena_t *arena, const spl_step_args_t *args, int32_t steps,
                int32_t per_step_outputs, void *stream);

/* Pool maintenance: every table with consumed pool records gets the earliest of them re-dealt
 * (one deal per table per call).  A reset with both pool records consumed deals inline. */
int spl_refill(spl_ctx_t *ctx, spl_arena_t *arena, void *stream);

int spl_encode(spl_ctx_t *ctx, spl_arena_t *arena, int32_t *obs, void *stream);
int spl_legal(spl_ctx_t *ctx, spl_arena_t *arena, int8_t *mask, void *stream);

/* Uniform-random legal action per table from a [n][45] int8 mask (0 if none is legal). */
int spl_sample_uniform(spl_ctx_t *ctx, int32_t n, const int8_t *mask, int32_t *actions,
                       uint64_t seed, uint64_t ply, int64_t table0, void *stream);

/* The flags of a step split for a gymnasium info dict (envs/splendor_env.py:70-90 info keys):
 * info[0*n + t] = illegal_action, info[n + t] = draw, info[2n + t] = turn_limit (0/1 bytes), and
 * *errors (8-byte aligned, device) += the number of tables whose flags carry SPL_F_OOB or
 * SPL_F_AFTER_TERMINAL (the reference's ValueError / RuntimeError): a running count, compared with
 * its previous value by the caller.  One launch, asynchronous on `stream`. */
int spl_step_info(int32_t n, const uint8_t *flags, uint8_t *info, uint64_t *errors, void *stream);

/* Host-view copies of `count` tables starting at `first` (synchronous on `stream`). */
int spl_table_download(spl_ctx_t *ctx, spl_arena_t *arena, int32_t first, int32_t count,
                       spl_table_t *host, void *stream);
int spl_table_upload(spl_ctx_t *ctx, spl_arena_t *arena, int32_t first, int32_t count,
                     const spl_table_t *host, void *stream);

/* TEST HOOK: how many MT19937 outputs a deal or token return takes from the register-only stream
 * before the full-state continuation takes over (default and maximum 454, the stream's reach;
 * process-wide, current device).  Results are identical for every value: the parity tests lower it
 * to drive every deal and token return through the continuation. */
int spl_debug_set_stream_limit(int outputs);

/* TEST HOOK: polls after which a dealer-rollout hand-off wait gives up and faults the launch (see
 * spl_ctx_faults; default and maximum 2^22, a fraction of a second; negative = default).  Process-wide,
 * current device.  0 makes the first wait that has to wait fault: tests force the fault path with it. */
int spl_debug_set_spin_limit(int64_t polls);
/* DIAGNOSTIC: partner hand-off tasks since the last clear, process-wide on the current device:
 * stats[0] stored by the partner's dealer wave, stats[1] claimed back by the team that posted them.
 * Synchronises the device; `clear` zeroes them. */
int spl_debug_partner_stats(uint64_t *stats, int clear);

/* TEST HOOK of the bounds-check build (libsplendor_amd_checked.so, -DSPL_BOUNDS_CHECK): the OR of the
 * invariant violations the kernels recorded (table / slot / deck / token-table / deal-scratch index,
 * byte-packed counts out of range), cleared when `clear`.  Synchronises the device.  The product
 * build returns SPL_E_ARG. */
int spl_debug_bounds_flags(uint32_t *flags, int clear);

/* Copy of the token-return RNG table (spl_ctx_create builds it on device), for tests.
 * Returns the number of uint32 words (4 per entry) when out == NULL. */
int64_t spl_ctx_token_lut(spl_ctx_t *ctx, uint32_t *out, int64_t words);

#ifdef __cplusplus
}
#endif
#endif /* SPLENDOR_AMD_H */

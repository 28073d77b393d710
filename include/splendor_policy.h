/*
 * splendor_policy.h — C-ABI of the fused ActorCritic forward for batched self-play (gfx950).
 *
 * The reference runs its PPO actor as torch modules on one observation at a time
 * (ppo_splendor.py:40-59 ActorCritic; :235-269 the rollout loop calls
 * agent.get_action_and_value per step and the opponent's frozen actor per env), with
 * masked_categorical (ppo_splendor.py:27-37) for sampling and the greedy masked argmax of
 * training_utils.py:263-276 frozen_policy_from / scripts/eval_suite.py model_greedy_policy_from
 * for opponents.  These entry points evaluate that network for a whole batch of tables in one
 * launch: observations (int32 [n][297]) and masks (int8 [n][45]) straight from the engine, tanh /
 * softmax / sampling fused.  Three precisions:
 *   SPL_PREC_FP32 (default)  the reference's fp32 with EXACT fp32 operands: every weight and
 *                            activation as three bf16 planes (24 significant bits: the fp32 value
 *                            itself), the six plane products of order <= 2 accumulated in fp32 on
 *                            v_mfma_f32_16x16x32_bf16 (the dropped terms are <= 2^-24 of each
 *                            product); the observation exact (one plane below 256, a residual plane
 *                            where a value is larger, < 2^16); fp32 tanh to a few ulp
 *                            (spl_policy32.hip, k_act32)
 *   SPL_PREC_FP32_F16X2      fp32 within 2^-22: two fp16 planes per operand (22 significant bits,
 *                            weights scaled per row by a power of two), three plane products on
 *                            v_mfma_f32_16x16x32_f16, tanh with ~1e-7 absolute error (k_act32h): the
 *                            round-4 form, faster, not an exact operand representation
 *   SPL_PREC_BF16 (opt-in)   bf16 MFMA (v_mfma_f32_32x32x16_bf16) with fp32 accumulation (spl_policy.hip)
 *
 *   spl_policy_bytes   size of a packed weight image (actor only, or actor + critic; per precision)
 *   spl_policy_pack    nn.Linear fp32 weights [out][in] + biases -> packed image (device)
 *   spl_policy_act     ActorCritic.get_action_and_value (SAMPLE) or the greedy masked argmax
 *                      (GREEDY) for n tables
 *
 * Conventions as in splendor_amd.h: caller-owned device buffers as raw pointers, `stream` a
 * hipStream_t as void*, 0 / negative SPL_E_* returns, spl_last_error() for the message.
 */
#ifndef SPLENDOR_POLICY_H
#define SPLENDOR_POLICY_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SPL_POLICY_ABI 5  /* 2: precision argument, args->image describes the image; 3: obs_u8;
                             4: fp32 images as two fp16 planes (spl_policy_bytes changed); each chunk also
                                carries its rows' tanh factors (same size: pack and act from one library);
                             5: SPL_PREC_FP32 is exact (three bf16 planes; spl_policy_bytes changed), the
                                two-fp16-plane form is SPL_PREC_FP32_F16X2 */

#define SPL_PREC_FP32 0
#define SPL_PREC_BF16 1
#define SPL_PREC_FP32_F16X2 2
#define SPL_IMG_CRITIC 1 /* spl_act_args_t.image bit 0: the image holds the critic; bits 1-2: SPL_PREC_* */

/* one nn.Sequential(Linear(297,256), Tanh, Linear(256,256), Tanh, Linear(256,out)):
 * weights row-major [out][in] (torch's nn.Linear.weight), biases [out], fp32, device memory */
typedef struct {
    const float *w1, *b1; /* [256][297], [256] */
    const float *w2, *b2; /* [256][256], [256] */
    const float *w3, *b3; /* [out][256], [out]: out = 45 (actor) or 1 (critic) */
} spl_mlp_t;

#define SPL_ACT_SAMPLE 0 /* masked categorical sample + log_prob + entropy (+ critic value)     */
#define SPL_ACT_GREEDY 1 /* argmax of the actor logits with illegal actions at -inf (first max)  */
#define SPL_ACT_VALUE 2  /* the critic alone (ActorCritic.get_value, ppo_splendor.py:51): fp32 images
                          * with a critic; writes args->value only, mask and action may be NULL     */

typedef struct {
    const int32_t *obs;  /* [n][297] int32, 16-byte aligned                                       */
    const int8_t *mask;  /* [n][45] int8 (nonzero = legal), 4-byte aligned                        */
    int32_t *action;     /* [n] out                                                               */
    float *logprob;      /* [n] out (SAMPLE; may be NULL)                                         */
    float *entropy;      /* [n] out, per table (SAMPLE; may be NULL; the reference reports mean)  */
    float *value;        /* [n] out: critic(x) (SAMPLE, VALUE; NULL in SAMPLE skips the critic)   */
    float *logits;       /* [n][45] out: raw actor logits before masking (may be NULL)            */
    uint64_t seed;       /* SAMPLE: Philox key; draw for table t at ply p = f(seed; table0+t, p)  */
    uint64_t ply;
    const uint64_t *ply_base; /* device, nullable: added to `ply` (lets a captured graph replay)  */
    int64_t table0;
    int32_t mode;        /* SPL_ACT_*                                                            */
    int32_t image;       /* how the image was packed: SPL_IMG_CRITIC if with a critic | precision << 1;
                            packed_bytes must equal spl_policy_bytes(critic, precision)              */
    const uint8_t *obs_u8; /* [n][300] or NULL: the observation as spl_step's obs_u8 bytes, read
                            instead of obs (fp32 images of either format only); obs may then be NULL */
} spl_act_args_t;

/* bytes of a packed image: with_critic 0 = actor only (greedy opponents), 1 = actor + critic;
 * SPL_E_ARG for an unknown precision */
int64_t spl_policy_bytes(int32_t with_critic, int32_t precision);
/* pack `actor` (and `critic` unless NULL) into `packed` (spl_policy_bytes(critic != NULL, precision)
 * bytes, 256-byte aligned device memory); asynchronous on `stream` */
int spl_policy_pack(const spl_mlp_t *actor, const spl_mlp_t *critic, int32_t precision, void *packed, void *stream);
/* evaluate the packed network on n tables; SAMPLE with args->value != NULL needs a packed image
 * that holds the critic */
int spl_policy_act(const void *packed, int64_t packed_bytes, int32_t n, const spl_act_args_t *args,
                   void *stream);

/* Per-table networks (the opponent pool of ppo_splendor.py:137-143, 366-370: each episode plays the
 * current policy or one frozen snapshot): `images` holds n_images actor-only fp32 images (either fp32
 * format, as args->image says), image i at
 * images + i * image_bytes; table t is evaluated with image group_of[t] (device [n]; tables with an
 * index outside 0..n_images-1 get no action).  Tables are counting-sorted by image into `scratch`
 * (spl_policy_group_scratch_bytes(n, n_images) bytes, caller-owned device memory, ZERO-FILLED before
 * its first use: the call leaves its counters zeroed for the next one); every image's full 128-table
 * workgroups and then its tail in 16-table workgroups (hidden units split over the waves) are
 * evaluated; results equal spl_policy_act on each image. */
int64_t spl_policy_group_scratch_bytes(int32_t n, int32_t n_images);
int spl_policy_act_grouped(const void *images, int64_t image_bytes, int32_t n_images, const int32_t *group_of,
                           void *scratch, int32_t n, const spl_act_args_t *args, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SPLENDOR_POLICY_H */

"""Fused, batched ActorCritic forward on the GPU (include/splendor_policy.h).

`FusedActorCritic(model)` packs a reference-architecture ActorCritic (ppo_splendor.py:40-59;
splendor_gym.policy.ActorCritic) into a weight image once, then evaluates it for a whole batch of
tables in one HIP launch straight from the engine's int32 observations and int8 masks:

  * ``act(obs, mask)`` = ``model.get_action_and_value(obs.float(), mask.float())`` without
    gradients: a masked-categorical sample (ppo_splendor.py:27-37 semantics, rows without a legal
    action sample from the raw logits), its log-probability, the per-table entropy and the
    critic's value.  The draw is a Philox stream keyed by (seed; table, ply), not torch's
    multinomial stream: same distribution, different samples.
  * ``greedy(obs, mask)`` = ``argmax(actor(obs).masked_fill(mask < 0.5, -inf))`` (first maximum;
    0 when nothing is legal) — the frozen-opponent policy of training_utils.py:263-276.
  * ``get_value(obs)`` = ``model.get_value(obs.float())`` (ppo_splendor.py:51, the bootstrap value
    of ppo_splendor.py:302): the critic alone, fp32.

precision="fp32" (default, the reference's precision): EXACT fp32 operands — every weight and hidden
activation split into three bf16 planes (24 significant bits: the fp32 value itself), the six plane
products of order <= 2 accumulated in fp32 on v_mfma_f32_16x16x32_bf16, the observation exact, tanh to
a few ulp (csrc/spl_policy32.hip, k_act32) — so logits and values equal the fp32 module's to within
fp32 rounding (tests/test_gpu_policy.py).  precision="fp32_f16x2": round 4's faster form, two fp16
planes per operand (22 significant bits), fp32 within 2^-22 per operand (k_act32h).
The trade-off: the default buys an EXACT operand representation, not a smaller output
error.  Against a float64 evaluation of the same module at 65 536 tables the end-to-end logit error is
4.7e-7 for "fp32", 3.0e-7 for "fp32_f16x2" and 5.4e-7 for torch fp32 itself (both forms' error is the
fp32 rounding of the sums; tests/test_gpu_policy.py::test_exact_format_error_against_float64 pins all
three), while "fp32_f16x2" is ~35 % faster (bench.py's config5_selfplay_f16x2 line).  The pool and the
agent default to "fp32" so that no operand is rounded before the products, as in the reference.
precision="bf16" (opt-in): bf16 MFMA with fp32 accumulation, logits to bf16 accuracy.  Call
``refresh()`` after the module's weights change (e.g. after each PPO update).
"""
import ctypes
import weakref

from . import _native
from ._native import (ACT_GREEDY, ACT_SAMPLE, ACT_VALUE, IMG_CRITIC, NUM_ACTIONS, OBS_DIM, OBS_U8, PREC_BF16, PREC_FP32,
                      PREC_FP32_F16X2, ActArgs, MlpDesc, check, ptr)

_PRECISIONS = {"fp32": PREC_FP32, "fp32_f16x2": PREC_FP32_F16X2, "bf16": PREC_BF16}
_FP32_FORMS = ("fp32", "fp32_f16x2")  # the spl_policy32.hip kernels: compact rows, get_value, grouped pools


def _mlp_desc(seq, keep):
    """spl_mlp_t of an nn.Sequential(Linear, Tanh, Linear, Tanh, Linear) (fp32 contiguous copies
    are kept alive in `keep`)."""
    lin = [m for m in seq if m.__class__.__name__ == "Linear"]
    if len(lin) != 3 or lin[0].in_features != OBS_DIM or lin[0].out_features != 256 or \
            lin[1].in_features != 256 or lin[1].out_features != 256 or lin[2].in_features != 256:
        raise ValueError("FusedActorCritic needs the reference architecture: Linear(297,256)-Tanh-"
                         "Linear(256,256)-Tanh-Linear(256,out)")
    ts = []
    for m in lin:
        ts.append(m.weight.detach().float().contiguous())
        ts.append(m.bias.detach().float().contiguous())
    keep.extend(ts)
    return MlpDesc(*[t.data_ptr() for t in ts])


class FusedActorCritic:
    def __init__(self, model, with_critic=True, device=None, precision="fp32"):
        torch = _native.require_gpu()
        self.torch = torch
        self.lib = _native.load_library()
        self.model = model
        self.with_critic = bool(with_critic)
        if precision not in _PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(_PRECISIONS)}")
        self.precision = precision
        self._prec = _PRECISIONS[precision]
        self._image_flags = (IMG_CRITIC if self.with_critic else 0) | (self._prec << 1)
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        if self.device.type != "cuda":
            raise ValueError("FusedActorCritic: the model must live on a GPU (no CPU fallback)")
        nbytes = self.lib.spl_policy_bytes(1 if self.with_critic else 0, self._prec)
        self.image = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self.refresh()

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def refresh(self):
        """Re-pack the module's current weights (asynchronous on the current stream)."""
        keep = []
        actor = _mlp_desc(self.model.actor, keep)
        if self.model.actor[-1].out_features != NUM_ACTIONS:
            raise ValueError("actor must have 45 outputs")
        critic = None
        if self.with_critic:
            if self.model.critic[-1].out_features != 1:
                raise ValueError("critic must have 1 output")
            critic = _mlp_desc(self.model.critic, keep)
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_policy_pack(ctypes.byref(actor), ctypes.byref(critic) if critic else None,
                                                     self._prec, self.image.data_ptr(), self._stream()))
        self._keep = keep  # the pack kernel reads them asynchronously

    def _check_inputs(self, obs, mask):
        t = self.torch
        u8 = obs.dtype == t.uint8 and self.precision in _FP32_FORMS  # compact rows (Engine.step obs_u8)
        if (obs.dtype != t.int32 and not u8) or obs.dim() != 2 or obs.shape[1] != (OBS_U8 if u8 else OBS_DIM) \
                or not obs.is_contiguous():
            raise ValueError("obs must be a contiguous int32 [n, 297] device tensor (fp32: or uint8 [n, 300] rows)")
        if mask.dtype not in (t.int8, t.uint8, t.bool) or tuple(mask.shape) != (obs.shape[0], NUM_ACTIONS) or \
                not mask.is_contiguous():
            raise ValueError("mask must be a contiguous int8 [n, 45] device tensor")
        if obs.device != self.device or mask.device != self.device:
            raise ValueError("obs/mask must be on the policy's device")
        return obs.shape[0]

    def _run(self, obs, mask, mode, action, logprob=None, entropy=None, value=None, logits=None, seed=0, ply=0,
             table0=0, ply_base=None):
        n = self._check_inputs(obs, mask) if mask is not None else obs.shape[0]
        u8 = obs.dtype == self.torch.uint8
        a = ActArgs(obs=None if u8 else obs.data_ptr(), obs_u8=obs.data_ptr() if u8 else None, mask=ptr(mask), action=ptr(action), logprob=ptr(logprob),
                    entropy=ptr(entropy), value=ptr(value), logits=ptr(logits), seed=int(seed) & (2**64 - 1),
                    ply=int(ply) & (2**64 - 1), ply_base=ptr(ply_base), table0=int(table0), mode=mode, image=self._image_flags)
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_policy_act(self.image.data_ptr(), self.image.numel(), n, ctypes.byref(a),
                                                    self._stream()))

    def act(self, obs, mask, seed=0, ply=0, table0=0, out=None, want_logits=False, ply_base=None):
        """(action int32 [n], logprob f32 [n], entropy f32 [n], value f32 [n, 1] or None[, logits]).
        The draw of table i is keyed by (seed; table0 + i, ply + *ply_base); ply_base is an
        optional int64 device scalar that a captured graph can advance between replays."""
        t = self.torch
        n = obs.shape[0]
        o = out or {}
        action = o.get("action", t.empty(n, dtype=t.int32, device=self.device))
        logprob = o.get("logprob", t.empty(n, dtype=t.float32, device=self.device))
        entropy = o.get("entropy", t.empty(n, dtype=t.float32, device=self.device))
        value = o.get("value", t.empty(n, 1, dtype=t.float32, device=self.device)) if self.with_critic else None
        logits = t.empty(n, NUM_ACTIONS, dtype=t.float32, device=self.device) if want_logits else None
        self._run(obs, mask, ACT_SAMPLE, action, logprob, entropy, value, logits, seed, ply, table0, ply_base)
        return (action, logprob, entropy, value, logits) if want_logits else (action, logprob, entropy, value)

    def greedy(self, obs, mask, out=None, want_logits=False):
        """argmax of the masked actor logits, int32 [n] (and the raw logits when asked)."""
        t = self.torch
        n = obs.shape[0]
        action = out if out is not None else t.empty(n, dtype=t.int32, device=self.device)
        logits = t.empty(n, NUM_ACTIONS, dtype=t.float32, device=self.device) if want_logits else None
        self._run(obs, mask, ACT_GREEDY, action, logits=logits)
        return (action, logits) if want_logits else action

    def get_value(self, obs, out=None):
        """ActorCritic.get_value (ppo_splendor.py:51): the critic's value, f32 [n, 1].  Needs
        with_critic and an fp32 precision."""
        t = self.torch
        if not self.with_critic or self.precision not in _FP32_FORMS:
            raise ValueError("get_value needs an fp32 image with the critic")
        if obs.dtype != t.int32 or obs.dim() != 2 or obs.shape[1] != OBS_DIM or not obs.is_contiguous() or \
                obs.device != self.device:
            raise ValueError("obs must be a contiguous int32 [n, 297] tensor on the policy's device")
        value = out if out is not None else t.empty(obs.shape[0], 1, dtype=t.float32, device=self.device)
        self._run(obs, None, ACT_VALUE, None, value=value)
        return value

    def opponent(self):
        """A batched opponent for DualStepVectorEnv: (obs, mask) -> int32 actions.  An fp32 one also
        takes the compact uint8 rows (accepts_u8), which the dual step then writes for it."""
        f = self

        class _Opponent:
            accepts_u8 = f.precision in _FP32_FORMS

            def __call__(self, obs, mask):
                return f.greedy(obs, mask)

        return _Opponent()


class OpponentPool:
    """The self-play opponent of ppo_splendor.py:137-143 / 366-370, batched: each table's episode
    plays either the CURRENT policy (probability p_current, and always while the pool is empty) or
    one of up to `pool_size` frozen snapshots chosen uniformly — drawn per table at every episode
    start (spl_dual_draw_opponents: Philox keyed by (seed; table, episode), so results do not depend
    on batching or sharding).  Every network is the greedy masked argmax of its actor
    (model_greedy_policy_from / frozen_policy_from), evaluated for all tables in ONE launch
    (spl_policy_act_grouped: tables sorted by network, one network per workgroup), at `precision`
    ("fp32": exact fp32 operands, the default; or "fp32_f16x2").

    Images: slot 0 is the current policy (re-packed by refresh(), e.g. after each PPO update);
    snapshots live in a ring of pool_size + 2 slots.  A snapshot that leaves the pool keeps its
    weights while any table's current episode still plays it (the per-table opponent tensors of the
    envs using the pool are tracked: DualStepVectorEnv registers its own), so episodes already
    playing it finish against it, as the reference's per-episode frozen copies do; add_snapshot
    writes the next ring slot that no pool member and no running episode uses, growing the ring
    (up to MAX_IMAGES) when every slot is busy.  The image ring and the grouping scratch are allocated
    at their maximum size up front, so growing never moves them: memory a hipGraph captured stays valid
    across add_snapshot (a graph holding act() bakes in the group count: re-capture it after the ring
    grows).  (The reference appends agent.state_dict(), whose
    tensors alias the live parameters, so its "frozen" pool entries are the current weights at the
    episode's start; add_snapshot here copies the weights at the time it is called.)"""

    MAX_IMAGES = 64

    def __init__(self, agent, pool_size: int = 12, p_current: float = 0.25, seed: int = 0, device=None,
                 precision="fp32"):
        torch = _native.require_gpu()
        if precision not in _FP32_FORMS:
            raise ValueError(f"OpponentPool precision must be one of {_FP32_FORMS}")
        self.precision = precision
        self._prec = _PRECISIONS[precision]
        self.torch = torch
        self.lib = _native.load_library()
        self.agent = agent
        self.pool_size, self.p_current, self.seed = int(pool_size), float(p_current), int(seed)
        self.device = torch.device(device) if device is not None else next(agent.parameters()).device
        self.image_bytes = int(self.lib.spl_policy_bytes(0, self._prec))
        self.n_images = 1 + self.pool_size + 2
        if self.n_images > self.MAX_IMAGES:
            raise ValueError(f"pool_size at most {self.MAX_IMAGES - 3}")
        # every image slot the ring can ever grow to (~1 MB each): never reallocated (see the class doc)
        self.images = torch.zeros(self.MAX_IMAGES * self.image_bytes, dtype=torch.uint8, device=self.device)
        self.pool = []                      # image slots in pool order (oldest first)
        self._next = 0                      # ring position of the next snapshot slot
        self.slots = torch.zeros(max(1, self.pool_size), dtype=torch.int32, device=self.device)
        self._scratch = None
        self._keep = []
        self._users = []  # weak references to the per-table image-slot tensors of the envs playing this pool
        self.refresh()

    def track(self, group_of):
        """Register a per-table opponent tensor (image slot per table): add_snapshot never overwrites
        a slot that one of its tables still plays.  Held weakly: an env that is dropped (or closed,
        untrack) stops reserving its slots."""
        self._users.append(weakref.ref(group_of))

    def untrack(self, group_of):
        """Stop reserving the slots of a tensor registered with track() (DualStepVectorEnv.close)."""
        self._users = [r for r in self._users if r() is not None and r() is not group_of]

    def _in_use(self):
        used = set()
        alive = []
        for r in self._users:
            g = r()
            if g is None:
                continue
            alive.append(r)
            used.update(int(x) for x in self.torch.unique(g).tolist())
        self._users = alive
        return used

    def _grow(self):
        """One more image slot (the ring is full of snapshots still in play); the buffer is already
        allocated at MAX_IMAGES, so nothing moves."""
        if self.n_images >= self.MAX_IMAGES:
            raise RuntimeError(f"OpponentPool: every one of the {self.MAX_IMAGES} image slots is in play; add "
                               "snapshots less often than episodes end")
        self.n_images += 1
        return self.n_images - 1

    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def _pack(self, model, slot):
        keep = []
        actor = _mlp_desc(model.actor, keep)
        ptr_ = self.images.data_ptr() + slot * self.image_bytes
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_policy_pack(ctypes.byref(actor), None, self._prec, ptr_, self._stream()))
        self._keep.append(keep)
        self._keep = self._keep[-8:]

    def refresh(self):
        """Re-pack the current policy (image 0) from the agent's live weights."""
        self._pack(self.agent, 0)

    def add_snapshot(self, model=None):
        """pool.append(snapshot); pool.pop(0) beyond pool_size (ppo_splendor.py:366-370).  `model`
        defaults to the agent (its weights now)."""
        busy = set(self.pool) | self._in_use() | {0}
        ring = self.n_images - 1
        slot = next((1 + (self._next + k) % ring for k in range(ring) if 1 + (self._next + k) % ring not in busy), None)
        if slot is None:
            slot = self._grow()
        self._next = slot % (self.n_images - 1)  # the ring position after `slot`
        self._pack(self.agent if model is None else model, slot)
        self.pool.append(slot)
        if len(self.pool) > self.pool_size:
            self.pool.pop(0)
        if self.pool:
            self.slots[:len(self.pool)].copy_(self.torch.tensor(self.pool, dtype=self.torch.int32))

    def draw(self, group_of, episode, draw_mask=None, table0=0):
        """Choose each (draw_mask-selected) table's opponent for its next episode."""
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_dual_draw_opponents(
                group_of.numel(), ptr(draw_mask), episode.data_ptr(), group_of.data_ptr(), self.slots.data_ptr(),
                len(self.pool), ctypes.c_float(self.p_current), self.seed & (2**64 - 1), int(table0), self._stream()))

    def finish_draw(self, io, group_of, episode, group_prev, table0=0):
        """spl_dual_finish of a dual step (io: a DualIo) fused with draw(group_of, episode,
        io.done): the tables that finished draw their next opponent; group_prev receives each
        table's opponent before the draw.  One launch (include/splendor_dual.h)."""
        d = _native.DualDraw(episode=episode.data_ptr(), group_of=group_of.data_ptr(), group_prev=group_prev.data_ptr(),
                             pool_slots=self.slots.data_ptr(), pool_len=len(self.pool), p_current=self.p_current,
                             seed=self.seed & (2**64 - 1), table0=int(table0))
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_dual_finish_draw(group_of.numel(), ctypes.byref(io), ctypes.byref(d),
                                                          self._stream()))

    def act(self, obs, mask, group_of, out=None):
        """Greedy action of each table's network: int32 [n].  obs: int32 [n, 297], or the compact
        uint8 [n, 300] rows of Engine.step(obs_u8=...)."""
        t = self.torch
        n = obs.shape[0]
        u8 = obs.dtype == t.uint8
        if (obs.dtype not in (t.int32, t.uint8) or obs.shape[1] != (OBS_U8 if u8 else OBS_DIM) or not obs.is_contiguous()
                or mask.dtype != t.int8 or not mask.is_contiguous()):
            raise ValueError("obs int32 [n, 297] (or uint8 [n, 300] compact rows) and mask int8 [n, 45], contiguous")
        # sized for every image the ring can hold, so growing the ring never reallocates it; its layout
        # follows the group count, so a grown ring re-zeroes it once (the counters must start at zero)
        nbytes = int(self.lib.spl_policy_group_scratch_bytes(n, self.MAX_IMAGES))
        if self._scratch is None or self._scratch.numel() < nbytes:  # zero-filled once (spl_policy_act_grouped)
            self._scratch = t.zeros(nbytes, dtype=t.uint8, device=self.device)
            self._scratch_groups = self.n_images
        elif self._scratch_groups != self.n_images:
            self._scratch.zero_()
            self._scratch_groups = self.n_images
        action = out if out is not None else t.empty(n, dtype=t.int32, device=self.device)
        a = ActArgs(obs=None if u8 else obs.data_ptr(), obs_u8=obs.data_ptr() if u8 else None, mask=mask.data_ptr(),
                    action=action.data_ptr(), logprob=None, entropy=None, value=None, logits=None, seed=0, ply=0,
                    ply_base=None, table0=0, mode=ACT_GREEDY, image=self._prec << 1)
        with t.cuda.device(self.device):
            check(self.lib, self.lib.spl_policy_act_grouped(self.images.data_ptr(), self.image_bytes, self.n_images,
                                                            group_of.data_ptr(), self._scratch.data_ptr(), n,
                                                            ctypes.byref(a), self._stream()))
        return action

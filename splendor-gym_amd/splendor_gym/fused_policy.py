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

precision="fp32" (default, the reference's precision): exact fp32 products and accumulation on
v_mfma_f32_16x16x4_f32 — logits and values equal the fp32 module's to summation-order rounding
(tests/test_gpu_policy.py: 1e-5 relative).  precision="bf16" (opt-in): bf16 MFMA with fp32
accumulation, logits to bf16 accuracy.  Call ``refresh()`` after the module's weights change (e.g.
after each PPO update).
"""
import ctypes

from . import _native
from ._native import (ACT_GREEDY, ACT_SAMPLE, IMG_CRITIC, NUM_ACTIONS, OBS_DIM, PREC_BF16, PREC_FP32, ActArgs, MlpDesc,
                      check, ptr)

_PRECISIONS = {"fp32": PREC_FP32, "bf16": PREC_BF16}


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
        if obs.dtype != t.int32 or obs.dim() != 2 or obs.shape[1] != OBS_DIM or not obs.is_contiguous():
            raise ValueError("obs must be a contiguous int32 [n, 297] device tensor")
        if mask.dtype not in (t.int8, t.uint8, t.bool) or tuple(mask.shape) != (obs.shape[0], NUM_ACTIONS) or \
                not mask.is_contiguous():
            raise ValueError("mask must be a contiguous int8 [n, 45] device tensor")
        if obs.device != self.device or mask.device != self.device:
            raise ValueError("obs/mask must be on the policy's device")
        return obs.shape[0]

    def _run(self, obs, mask, mode, action, logprob=None, entropy=None, value=None, logits=None, seed=0, ply=0,
             table0=0, ply_base=None):
        n = self._check_inputs(obs, mask)
        a = ActArgs(obs=obs.data_ptr(), mask=mask.data_ptr(), action=action.data_ptr(), logprob=ptr(logprob),
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

    def opponent(self):
        """A batched opponent for DualStepVectorEnv: (obs, mask) -> int32 actions."""
        return lambda obs, mask: self.greedy(obs, mask)

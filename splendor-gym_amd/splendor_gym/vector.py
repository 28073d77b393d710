"""SplendorVectorEnv: N tables per GPU launch with gymnasium-0.29 SyncVectorEnv semantics.

Replaces the reference's per-env Python loop (ppo_splendor.py:151-159 SyncVectorEnv of
SplendorEnv, stepped one env at a time at :235-269) with one spl_step launch over all tables.
Semantics per table are SplendorEnv.step's; vector conventions follow gymnasium 0.29:

* reset(seed=int) seeds env i with seed + i; reset(seed=None) continues every env's stream.
* same-step autoreset: a terminated table is re-dealt inside the step; the returned obs/mask
  are the new episode's, the terminal ones are in info["final_observation"].
* info values are vectorised with a boolean "_key" companion mask.
* copy=True (gymnasium's default): the arrays a step returns are never written by a later step
  while anything still references them (below).  copy=False returns the same buffers every step.

Outputs stay on the GPU as torch tensors (obs int32 [N,297], mask int8 [N,45], ...) unless
``to_numpy=True``, which returns numpy arrays and gymnasium-style object arrays for
final_observation / final_info (the form SB3/CleanRL code indexes).

One step is one spl_step launch: the kernel writes the observation, mask, reward, terminated, flags,
winner, terminal rows, the info planes (illegal_action / draw / turn_limit / truncated) and the
running error count (include/splendor_amd.h spl_step_args_t.info / .errors).  Each output set is one
device block with its views and its argument block built once; copy=True keeps a small ring of such
blocks and takes a fresh one whenever a block's storage is still referenced outside the env
(torch storage use count), so returned tensors behave like fresh arrays at no per-step copy.
"""
import ctypes
import sys

import numpy as np

from . import _native
from ._gym_compat import spaces
from .device import Engine
from .engine.encode import OBSERVATION_DIM, TOTAL_ACTIONS
from .seeding import vector_seeds


class _OutBlock:
    """One set of step outputs in one device allocation, its tensor views and its spl_step
    argument block (bound to the block's pointers)."""

    _SPECS = (("obs", "int32", (OBSERVATION_DIM,)), ("mask", "int8", (TOTAL_ACTIONS,)), ("reward", "float32", ()),
              ("terminated", "uint8", ()), ("flags", "uint8", ()), ("winner", "int8", ()), ("info", "uint8", (4,)),
              ("final_obs", "int32", (OBSERVATION_DIM,)))

    def __init__(self, torch, n, device, autoreset, table0):
        offs, off = [], 0
        for name, dt, shape in self._SPECS:
            nb = n * int(np.prod(shape, dtype=np.int64)) * np.dtype(dt).itemsize
            offs.append((name, dt, shape, off, nb))
            off = (off + nb + 255) // 256 * 256
        self.raw = torch.zeros(off, dtype=torch.uint8, device=device)
        for name, dt, shape, o, nb in offs:
            v = self.raw[o:o + nb].view(getattr(torch, dt))
            if name == "info":
                v = v.view(4, n)
            elif shape:
                v = v.view(n, *shape)
            setattr(self, name, v)
        del v
        self.term_b = self.terminated.view(torch.bool)
        self.illegal, self.draw, self.turn_limit, self.truncated = self.info.view(torch.bool).unbind(0)
        self.to_play = self.obs[:, 294]
        self.args = _native.StepArgs(obs=self.obs.data_ptr(), mask=self.mask.data_ptr(), reward=self.reward.data_ptr(),
                                     terminated=self.terminated.data_ptr(), flags=self.flags.data_ptr(),
                                     winner=self.winner.data_ptr(),
                                     final_obs=self.final_obs.data_ptr() if autoreset else None,
                                     autoreset=1 if autoreset else 0, table0=table0, info=self.info.data_ptr())
        self.args_ref = ctypes.byref(self.args)
        # what a step hands out; a caller still holding one of these (or a view of the block) keeps
        # the block from being written again
        self.public = (self.obs, self.mask, self.reward, self.term_b, self.truncated, self.to_play, self.illegal,
                       self.draw, self.turn_limit, self.winner, self.final_obs)
        self._use_count = getattr(torch._C, "_storage_Use_Count", None)
        self._cdata = self.raw.untyped_storage()._cdata
        self.base_refs = self._refs()
        self.base_use = self.use_count()

    def _refs(self):
        return tuple(sys.getrefcount(t) for t in self.public)

    def use_count(self):
        return self._use_count(self._cdata) if self._use_count else 0

    def referenced(self):
        """True while a returned tensor object, or any other tensor sharing the block's storage (a
        caller's view or slice), is alive outside this block object."""
        return self._refs() != self.base_refs or self.use_count() != self.base_use


class SplendorVectorEnv:
    metadata = {"render_modes": [], "autoreset_mode": "same-step"}
    RING = 3  # output blocks kept for copy=True (a loop holding one step's results while stepping needs 2)
    # check_actions="deferred": the running error count is copied back after every DEFER_EVERY-th step
    # (a step's error is raised at the latest DEFER_EVERY + DEFER_LAG steps later, or by reset())
    DEFER_EVERY = 4
    DEFER_LAG = 2
    DEFER_RING = 8

    def __init__(self, num_envs, num_players=2, device=None, autoreset=True, refill_period=None, table0=0,
                 to_numpy=False, check_actions="sync", copy=True):
        if check_actions not in ("sync", "deferred"):
            raise ValueError('check_actions must be "sync" or "deferred"')
        # "sync": the reference's exceptions (out-of-range action, step after termination) are raised
        # by the step() that caused them, which reads one count back from the GPU per step when the
        # actions are a device tensor (host actions are range-checked on the host).  "deferred":
        # the count is copied back asynchronously every DEFER_EVERY steps and checked without blocking
        # by later calls; a step's error is raised at the latest DEFER_EVERY * (DEFER_LAG + 1) steps
        # after it (or by reset()), so the host never drains the GPU queue.
        self.check_actions = check_actions
        self.num_envs = int(num_envs)
        self.num_players = int(num_players)
        self.autoreset = bool(autoreset)
        self.to_numpy = bool(to_numpy)
        self.copy = bool(copy)
        self.single_action_space = spaces.Discrete(TOTAL_ACTIONS)
        self.single_observation_space = spaces.Box(low=0, high=50, shape=(OBSERVATION_DIM,), dtype=np.int32)
        self.action_space = spaces.MultiDiscrete(np.full(self.num_envs, TOTAL_ACTIONS))
        self.observation_space = spaces.Box(low=0, high=50, shape=(self.num_envs, OBSERVATION_DIM), dtype=np.int32)
        self.engine = Engine(self.num_envs, self.num_players, device=device, refill_period=refill_period,
                             table0=table0)
        self.device = self.engine.device
        self._seeded = False
        torch = self.engine.torch
        self._torch = torch
        self._errors = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._errors_seen = 0
        self._ring = [self._new_block()]
        self._cur = 0
        self._pending = []  # deferred check: (ring slot, step index) of copies not yet checked
        self._unchecked = 0  # steps since the last error-count copy (deferred) that may carry an error
        self._pin = torch.zeros(self.DEFER_RING, dtype=torch.int64).pin_memory() if check_actions == "deferred" else None
        self._events = [torch.cuda.Event() for _ in range(self.DEFER_RING)] if check_actions == "deferred" else None
        self._steps = 0
        self._qslot = 0  # deferred check: the pinned slot / event the next copy uses (rotating)
        e = self.engine
        self._lib, self._ctx, self._desc = e.lib, e.ctx, ctypes.byref(e.desc)
        self._stream_obj = torch.cuda.current_stream(self.device)
        self._stream = ctypes.c_void_p(self._stream_obj.cuda_stream)

    def _new_block(self):
        b = _OutBlock(self._torch, self.num_envs, self.device, self.autoreset, self.engine.table0)
        b.args.errors = self._errors.data_ptr()
        return b

    @property
    def block(self):
        """The output block of the latest reset/step."""
        return self._ring[self._cur]

    def _next_block(self):
        """The block the next reset/step writes: with copy=True one no returned tensor still uses."""
        if not self.copy:
            return self._ring[0]
        for k in range(1, self.RING + 1):
            i = (self._cur + k) % self.RING
            if i >= len(self._ring):
                self._ring.append(self._new_block())
                self._cur = len(self._ring) - 1
                return self._ring[-1]
            if not self._ring[i].referenced():
                self._cur = i
                return self._ring[i]
        # every block is held by the caller: replace the oldest one with a fresh allocation
        i = (self._cur + 1) % self.RING
        self._ring[i] = self._new_block()
        self._cur = i
        return self._ring[i]

    # ----------------------------------------------------------------------------------------
    def _out(self, t):
        return t.cpu().numpy() if self.to_numpy else t

    def _stream_ptr(self):
        s = self._torch.cuda.current_stream(self.device)
        if s is not self._stream_obj:
            self._stream_obj, self._stream = s, ctypes.c_void_p(s.cuda_stream)
        return self._stream

    def reset(self, *, seed=None, options=None):
        """Reset every table.  This is also the recovery from a faulted launch: a fault seen
        since the last clear (step() raised LaunchFault for it) is cleared once every table has been
        re-dealt, and reported as info["recovered_fault"] = the faulted launch's serial.  The fault word
        is read after the re-deal has been enqueued and the device has drained: a launch
        still in flight at the call that faults later is covered by this reset too, since the re-deal
        follows it in stream order."""
        if self._unchecked and self.check_actions == "deferred":
            self._queue_check()
        self._raise_pending(block_all=True)
        seeds = vector_seeds(seed, self.num_envs)
        if seeds is None and not self._seeded:
            seeds = [None] * self.num_envs  # gymnasium: first reset without a seed draws entropy
        b = self._next_block()
        self.engine.reset(seeds=seeds, obs_out=b.obs, mask_out=b.mask)
        self._seeded = True
        self.engine.torch.cuda.synchronize(self.device)
        fault = self.engine.faults()
        info = {"action_mask": self._out(b.mask), "to_play": self._out(b.to_play)}
        if fault:  # every table was just re-dealt: the undefined state is gone
            self.engine.clear_faults()
            info["recovered_fault"] = fault
        if self.to_numpy:
            info["_action_mask"] = np.ones(self.num_envs, bool)
            info["_to_play"] = np.ones(self.num_envs, bool)
        return self._out(b.obs), info

    def _raise_errors(self, flags):
        """Raise the reference's exception for the first table whose flags carry an error."""
        bad = ((flags & (_native.F_OOB | _native.F_AFTER_TERMINAL)) != 0).nonzero().flatten().tolist()
        f = int(flags[bad[0]].item())
        if f & _native.F_OOB:
            raise ValueError(f"Action out of bounds for action_space (envs {bad[:8]})")
        raise RuntimeError(f"Cannot call step() after episode termination. Call reset(). (envs {bad[:8]})")

    def _queue_check(self):
        """Copy the running error count back asynchronously (deferred mode)."""
        self._unchecked = 0
        if len(self._pending) >= self.DEFER_RING - 1:
            self._raise_pending(block_all=True)
        # a rotating slot: a pending copy's slot is never reused before it is checked
        slot = self._qslot
        self._qslot = (slot + 1) % self.DEFER_RING
        self._pin[slot:slot + 1].copy_(self._errors, non_blocking=True)
        self._events[slot].record(self._stream_obj)
        self._pending.append((slot, self._steps))

    def _raise_pending(self, block_all=False):
        """Deferred check: raise the error of an earlier step once its count has come back (copies
        that have landed are checked without blocking; one DEFER_LAG steps old, or every one when
        block_all, is waited for)."""
        while self._pending:
            slot, step = self._pending[0]
            ev = self._events[slot]
            if not (block_all or self._steps - step >= self.DEFER_LAG * self.DEFER_EVERY or ev.query()):
                break
            ev.synchronize()
            self._pending.pop(0)
            count = int(self._pin[slot])
            if count != self._errors_seen:
                self._errors_seen = count
                self._pending.clear()
                raise ValueError(f"step {step}: an out-of-range action or a step after termination (the reference's "
                                 "ValueError / RuntimeError; check_actions='deferred' reports it a few calls late)")

    def _device_actions(self, actions):
        """(int32 contiguous device tensor, host_checked) for any action container."""
        torch = self._torch
        if isinstance(actions, torch.Tensor):
            if not (actions.device == self.device and actions.dtype == torch.int32 and actions.is_contiguous()):
                actions = actions.to(device=self.device, dtype=torch.int32).contiguous()
            host_checked = False
        else:
            a = np.asarray(actions)
            host_checked = False
            if a.shape == (self.num_envs,) and np.issubdtype(a.dtype, np.integer):
                bad = np.flatnonzero((a < 0) | (a >= TOTAL_ACTIONS))
                if bad.size:  # the kernel would flag these tables OOB
                    raise ValueError(f"Action out of bounds for action_space (envs {bad[:8].tolist()})")
                host_checked = True
            actions = torch.as_tensor(np.ascontiguousarray(a, np.int32)).to(self.device)
        if actions.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions")
        return actions, host_checked

    def step(self, actions):
        """One spl_step launch over every table.  copy=True: the returned tensors stay valid until the
        caller drops them; copy=False: they are the env's buffers, overwritten by the next step.
        Raises LaunchFault when a launch of the engine faulted (host-mapped fault word, no sync)."""
        self.engine.check_faults()
        self._raise_pending()
        a, host_checked = self._device_actions(actions)
        b = self._next_block()
        args = b.args
        args.actions = a.data_ptr()
        _native.check(self._lib, self._lib.spl_step(self._ctx, self._desc, b.args_ref, self._stream_ptr()))
        self._keep_actions = a
        self._steps += 1
        # the step-after-termination error needs autoreset off; out-of-range host actions were caught
        if not (host_checked and self.autoreset):
            self._unchecked += 1
            if self.check_actions == "sync":
                count = int(self._errors.item())
                if count != self._errors_seen:
                    self._errors_seen = count
                    self._raise_errors(b.flags)
            elif self._unchecked >= self.DEFER_EVERY:
                self._queue_check()
        info = {
            "action_mask": b.mask,
            "to_play": b.to_play,
            "illegal_action": b.illegal,
            "draw": b.draw,
            "turn_limit": b.turn_limit,
            "winner": b.winner,
        }
        if self.autoreset:
            info["final_observation"] = b.final_obs
            info["_final_observation"] = b.term_b
        if not self.to_numpy:
            return b.obs, b.reward, b.term_b, b.truncated, info
        return self._numpy_step(b.obs, b.reward, b.term_b, b.truncated, info)

    @property
    def last_flags(self):
        """SPL_F_* bits of the latest step, one byte per table (device tensor)."""
        return self.block.flags

    def _numpy_step(self, obs, reward, terminated, truncated, info):
        n = self.num_envs
        term = terminated.cpu().numpy()
        out = {"action_mask": info["action_mask"].cpu().numpy(), "_action_mask": np.ones(n, bool),
               "to_play": info["to_play"].cpu().numpy(), "_to_play": np.ones(n, bool)}
        for key in ("illegal_action", "draw", "turn_limit"):
            v = info[key].cpu().numpy()
            out[key], out["_" + key] = v, v.copy()
        if self.autoreset and term.any():
            fobs = info["final_observation"].cpu().numpy()
            win = info["winner"].cpu().numpy()
            tl = out["turn_limit"]
            fo = np.empty(n, dtype=object)
            fi = np.empty(n, dtype=object)
            for i in np.flatnonzero(term):
                fo[i] = fobs[i].copy()
                w = int(win[i])
                fr = ({p: (-0.1 if tl[i] else 0.0) for p in range(self.num_players)} if w < 0 else
                      {p: (1.0 if p == w else -1.0) for p in range(self.num_players)})
                d = {"to_play": 0, "final_rewards": fr}
                if tl[i]:
                    d["turn_limit"] = True
                if out["draw"][i]:
                    d["draw"] = True
                fi[i] = d
            out["final_observation"], out["_final_observation"] = fo, term.copy()
            out["final_info"], out["_final_info"] = fi, term.copy()
        return obs.cpu().numpy(), reward.cpu().numpy(), term, truncated.cpu().numpy(), out

    def sample_actions(self, seed=0, ply=0):
        """Uniform-random legal action per env over the current masks, drawn on the device
        (random_opponent)."""
        return self.engine.sample_uniform(mask=self.block.mask, seed=seed, ply=ply)

    def close(self):
        self.engine.close()

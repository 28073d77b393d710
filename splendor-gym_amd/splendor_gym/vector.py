"""SplendorVectorEnv: N tables per GPU launch with gymnasium-0.29 SyncVectorEnv semantics.

Replaces the reference's per-env Python loop (ppo_splendor.py:151-159 SyncVectorEnv of
SplendorEnv, stepped one env at a time at :235-269) with one spl_step launch over all tables.
Semantics per table are SplendorEnv.step's; vector conventions follow gymnasium 0.29:

* reset(seed=int) seeds env i with seed + i; reset(seed=None) continues every env's stream.
* same-step autoreset: a terminated table is re-dealt inside the step; the returned obs/mask
  are the new episode's, the terminal ones are in info["final_observation"].
* info values are vectorised with a boolean "_key" companion mask.

Outputs stay on the GPU as torch tensors (obs int32 [N,297], mask int8 [N,45], ...) unless
``to_numpy=True``, which returns numpy arrays and gymnasium-style object arrays for
final_observation / final_info (the form SB3/CleanRL code indexes).
"""
import numpy as np

from . import _native
from ._gym_compat import spaces
from .device import Engine
from .engine.encode import OBSERVATION_DIM, TOTAL_ACTIONS
from .seeding import vector_seeds


class SplendorVectorEnv:
    metadata = {"render_modes": [], "autoreset_mode": "same-step"}

    def __init__(self, num_envs, num_players=2, device=None, autoreset=True, refill_period=None, table0=0,
                 to_numpy=False, check_actions="sync"):
        if check_actions not in ("sync", "deferred"):
            raise ValueError('check_actions must be "sync" or "deferred"')
        # "sync": the reference's exceptions (out-of-range action, step after termination) are raised
        # by the step() that caused them, which reads one flag back from the GPU per step when the
        # actions are a device tensor (host actions are range-checked on the host).  "deferred":
        # the same check is read back asynchronously and raised by the NEXT step()/reset() call, so
        # the host never waits for the step kernel.
        self.check_actions = check_actions
        self.num_envs = int(num_envs)
        self.num_players = int(num_players)
        self.autoreset = bool(autoreset)
        self.to_numpy = bool(to_numpy)
        self.single_action_space = spaces.Discrete(TOTAL_ACTIONS)
        self.single_observation_space = spaces.Box(low=0, high=50, shape=(OBSERVATION_DIM,), dtype=np.int32)
        self.action_space = spaces.MultiDiscrete(np.full(self.num_envs, TOTAL_ACTIONS))
        self.observation_space = spaces.Box(low=0, high=50, shape=(self.num_envs, OBSERVATION_DIM), dtype=np.int32)
        self.engine = Engine(self.num_envs, self.num_players, device=device, refill_period=refill_period,
                             table0=table0)
        self.device = self.engine.device
        self._seeded = False
        torch = self.engine.torch
        # info["illegal_action"], ["draw"], ["turn_limit"] planes and a running count of the tables
        # whose flags carry an error, both written by one spl_step_info launch per step
        self._info = torch.zeros((3, self.num_envs), dtype=torch.uint8, device=self.device)
        self._info_b = self._info.view(torch.bool)
        self._errors = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._errors_seen = 0
        self._truncated = torch.zeros(self.num_envs, dtype=torch.bool, device=self.device)
        self._pending = None  # deferred check: (pinned count, event, step index)
        self._steps = 0

    # ----------------------------------------------------------------------------------------
    def _out(self, t):
        return t.cpu().numpy() if self.to_numpy else t

    def reset(self, *, seed=None, options=None):
        self._raise_pending()
        seeds = vector_seeds(seed, self.num_envs)
        if seeds is None and not self._seeded:
            seeds = [None] * self.num_envs  # gymnasium: first reset without a seed draws entropy
        obs, mask = self.engine.reset(seeds=seeds)
        self._seeded = True
        info = {"action_mask": self._out(mask), "to_play": self._out(obs[:, 294])}
        if self.to_numpy:
            info["_action_mask"] = np.ones(self.num_envs, bool)
            info["_to_play"] = np.ones(self.num_envs, bool)
        return self._out(obs), info

    def _raise_errors(self, flags):
        """Raise the reference's exception for the first table whose flags carry an error."""
        bad = ((flags & (_native.F_OOB | _native.F_AFTER_TERMINAL)) != 0).nonzero().flatten().tolist()
        f = int(flags[bad[0]].item())
        if f & _native.F_OOB:
            raise ValueError(f"Action out of bounds for action_space (envs {bad[:8]})")
        raise RuntimeError(f"Cannot call step() after episode termination. Call reset(). (envs {bad[:8]})")

    def _raise_pending(self):
        """Deferred check: raise the error of an earlier step once its count has come back."""
        if self._pending is None:
            return
        count, event, step = self._pending
        self._pending = None
        event.synchronize()
        if int(count.item()) != self._errors_seen:
            self._errors_seen = int(count.item())
            raise ValueError(f"step {step}: an out-of-range action or a step after termination (the "
                             f"reference's ValueError / RuntimeError; check_actions='deferred' reports it one call late)")

    def step(self, actions):
        """Returned tensors are the env's per-step buffers (overwritten by the next step), as the
        observation always is; copy what must outlive the step."""
        e = self.engine
        torch = e.torch
        self._raise_pending()
        host_checked = False
        if not isinstance(actions, torch.Tensor):
            a = np.asarray(actions)
            if a.shape == (self.num_envs,) and np.issubdtype(a.dtype, np.integer):
                bad = np.flatnonzero((a < 0) | (a >= TOTAL_ACTIONS))
                if bad.size:  # the kernel would flag these tables OOB
                    raise ValueError(f"Action out of bounds for action_space (envs {bad[:8].tolist()})")
                host_checked = True
        obs, mask, reward, term, flags = e.step(actions, autoreset=self.autoreset, final_obs=True)
        self._steps += 1
        _native.check(e.lib, e.lib.spl_step_info(self.num_envs, flags.data_ptr(), self._info.data_ptr(),
                                                 self._errors.data_ptr(), e.stream()))
        # the step-after-termination error needs autoreset off; out-of-range host actions were caught
        if not (host_checked and self.autoreset):
            if self.check_actions == "sync":
                count = int(self._errors.item())
                if count != self._errors_seen:
                    self._errors_seen = count
                    self._raise_errors(flags)
            else:
                count = torch.empty(1, dtype=torch.int64, pin_memory=True)
                count.copy_(self._errors, non_blocking=True)
                event = torch.cuda.Event()
                event.record(torch.cuda.current_stream(self.device))
                self._pending = (count, event, self._steps)
        terminated = term.view(torch.bool)  # 0/1 bytes
        info = {
            "action_mask": mask,
            "to_play": obs[:, 294],
            "illegal_action": self._info_b[0],
            "draw": self._info_b[1],
            "turn_limit": self._info_b[2],
            "winner": e.winner,
        }
        if self.autoreset:
            info["final_observation"] = e.final_obs
            info["_final_observation"] = terminated
        if not self.to_numpy:
            return obs, reward, terminated, self._truncated, info
        return self._numpy_step(obs, reward, terminated, self._truncated, info)

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
        """Uniform-random legal action per env, drawn on the device (random_opponent)."""
        return self.engine.sample_uniform(seed=seed, ply=ply)

    def close(self):
        self.engine.close()

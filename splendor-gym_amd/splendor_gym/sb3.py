"""stable-baselines3 VecEnv surface over SplendorVectorEnv (BASELINE.json north_star: "the SB3/CleanRL
vector-env API stay drop-in").

SB3 drives environments through ``VecEnv`` (stable_baselines3/common/vec_env/base_vec_env.py); its
``DummyVecEnv`` steps one gymnasium env per index and, when an env is done, stores the terminal
observation in ``infos[i]["terminal_observation"]``, sets ``infos[i]["TimeLimit.truncated"]``, resets
that env and keeps the reset info in ``reset_infos[i]``.  ``SplendorSB3VecEnv`` gives the same
results for N Splendor tables stepped by ONE spl_step launch:

* ``reset()`` -> obs ndarray int32 [N, 297]; ``seed(s)`` makes the next reset seed env i with s + i
  (as SB3 does; the reference's ``reset(seed=)`` per env).
* ``step_async(actions)`` / ``step_wait()`` -> (obs, rewards float32 [N], dones bool [N], infos).
  ``infos[i]`` is the dict the reference ``SplendorEnv.step`` returns for env i
  (envs/splendor_env.py:51-90: action_mask, to_play, illegal_action / draw / turn_limit /
  final_rewards as they apply) plus SB3's ``TimeLimit.truncated`` and, for done envs,
  ``terminal_observation``; the returned obs row of a done env is the next episode's first
  observation and its reset info is ``reset_infos[i]``.
* ``get_attr`` / ``set_attr`` / ``env_method`` / ``env_is_wrapped`` per index; ``env_method("action_masks")``
  serves sb3-contrib's MaskablePPO (``get_action_masks``).

``infos`` is a lazy sequence: env i's dict is built on first access (SB3 indexes ``infos[idx]`` for
done envs; building 65 536 dicts per step would cost more than the step).  The step path stays one
kernel launch plus one pinned device->host copy of the step's outputs.

stable-baselines3 is not installed in this image: when it is importable the class derives from its
``VecEnv``; otherwise from a local base with the same helper methods.  The adapter's semantics are
pinned against a DummyVecEnv-style loop over reference-semantics single envs
(tests/test_sb3_vecenv.py), not against SB3 itself ("parity unpinned" against the library).
"""
from collections.abc import Sequence

import numpy as np

try:  # pragma: no cover - depends on the environment
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase
    HAVE_SB3 = True
except ImportError:  # a stand-in with VecEnv's concrete helpers (SB3 2.x base_vec_env.py)
    HAVE_SB3 = False

    class _VecEnvBase:
        def __init__(self, num_envs, observation_space, action_space):
            self.num_envs = num_envs
            self.observation_space = observation_space
            self.action_space = action_space
            self.reset_infos = [{} for _ in range(num_envs)]
            self._seeds = [None for _ in range(num_envs)]
            self._options = [{} for _ in range(num_envs)]
            self.render_mode = None
            self.metadata = {"render_modes": ["human"]}
            self.closed = False

        def step(self, actions):
            self.step_async(actions)
            return self.step_wait()

        def seed(self, seed=None):
            if seed is None:
                seed = int(np.random.randint(0, np.iinfo(np.uint32).max, dtype=np.uint32))
            self._seeds = [seed + idx for idx in range(self.num_envs)]
            return self._seeds

        def set_options(self, options=None):
            self._options = (options if isinstance(options, list) else [options or {}] * self.num_envs)

        def _reset_seeds(self):
            self._seeds = [None for _ in range(self.num_envs)]

        def _reset_options(self):
            self._options = [{} for _ in range(self.num_envs)]

        def _get_indices(self, indices):
            if indices is None:
                return range(self.num_envs)
            if isinstance(indices, int):
                return [indices]
            return indices

        def get_images(self):
            return [None for _ in range(self.num_envs)]

        def render(self, mode=None):
            return None

        @property
        def unwrapped(self):
            return self

        def getattr_depth_check(self, name, already_found):
            return None


def _np(x):
    """A torch tensor (any device) or array-like as a numpy array."""
    if hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class _LazyInfos(Sequence):
    """list-of-dicts interface; env i's dict is built by `build(i)` on first access and kept."""

    def __init__(self, n, build):
        self._n, self._build, self._cache = n, build, {}

    def __len__(self):
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        i = int(i)
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        d = self._cache.get(i)
        if d is None:
            d = self._cache[i] = self._build(i)
        return d

    def __repr__(self):
        return f"<{self._n} SB3 info dicts, {len(self._cache)} built>"


class SplendorSB3VecEnv(_VecEnvBase):
    """`num_envs` Splendor tables as an SB3 VecEnv (see the module docstring).

    venv: an existing SplendorVectorEnv-like object (autoreset on, torch or numpy outputs) to wrap;
          by default one is created with `num_envs`, `num_players` and `device`.
    """

    def __init__(self, num_envs=None, num_players=2, device=None, venv=None, render_mode=None):
        if venv is None:
            from .vector import SplendorVectorEnv
            venv = SplendorVectorEnv(int(num_envs), num_players, device=device, autoreset=True, copy=False)
        if not getattr(venv, "autoreset", True):
            raise ValueError("SplendorSB3VecEnv needs a same-step autoreset vector env")
        self.venv = venv
        self.num_players = int(getattr(venv, "num_players", num_players))
        super().__init__(venv.num_envs, venv.single_observation_space, venv.single_action_space)
        self.render_mode = render_mode
        self._actions = None
        self._attrs = [dict() for _ in range(self.num_envs)]  # set_attr values of names the envs lack
        self._last = None  # (obs, mask) numpy of the current observations (action_masks, to_play)

    # --- reset / step ------------------------------------------------------------------------------
    def reset(self):
        seeds = self._seeds
        if all(s is None for s in seeds):
            obs, info = self.venv.reset(seed=None)
        else:
            if any(s is None for s in seeds) or any(s != seeds[0] + i for i, s in enumerate(seeds)):
                raise ValueError("SplendorSB3VecEnv.seed(): per-env seeds must be seed + index (VecEnv.seed)")
            obs, info = self.venv.reset(seed=int(seeds[0]))
        self._reset_seeds()
        self._reset_options()
        obs = _np(obs)
        mask = _np(info["action_mask"])
        self._last = (obs, mask)
        self.reset_infos = [{"action_mask": mask[i].copy(), "to_play": int(obs[i, 294])} for i in range(self.num_envs)]
        return obs

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        if self._actions is None:
            raise RuntimeError("step_wait() without step_async()")
        actions, self._actions = self._actions, None
        obs, rew, term, trunc, info = self.venv.step(actions)
        obs, mask = _np(obs), _np(info["action_mask"])
        rew = _np(rew).astype(np.float32, copy=False)
        term = _np(term).astype(bool, copy=False)
        trunc = _np(trunc).astype(bool, copy=False)
        dones = term | trunc
        flags = {k: _np(info[k]).astype(bool, copy=False) for k in ("illegal_action", "draw", "turn_limit")}
        done_idx = np.flatnonzero(dones)
        final = {}
        winner = None
        if done_idx.size:
            fo = info["final_observation"]
            if hasattr(fo, "index_select"):  # device rows of the done envs only
                import torch
                rows = fo.index_select(0, torch.as_tensor(done_idx, device=fo.device)).cpu().numpy()
            else:
                fo = np.asarray(fo)
                rows = np.stack([np.asarray(fo[i]) for i in done_idx]) if fo.dtype == object else fo[done_idx]
            final = {int(i): rows[k] for k, i in enumerate(done_idx)}
            winner = _np(info["winner"])
            for i in done_idx:  # SB3 DummyVecEnv: the reset info of an auto-reset env
                self.reset_infos[i] = {"action_mask": mask[i].copy(), "to_play": int(obs[i, 294])}
        self._last = (obs, mask)
        n_act = int(getattr(self.action_space, "n", 45))
        P = self.num_players

        def build(i):
            if i in final:
                fob = final[i]
                d = {"action_mask": np.zeros(n_act, np.int8), "to_play": int(fob[294])}
                if flags["draw"][i]:
                    d["draw"] = True
                else:
                    if flags["turn_limit"][i]:
                        d["turn_limit"] = True
                    w = int(winner[i])
                    d["final_rewards"] = ({p: (-0.1 if flags["turn_limit"][i] else 0.0) for p in range(P)} if w < 0
                                          else {p: (1.0 if p == w else -1.0) for p in range(P)})
                d["TimeLimit.truncated"] = bool(trunc[i] and not term[i])
                d["terminal_observation"] = fob
                return d
            d = {"action_mask": mask[i].copy(), "to_play": int(obs[i, 294])}
            if flags["illegal_action"][i]:
                d = {"illegal_action": True, **d}
            d["TimeLimit.truncated"] = False
            return d

        return obs, rew, dones, _LazyInfos(self.num_envs, build)

    def close(self):
        if not getattr(self, "closed", False):
            self.venv.close()
            self.closed = True

    # --- per-env access ----------------------------------------------------------------------------
    _SHARED = ("num_players", "render_mode", "metadata", "observation_space", "action_space", "spec")

    def get_attr(self, attr_name, indices=None):
        idx = self._get_indices(indices)
        if attr_name in ("observation_space", "action_space"):
            return [getattr(self.venv, "single_" + attr_name)] * len(idx)
        if attr_name == "render_mode":
            return [self._attrs[i].get("render_mode", self.render_mode) for i in idx]
        if attr_name == "num_players":
            return [self.num_players] * len(idx)
        if attr_name == "metadata":
            return [{"render_modes": ["human"], "name": "Splendor-v0"}] * len(idx)
        if attr_name == "spec":
            return [None] * len(idx)
        if attr_name in ("current_player", "to_play"):
            return [int(self._last[0][i, 294]) for i in idx]
        if attr_name == "state":  # host views of the device tables (engine/state.py)
            from .engine.state import SplendorState
            eng = self.venv.engine
            return [SplendorState.from_record(eng.download(int(i), 1)[0]) for i in idx]
        if all(attr_name in self._attrs[i] for i in idx):
            return [self._attrs[i][attr_name] for i in idx]
        raise AttributeError(f"SplendorEnv has no attribute {attr_name!r}")

    def set_attr(self, attr_name, value, indices=None):
        for i in self._get_indices(indices):
            self._attrs[i][attr_name] = value

    def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
        idx = self._get_indices(indices)
        if method_name == "action_masks":  # sb3-contrib MaskablePPO (common/maskable/utils.py)
            return [self._last[1][i].astype(bool) for i in idx]
        if method_name == "get_final_rewards":  # envs/splendor_env.py:92-115: only on a terminal state
            raise RuntimeError("Cannot get final rewards for non-terminal state (tables are auto-reset; the final "
                               "rewards of an ended episode are in its step's info['final_rewards'])")
        if method_name == "render":
            from .scripts.game_logger import SplendorGameLogger
            states = self.get_attr("state", idx)
            for s in states:
                print(SplendorGameLogger().format_game_state(s))
            return [None] * len(idx)
        raise AttributeError(f"SplendorEnv has no method {method_name!r} reachable through env_method")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._get_indices(indices))

    def action_masks(self):
        """[N, 45] bool legal-action masks of the current observations (MaskablePPO's VecEnv hook)."""
        return self._last[1].astype(bool)

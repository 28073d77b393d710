"""Test double: the reference SplendorEnv surface (reset/step/state/info keys/exceptions,
envs/splendor_env.py:41-115) computed by the CPU oracle, so host-side wrappers can be checked
against the reference's fixtures without a GPU.  Test infrastructure only."""
import numpy as np

from oracle.oracle import PCG, Oracle, OracleVec, mask_bits_to_int8, pcg_state_of, view_to_table

F_ILLEGAL, F_DRAW, F_TURN_LIMIT, F_AFTER_TERMINAL, F_OOB = 0x01, 0x02, 0x04, 0x08, 0x10




class OracleSplendorEnv:
    _orc = None

    def __init__(self, num_players=2):
        if OracleSplendorEnv._orc is None:
            OracleSplendorEnv._orc = Oracle()
        self.o, self.P = OracleSplendorEnv._orc, num_players
        self.view, self._pcg = None, None

    @property
    def state(self):
        """Reference-shaped snapshot (this package's host view type) of the oracle table."""
        from splendor_gym.engine.state import SplendorState
        return None if self.view is None else SplendorState.from_record(view_to_table(self.view))

    def close(self):
        pass

    def reset(self, *, seed=None, options=None):
        import ctypes
        if seed is not None or self._pcg is None:
            self._pcg = PCG(*pcg_state_of(seed), 0, 0)
        engine_seed = self.o.L.orc_engine_seed(ctypes.byref(self._pcg))
        self.view = self.o.initial_state(self.P, engine_seed)
        obs = self.o.encode(self.view)
        return obs, {"action_mask": mask_bits_to_int8(self.o.legal(self.view)), "to_play": int(obs[294])}

    def step(self, action):
        r = self.o.env_step(self.view, int(action))
        if r["error"] & F_AFTER_TERMINAL:
            raise RuntimeError("Cannot call step() after episode termination. Call reset().")
        if r["error"] & F_OOB:
            raise ValueError("Action out of bounds for action_space")
        self.view = r["after"]
        obs, to_play = r["obs"], int(r["obs"][294])
        if r["flags"] & F_DRAW:
            return obs, 0.0, True, False, {"action_mask": np.zeros(45, np.int8), "to_play": to_play, "draw": True}
        if r["flags"] & F_ILLEGAL:
            return obs, -0.01, False, False, {"illegal_action": True, "action_mask": mask_bits_to_int8(r["mask"]),
                                              "to_play": to_play}
        info = {"action_mask": mask_bits_to_int8(r["mask"]), "to_play": to_play}
        if r["terminated"]:
            if r["flags"] & F_TURN_LIMIT:
                info["turn_limit"] = True
            info["final_rewards"] = {p: float(v) for p, v in enumerate(r["final_rewards"])}
        return obs, float(np.float32(r["reward"])), bool(r["terminated"]), False, info


class OracleVectorEnv:
    """Test double of SplendorVectorEnv (same-step autoreset, numpy outputs, the info keys the
    vector env returns), computed by the CPU oracle's batched env (OracleVec)."""

    def __init__(self, num_envs, num_players=2):
        from splendor_gym._gym_compat import spaces
        if OracleSplendorEnv._orc is None:
            OracleSplendorEnv._orc = Oracle()
        self.o, self.num_envs, self.num_players, self.autoreset = OracleSplendorEnv._orc, num_envs, num_players, True
        self.single_action_space = spaces.Discrete(45)
        self.single_observation_space = spaces.Box(low=0, high=50, shape=(297,), dtype=np.int32)
        self.vec = None
        self.closed = False

    def reset(self, *, seed=None, options=None):
        if seed is None and self.vec is None:
            raise ValueError("the oracle double needs a seed for its first reset")
        if seed is not None:
            self.vec = OracleVec(self.o, self.num_envs, self.num_players, [seed + i for i in range(self.num_envs)])
        else:  # continue every env's stream: one autoreset-free reset is not modelled by the double
            raise NotImplementedError
        return self.vec.obs.copy(), {"action_mask": mask_bits_to_int8(self.vec.mask), "to_play": self.vec.obs[:, 294]}

    def step(self, actions):
        r = self.vec.step(np.asarray(actions, np.int32), want_final=True)
        fl = r["flags"]
        if (fl & (F_OOB | F_AFTER_TERMINAL)).any():
            raise ValueError("out-of-range action or step after termination")
        term = r["terminated"].astype(bool)
        info = {"action_mask": mask_bits_to_int8(r["mask"]), "to_play": r["obs"][:, 294],
                "illegal_action": (fl & F_ILLEGAL) != 0, "draw": (fl & F_DRAW) != 0,
                "turn_limit": (fl & F_TURN_LIMIT) != 0, "winner": r["winner"],
                "final_observation": r["final_obs"], "_final_observation": term}
        return r["obs"], r["reward"], term, np.zeros(self.num_envs, bool), info

    def close(self):
        self.closed = True

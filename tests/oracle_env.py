"""Test double: the reference SplendorEnv surface (reset/step/state/info keys/exceptions,
envs/splendor_env.py:41-115) computed by the CPU oracle, so host-side wrappers can be checked
against the reference's fixtures without a GPU.  Test infrastructure only."""
import numpy as np

from oracle.oracle import PCG, Oracle, mask_bits_to_int8, pcg_state_of, view_to_table

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

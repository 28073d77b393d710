"""SplendorEnv: the reference's single-table Gymnasium env, stepped by the HIP engine.

Drop-in for reference splendor_gym/envs/splendor_env.py:23-130 — same constructor, spaces, info
keys, reward values and exceptions.  The table lives on the GPU (an Engine of one table,
autoreset off); each call launches the step kernel, which reads the action from and writes its ~1.3 KB
of outputs to pinned host memory (Engine(host_io=True)), and waits for it.
For throughput use SplendorVectorEnv (thousands of tables per launch).
"""
from typing import Any, Dict, Optional, Tuple

import numpy as np

from .. import _native
from .._gym_compat import Env, spaces
from ..engine.encode import OBSERVATION_DIM, TOTAL_ACTIONS
from ..engine.state import SplendorState


class SplendorEnv(Env):
    metadata = {"render_modes": ["human"], "name": "Splendor-v0"}

    def __init__(self, num_players: int = 2, render_mode: Optional[str] = None, seed: Optional[int] = None,
                 device=None):
        super().__init__()
        if num_players != 2:  # reference envs/splendor_env.py:28-29
            raise NotImplementedError("Current env supports 2 players only.")
        self.num_players = num_players
        self.render_mode = render_mode
        self.action_space = spaces.Discrete(TOTAL_ACTIONS)
        self.observation_space = spaces.Box(low=0, high=50, shape=(OBSERVATION_DIM,), dtype=np.int32)
        self.current_player = 0
        self._device = device
        self._eng = None
        self._view = None        # host view handed out by .state (write-through, see `state`)
        self._view_rec = None    # its record bytes when handed out
        self._seeded = False
        self._terminal = False
        self._cards = {}
        _native.load_library()  # fail loudly at construction if the HIP engine is missing
        _native.require_gpu()

    # --------------------------------------------------------------------------------------
    def _engine(self):
        if self._eng is None:
            from ..device import Engine
            e = Engine(1, self.num_players, device=self._device, refill_period=0, host_io=True)
            base = e.io.data_ptr()
            if e.host_io:  # the pinned I/O block the kernels read and write
                h, self._push, self._pull = e.io.numpy(), None, None
            else:          # pinned memory not mapped at its own address: device block + copies per call
                hb = e.torch.zeros(e.io.numel(), dtype=e.torch.uint8)
                h = hb.numpy()
                a0, a1 = e.actions.data_ptr() - base, e.actions.data_ptr() - base + 4
                self._push = lambda: e.io[a0:a1].copy_(hb[a0:a1])
                self._pull = lambda: hb[:e.io_step_bytes].copy_(e.io[:e.io_step_bytes])

            def view(t, dt, count):
                return np.frombuffer(h, dtype=dt, count=count, offset=t.data_ptr() - base)
            self._v = dict(actions=view(e.actions, np.int32, 1), obs=view(e.obs, np.int32, OBSERVATION_DIM),
                           mask=view(e.mask, np.int8, TOTAL_ACTIONS), reward=view(e.reward, np.float32, 1),
                           terminated=view(e.terminated, np.uint8, 1), flags=view(e.flags, np.uint8, 1),
                           winner=view(e.winner, np.int8, 1))
            self._launch = e.host_stepper()
            self._eng = e
        return self._eng

    def _fetch(self):
        """This table's step outputs (obs, mask, reward, flags, ...), written by the kernel straight
        into the pinned I/O block: wait for the launch, then read them."""
        e, v = self._eng, self._v
        e.torch.cuda.current_stream(e.device).synchronize()
        if self._pull is not None:
            self._pull()
        self._out = dict(reward=float(v["reward"][0]), terminated=int(v["terminated"][0]), flags=int(v["flags"][0]),
                         winner=int(v["winner"][0]))
        return v["obs"].copy(), v["mask"].copy()

    def reset(self, *, seed: Optional[int] = None, options: Optional[Dict[str, Any]] = None):
        super().reset(seed=seed)
        eng = self._engine()
        # a new game deals fresh, canonical cards (state.py:183-184): drop the previous episode's
        # edited card table BEFORE the reset kernel encodes the first obs and mask from it
        self._cards = {}
        eng.set_card_table(None)
        if seed is not None or not self._seeded:  # gymnasium: reseed, or first reset from entropy
            eng.reset(seeds=[seed])
            self._seeded = True
        else:                                     # continue this env's np_random stream
            eng.reset(seeds=None)
        self._view = None
        obs, mask = self._fetch()
        self._terminal = False
        self.current_player = int(obs[294])
        return obs, {"action_mask": mask, "to_play": int(obs[294])}

    def step(self, action) -> Tuple[np.ndarray, float, bool, bool, Dict[str, Any]]:
        if self._eng is None:
            raise AssertionError("Call reset() first")
        e = self._eng
        try:
            a = int(action)
        except (TypeError, ValueError):
            raise ValueError("Action out of bounds for action_space")
        a = max(min(a, 2**31 - 1), -(2**31))
        self._flush_view()
        self._v["actions"][0] = a  # read by the kernel from pinned memory (no kernel is in flight here)
        if self._push is not None:
            self._push()
        self._launch()              # = e.step(e.actions, autoreset=False)
        self._view = None
        obs, mask = self._fetch()
        o = self._out
        flags = o["flags"]
        if flags & _native.F_AFTER_TERMINAL:  # envs/splendor_env.py:53-54
            raise RuntimeError("Cannot call step() after episode termination. Call reset().")
        if flags & _native.F_OOB:             # :62-63
            raise ValueError("Action out of bounds for action_space")
        to_play = int(obs[294])
        self.current_player = to_play
        if flags & _native.F_DRAW:            # :56-61
            self._terminal = True
            return obs, 0.0, True, False, {"action_mask": np.zeros(TOTAL_ACTIONS, dtype=np.int8),
                                           "to_play": to_play, "draw": True}
        if flags & _native.F_ILLEGAL:         # :64-66
            return obs, -0.01, False, False, {"illegal_action": True, "action_mask": mask, "to_play": to_play}
        reward = o["reward"]
        terminated = bool(o["terminated"])
        info = {"action_mask": mask, "to_play": to_play}
        if terminated:
            self._terminal = True
            if flags & _native.F_TURN_LIMIT:
                info["turn_limit"] = True
            info["final_rewards"] = self._final_rewards(o["winner"], bool(flags & _native.F_TURN_LIMIT))
        return obs, reward, terminated, False, info

    def _final_rewards(self, w, turn_limit):
        # envs/splendor_env.py:92-115
        if w < 0:
            return {p: (-0.1 if turn_limit else 0.0) for p in range(self.num_players)}
        return {p: (1.0 if p == w else -1.0) for p in range(self.num_players)}

    def get_final_rewards(self) -> Dict[int, float]:
        s = self.state
        if not (s.game_over and s.to_play == 0):
            raise RuntimeError("Cannot get final rewards for non-terminal state")
        return self._final_rewards(-1 if s.winner_index is None else s.winner_index, s.turn_limit_reached)

    # ---- host view of the device table ---------------------------------------------------
    @property
    def state(self) -> Optional[SplendorState]:
        """The table as a reference-shaped SplendorState, WRITE-THROUGH: the same object is returned
        until the next step/reset, and in-place edits of it (bank, players, board, decks, nobles,
        counters — tests/utils.py:25-53 style) are uploaded to the device before the next step,
        legal_mask() or render().  Card/noble data itself is the constant device table."""
        if self._eng is None:
            return None
        if self._view is None:
            self._view = SplendorState.from_record(self._eng.download(0, 1)[0], cards=self._cards)
            self._view_rec = self._view.to_record().tobytes()
        return self._view

    def cached_to_play(self) -> Optional[int]:
        """state.to_play without a device download (None before reset): from an outstanding
        write-through view if one was handed out, else from the last observation (obs[294])."""
        if self._eng is None:
            return None
        if self._view is not None:
            return int(self._view.to_play)
        return int(self.current_player)

    def _flush_view(self):
        """Upload host edits of the view handed out by `state` (no-op when unchanged).  Edited card
        fields (card.cost = ...) switch the env to a context built from the state's card table for
        the rest of the episode (the edited Card object stays in every later view)."""
        if self._view is None:
            return
        rec = self._view.to_record()
        if rec.tobytes() != self._view_rec:
            self._eng.upload(rec)
            self._view_rec = rec.tobytes()
        self._cards.update(self._view.cards())
        self._eng.set_card_table(self._view.card_table())

    def set_state(self, state: SplendorState) -> None:
        """Replace the device table by `state` (also what in-place edits of .state do implicitly)."""
        eng = self._engine()
        eng.upload(state.to_record())
        self._cards = dict(state.cards())
        eng.set_card_table(state.card_table())
        self._view = None
        self.current_player = int(state.to_play)

    def legal_mask(self) -> np.ndarray:
        """engine legal_moves(self.state) as int8[45], computed on the device (rules.py:40-93)."""
        e = self._engine()
        self._flush_view()
        e.legal()
        e.torch.cuda.current_stream(e.device).synchronize()  # the mask lands in the pinned I/O block
        return e.mask[0].cpu().numpy().copy()

    def render(self):
        """Print the reference logger's compact text of the table (envs/splendor_env.py:119-126)."""
        if self.render_mode not in ("human", None):
            return
        assert self.state is not None
        self._flush_view()
        from ..scripts.game_logger import SplendorGameLogger
        print(SplendorGameLogger().format_game_state(self.state))


def make(num_players: int = 2, render_mode: Optional[str] = None, seed: Optional[int] = None) -> SplendorEnv:
    return SplendorEnv(num_players=num_players, render_mode=render_mode, seed=seed)

"""The reference's functional engine API (splendor_gym/engine/__init__.py:1-13, engine/rules.py:33-312)
on host views, evaluated by the HIP engine.

    initial_state(num_players, seed)  rules.py:33-34 / state.py:181-211  -> spl_deal
    legal_moves(state)                rules.py:40-93                      -> spl_legal
    apply_action(state, action)       rules.py:196-287                    -> spl_step (no autoreset)
    encode_observation(state)         encode.py:124-187                   -> spl_encode
    compute_winner / is_terminal / winner   rules.py:290-312 (field reads on the view)

Each call uploads the view into a one-table scratch arena on the current GPU, launches the kernel
and downloads the result (synchronous; for debugging, logging and crafted-state tests — the
batched Engine / SplendorVectorEnv are the throughput paths).  There is no CPU fallback.

Cards edited in place (``state.board[1][0].cost = {...}``, the reference's
tests/test_afford_nobles_obs.py:16-17) are honoured: a state whose cards differ from the canonical
data is evaluated on a scratch arena whose context was built from that state's card table
(SplendorState.card_table), and apply_action's result keeps the input's Card objects.

Deviation (documented in DESIGN.md §12): apply_action validates the move as SplendorEnv.step does
and raises ValueError for a move that is illegal in the state (the reference applies it
unchecked) and RuntimeError on a terminal state.
"""
from typing import List, Optional

import numpy as np

from .. import _native
from .encode import TOTAL_ACTIONS
from .state import SplendorState

_SCRATCH = {}
_CUSTOM_KEEP = 8  # scratch engines kept for edited card tables (oldest dropped first)


def _scratch(num_players, cards=None):
    """One-table arena per (player count, device, card table) on the current device (created on first
    use); cards = an edited int32 [90, 8] card table or None for the canonical one."""
    import torch
    from ..device import Engine
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None
    key = (int(num_players), dev, None if cards is None else cards.tobytes())
    eng = _SCRATCH.get(key)
    if eng is None:
        if cards is not None:
            custom = [k for k in _SCRATCH if k[2] is not None]
            for k in custom[:max(0, len(custom) - _CUSTOM_KEEP + 1)]:
                _SCRATCH.pop(k).close()
        eng = Engine(1, int(num_players), refill_period=0, cards=cards)
        _SCRATCH[key] = eng
    return eng


def _load(state):
    eng = _scratch(state.num_players, state.card_table())
    eng.upload(state.to_record())
    return eng


def initial_state(num_players: int = 2, seed: int = 0) -> SplendorState:
    eng = _scratch(num_players)
    eng.deal([seed], obs=False)
    return SplendorState.from_record(eng.download(0, 1)[0])


def legal_moves(state) -> List[int]:
    eng = _load(state)
    return [int(x) for x in eng.legal()[0].cpu().numpy()]


def encode_observation(state) -> np.ndarray:
    eng = _load(state)
    return eng.encode()[0].cpu().numpy().copy()


def apply_action(state, action: int) -> SplendorState:
    """The state after `action` (a new object; `state` is not modified)."""
    a = int(action)
    if not 0 <= a < TOTAL_ACTIONS:
        raise ValueError("Invalid action index")  # rules.py:256-257
    eng = _load(state)
    eng.step([a], autoreset=False, final_obs=False)
    flags = int(eng.flags[0].item())
    if flags & _native.F_AFTER_TERMINAL:
        raise RuntimeError("apply_action on a terminal state (game over and to_play == 0)")
    if flags & (_native.F_ILLEGAL | _native.F_DRAW):
        raise ValueError(f"action {a} is not legal in this state (the device engine applies legal moves only)")
    return SplendorState.from_record(eng.download(0, 1)[0], cards=state.cards())


def compute_winner(state) -> Optional[int]:
    """Highest (prestige, -cards bought, -cards reserved); a tie of the top two -> None (rules.py:290-303)."""
    keys = sorted(((p.prestige, -sum(p.bonuses), -len(p.reserved)), i) for i, p in enumerate(state.players))
    keys.reverse()
    if len(keys) >= 2 and keys[0][0] == keys[1][0]:
        return None
    return keys[0][1]


def is_terminal(state) -> bool:
    return bool(state.game_over and state.to_play == 0)


def winner(state) -> Optional[int]:
    return state.winner_index

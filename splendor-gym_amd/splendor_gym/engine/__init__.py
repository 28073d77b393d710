"""The reference engine package surface (splendor_gym/engine/__init__.py:1-13): host views
(state.py) and the functional rules API (rules.py), whose rules run on the GPU
(csrc/spl_engine.hip) — importing touches no device."""
from . import encode  # noqa: F401
from .rules import apply_action, compute_winner, initial_state, is_terminal, legal_moves, winner  # noqa: F401
from .state import Card, Noble, PlayerState, SplendorState  # noqa: F401

__all__ = ["SplendorState", "PlayerState", "Card", "Noble", "legal_moves", "apply_action", "is_terminal", "winner",
           "initial_state", "compute_winner", "encode"]

"""Engine constants and host views.  The rules themselves run on the GPU (csrc/spl_engine.hip);
this package keeps the reference's module names (splendor_gym/engine/__init__.py:1-13)."""
from .state import Card, Noble, PlayerState, SplendorState  # noqa: F401
from . import encode  # noqa: F401

__all__ = ["SplendorState", "PlayerState", "Card", "Noble", "encode"]

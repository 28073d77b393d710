"""splendor_gym (MI355X): drop-in for the reference package, engine on the GPU.

`from splendor_gym.envs import SplendorEnv` and `splendor_gym.engine.encode` constants keep their
reference names (ppo_splendor.py:10, scripts/random_rollout.py:4).  Importing does not touch the
GPU; constructing an env loads the HIP library and fails loudly without it.
"""
from .envs import SplendorEnv, make  # noqa: F401
from .vector import SplendorVectorEnv  # noqa: F401

__all__ = ["SplendorEnv", "make", "SplendorVectorEnv"]

"""Two-player self-play views of SplendorEnv (reference splendor_gym/wrappers/).

Per-env wrappers with the reference's constructors, rewards, info keys and errors; they drive the
GPU-backed SplendorEnv through its public step/reset/state.  For thousands of tables per launch use
splendor_gym.selfplay.DualStepVectorEnv instead.
"""
from .dual_step_native import DualStepNativeWrapper  # noqa: F401
from .dual_step_selfplay import DualStepSelfPlayWrapper  # noqa: F401
from .selfplay import SelfPlayWrapper, random_opponent  # noqa: F401

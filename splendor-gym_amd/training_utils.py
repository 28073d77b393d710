"""The env-construction piece of the reference's training_utils.py (training_utils.py:198-234):
`make_env` with the same signature and wrapper choice, over the GPU-backed SplendorEnv.

The rest of the reference module (TensorBoard logging, plots, checkpoints, evaluation suite)
is training infrastructure outside the env-step hot path and is not provided here.
"""
from splendor_gym.envs import SplendorEnv
from splendor_gym.wrappers.selfplay import SelfPlayWrapper, random_opponent

__all__ = ["make_env", "random_opponent"]


def make_env(seed: int, opponent_policy=None, opponent_supplier=None, random_starts: bool = False,
             use_dual_step: bool = False, use_dual_player: bool = True):
    """Thunk building one 2-player SplendorEnv behind a self-play wrapper, reset with `seed`:
    DualStepNativeWrapper when use_dual_player (default), else DualStepSelfPlayWrapper when
    use_dual_step, else SelfPlayWrapper.  The opponent defaults to random_opponent."""
    if opponent_policy is None and opponent_supplier is None:
        opponent_policy = random_opponent

    def thunk():
        env = SplendorEnv(num_players=2)
        if use_dual_player:
            from splendor_gym.wrappers.dual_step_native import DualStepNativeWrapper as W
        elif use_dual_step:
            from splendor_gym.wrappers.dual_step_selfplay import DualStepSelfPlayWrapper as W
        else:
            W = SelfPlayWrapper
        env = W(env, opponent_policy=opponent_policy or random_opponent, opponent_supplier=opponent_supplier,
                random_starts=random_starts)
        env.reset(seed=seed)
        return env

    return thunk

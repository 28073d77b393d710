"""Shared pieces of the self-play wrappers: opponent choice per episode and the opening moves
before the agent's first turn (reference selfplay.py:20-40, dual_step_*.py:45-79)."""
import numpy as np


def random_opponent(obs, info):
    """Uniform choice among the legal actions of info["action_mask"] with numpy's global RNG;
    0 when no mask or no legal action (reference wrappers/selfplay.py:66-73)."""
    mask = info.get("action_mask")
    if mask is None:
        return 0
    legal = np.flatnonzero(mask)
    return int(np.random.choice(legal)) if len(legal) else 0


def episode_opponent(wrapper):
    """The policy for the next episode: a fresh one from the supplier, else the fixed one."""
    return wrapper.opponent_supplier() if wrapper.opponent_supplier is not None else wrapper.opponent_policy


def play_opening(wrapper, obs, info, on_opponent_move=None):
    """After env.reset: the opponent moves while it is to play, until the game ends.  With random
    starts the reference first flips numpy's global coin when the opponent is to play; heads gives
    it one move before the same loop, so either outcome plays the same moves — the flip only
    consumes the draw, which is kept for identical global RNG use."""
    env = wrapper.env
    if wrapper.random_starts and info.get("to_play", 0) == 1:
        np.random.rand()
    while info.get("to_play", 0) == 1:
        obs, _, term, trunc, info = env.step(wrapper._opp_policy(obs, info))
        if on_opponent_move is not None:
            on_opponent_move()
        if term or trunc:
            break
    return obs, info


def final_reward(info, player):
    """info["final_rewards"][player] when the step reported them, else 0.0."""
    fr = info.get("final_rewards")
    return fr[player] if fr is not None and player in fr else 0.0

"""Scripted opponents of the reference evaluation suite, as per-env callables (obs, info) -> action
with the reference behaviour (scripts/eval_suite.py:9-78; wrappers/selfplay.py:66-73).

Their batched device forms are the SPL_POLICY_* policies of the step kernel
(`DualStepVectorEnv(opponent="greedy_v1" | "basic_priority" | "random")`): greedy_v1 is
deterministic and identical; the random choices of the other two use the device Philox stream
instead of numpy's global generator.
"""
import numpy as np

from .wrappers._common import random_opponent  # noqa: F401  (wrappers/selfplay.py:66-73)

BOARD_OBS_OFFSET = 32  # first visible card's 13 observation ints (engine/encode.py:144-147)


def greedy_opponent_v1(obs, info):
    """First legal action among buys (visible or reserved), else take-2, take-3, reserve
    (eval_suite.py:9-29)."""
    legal = np.flatnonzero(info["action_mask"])
    if len(legal) == 0:
        return 0
    buys = legal[((legal >= 15) & (legal <= 26)) | ((legal >= 42) & (legal <= 44))]
    for group in (buys, legal[(legal >= 10) & (legal <= 14)], legal[legal <= 9], legal[(legal >= 27) & (legal <= 41)]):
        if len(group):
            return int(group[0])
    return int(legal[0])


def basic_priority_opponent(obs, info):
    """Visible buy with the most points (random tie-break), else a random reserved buy, else a
    random take-3, take-2, reserve (eval_suite.py:32-78)."""
    legal = np.flatnonzero(info["action_mask"])
    if len(legal) == 0:
        return 0
    vis = legal[(legal >= 15) & (legal <= 26)]
    if len(vis):
        pts = np.array([int(obs[BOARD_OBS_OFFSET + (a - 15) * 13 + 2]) for a in vis])
        return int(np.random.choice(vis[pts == pts.max()]))
    for lo, hi in ((42, 44), (0, 9), (10, 14), (27, 41)):
        group = legal[(legal >= lo) & (legal <= hi)]
        if len(group):
            return int(np.random.choice(group))
    return int(legal[0])

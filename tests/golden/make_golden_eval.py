"""Fixtures for batched evaluation: the REFERENCE scripts/eval_suite.py eval_vs_opponent run with
deterministic policies (agent = first legal action, or last legal action; opponent =
greedy_opponent_v1 / random-free), loaded as in make_golden.py.

    python tests/golden/make_golden_eval.py     # here, with /root/reference present
"""
import json
import os

import numpy as np

import make_golden as mg  # noqa: F401  (installs the reference + gymnasium stand-in)

HERE = os.path.dirname(os.path.abspath(__file__))


def first_legal(obs, info):
    legal = np.flatnonzero(info["action_mask"])
    return int(legal[0]) if len(legal) else 0


def last_legal(obs, info):
    legal = np.flatnonzero(info["action_mask"])
    return int(legal[-1]) if len(legal) else 0


if __name__ == "__main__":
    from splendor_gym.scripts import eval_suite as es
    out = []
    for agent_name, agent in (("first_legal", first_legal), ("last_legal", last_legal)):
        for seed, n in ((0, 60), (7, 40)):
            res = es.eval_vs_opponent(es.make_selfplay_env_with(es.greedy_opponent_v1, 0), agent, n_games=n, seed=seed)
            out.append({"agent": agent_name, "opponent": "greedy_v1", "seed": seed, "n_games": n,
                        "result": {k: (float(v) if isinstance(v, (float, np.floating)) else int(v)) for k, v in res.items()}})
            print(agent_name, seed, res)
    with open(os.path.join(HERE, "eval.json"), "w") as f:
        json.dump(out, f, indent=1)

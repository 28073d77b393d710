"""Self-play wrappers (reference splendor_gym/wrappers/) replayed against fixtures from the
reference wrappers themselves (tests/golden/make_golden_wrappers.py): on CPU over the oracle-backed
test double, on the GPU over the real SplendorEnv."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def fixtures():
    with open(os.path.join(GOLD, "wrappers.json")) as f:
        return json.load(f)


def _digest(obs):
    import hashlib
    return int.from_bytes(hashlib.blake2b(np.asarray(obs, dtype=np.int32).tobytes(), digest_size=8).digest(),
                          "little")


def _mask_bits(mask):
    return sum(1 << i for i, x in enumerate(np.asarray(mask)) if x)


def _info_rec(info, keys):
    r = {k: (v.item() if isinstance(v, np.generic) else v) for k, v in info.items() if k in keys}
    if "final_rewards" in info:
        r["final_rewards"] = {str(k): float(v) for k, v in info["final_rewards"].items()}
    r["mask"] = _mask_bits(info["action_mask"])
    return r


def _wrapper_class(kind):
    from splendor_gym.wrappers import DualStepNativeWrapper, DualStepSelfPlayWrapper, SelfPlayWrapper
    return {"selfplay": SelfPlayWrapper, "dual_step_selfplay": DualStepSelfPlayWrapper,
            "dual_step_native": DualStepNativeWrapper}[kind]


def _pick(rs, info):
    legal = np.flatnonzero(info["action_mask"])
    return int(legal[rs.integers(len(legal))]) if len(legal) else 0


def replay(game, make_env):
    keys = ("to_play", "turn_count", "agent_action", "opponent_action", "opponent_reward", "phase",
            "turn_complete", "game_ended_on", "total_agent_actions", "total_opponent_actions",
            "total_agent_steps", "total_opponent_steps", "illegal_action", "draw", "turn_limit")
    g, kind = game["game"], game["kind"]
    rs_agent, rs_opp = np.random.default_rng(5000 + g), np.random.default_rng(9000 + g)
    w = _wrapper_class(kind)(make_env(), opponent_policy=lambda obs, info: _pick(rs_opp, info),
                             random_starts=game["random_starts"])
    np.random.seed(g)
    obs, info = w.reset(seed=game["env_seed"])
    assert _digest(obs) == game["reset"]["obs"]
    assert _info_rec(info, keys) == game["reset"]["info"]
    for t, want in enumerate(game["steps"]):
        a = _pick(rs_agent, info)
        assert a == want["a"], (kind, g, t)
        if kind == "dual_step_native":
            ao, ar, oo, orr, done, info = w.dual_step(a)
            got = {"a": a, "obs": _digest(ao), "reward": float(ar), "opp_obs": _digest(oo), "opp_reward": float(orr),
                   "done": bool(done)}
        else:
            obs, r, term, trunc, info = w.step(a)
            got = {"a": a, "obs": _digest(obs), "reward": float(r), "done": bool(term), "trunc": bool(trunc)}
        got["info"] = _info_rec(info, keys)
        assert got == want, (kind, g, t)


def illegal(case, make_env):
    w = _wrapper_class(case["kind"])(make_env(), opponent_policy=lambda obs, info: 0, random_starts=False)
    w.reset(seed=77)
    with pytest.raises(Exception) as ei:
        (w.dual_step if case["kind"] == "dual_step_native" else w.step)(case["action"])
    assert type(ei.value).__name__ == case["raises"]


def test_wrappers_match_reference_on_oracle_env(fixtures):
    from oracle_env import OracleSplendorEnv
    for game in fixtures["games"]:
        replay(game, OracleSplendorEnv)
    for case in fixtures["illegal"]:
        illegal(case, OracleSplendorEnv)


@pytest.mark.gpu
def test_wrappers_match_reference_on_gpu_env(fixtures):
    from splendor_gym.envs import SplendorEnv
    games = [g for g in fixtures["games"] if g["game"] < 4]  # 12 games, ~500 steps: per-step kernel launches
    for game in games:
        replay(game, SplendorEnv)
    for case in fixtures["illegal"]:
        illegal(case, SplendorEnv)


@pytest.mark.gpu
def test_make_env_dual_step():
    """training_utils.make_env: same signature and wrapper choice as the reference."""
    import training_utils
    from splendor_gym.wrappers import DualStepNativeWrapper, DualStepSelfPlayWrapper, SelfPlayWrapper
    env = training_utils.make_env(seed=3)()
    assert isinstance(env, DualStepNativeWrapper)
    assert isinstance(training_utils.make_env(3, use_dual_player=False, use_dual_step=True)(), DualStepSelfPlayWrapper)
    assert isinstance(training_utils.make_env(3, use_dual_player=False)(), SelfPlayWrapper)
    np.random.seed(0)
    obs, info = env.reset(seed=3)
    done, n = False, 0
    while not done and n < 400:
        a = int(np.random.choice(np.flatnonzero(info["action_mask"])))
        ao, ar, oo, orr, done, info = env.dual_step(a)
        n += 1
    assert done and ar in (1.0, -1.0, 0.0, -0.1)

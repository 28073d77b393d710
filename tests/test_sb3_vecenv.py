"""The stable-baselines3 VecEnv adapter (splendor_gym.sb3) against SB3's DummyVecEnv semantics over
reference-semantics single envs (BASELINE.json north_star: "the SB3/CleanRL vector-env API stay
drop-in").  stable-baselines3 is not installed here, so the DummyVecEnv loop is restated in the test
(stable_baselines3/common/vec_env/dummy_vec_env.py step_wait/reset): parity against SB3 itself is
unpinned.  CPU: the adapter over the oracle-backed vector double; GPU: over the HIP SplendorVectorEnv,
bit-equal to the CPU run."""
import numpy as np
import pytest

from oracle_env import OracleSplendorEnv, OracleVectorEnv
from splendor_gym.sb3 import SplendorSB3VecEnv


class DummyVecEnvRef:
    """SB3 DummyVecEnv's step/reset restated over oracle single envs."""

    def __init__(self, n, seed):
        self.envs = [OracleSplendorEnv() for _ in range(n)]
        self.seed = seed
        self.reset_infos = [{} for _ in range(n)]

    def reset(self):
        obs = []
        for i, e in enumerate(self.envs):
            o, self.reset_infos[i] = e.reset(seed=self.seed + i)
            obs.append(o)
        return np.stack(obs)

    def step(self, actions):
        obs, rews, dones, infos = [], [], [], []
        for i, e in enumerate(self.envs):
            o, r, term, trunc, info = e.step(int(actions[i]))
            done = term or trunc
            info["TimeLimit.truncated"] = trunc and not term
            if done:
                info["terminal_observation"] = o
                o, self.reset_infos[i] = e.reset()
            obs.append(o)
            rews.append(r)
            dones.append(done)
            infos.append(info)
        return np.stack(obs), np.array(rews, np.float32), np.array(dones), infos


def assert_info_equal(a, b, ctx):
    assert set(a) == set(b), (ctx, sorted(a), sorted(b))
    for k in a:
        va, vb = a[k], b[k]
        if isinstance(va, np.ndarray) or isinstance(vb, np.ndarray):
            assert np.array_equal(np.asarray(va), np.asarray(vb)), (ctx, k)
        else:
            assert va == vb and type(va) is type(vb), (ctx, k, va, vb)


def run_parity(venv, n, seed, steps):
    ad = SplendorSB3VecEnv(venv=venv)
    ref = DummyVecEnvRef(n, seed)
    assert ad.seed(seed) == [seed + i for i in range(n)]
    o = ad.reset()
    assert np.array_equal(o, ref.reset())
    for i in range(n):
        assert_info_equal(ad.reset_infos[i], ref.reset_infos[i], ("reset", i))
    rng = np.random.default_rng(seed)
    dones_seen = illegal_seen = 0
    trace = []
    for k in range(steps):
        masks = np.stack(ad.env_method("action_masks"))
        legal_pick = np.array([rng.choice(np.flatnonzero(m)) if m.any() else 0 for m in masks])
        # one action in ten is an arbitrary in-range (possibly illegal) action
        acts = np.where(rng.random(n) < 0.1, rng.integers(0, 45, n), legal_pick)
        ad.step_async(acts)
        obs, rew, dones, infos = ad.step_wait()
        robs, rrew, rdones, rinfos = ref.step(acts)
        assert np.array_equal(obs, robs), k
        assert np.array_equal(rew, rrew), k
        assert np.array_equal(dones, rdones), k
        assert len(infos) == n
        for i in range(n):
            assert_info_equal(infos[i], rinfos[i], (k, i))
            if dones[i]:
                assert_info_equal(ad.reset_infos[i], ref.reset_infos[i], ("reset", k, i))
        dones_seen += int(dones.sum())
        illegal_seen += sum(1 for i in range(n) if infos[i].get("illegal_action"))
        trace.append((obs.copy(), rew.copy(), dones.copy()))
    assert dones_seen > 0 and illegal_seen > 0
    return ad, trace


def test_sb3_adapter_matches_dummy_vec_env_over_reference_envs():
    ad, _ = run_parity(OracleVectorEnv(12), 12, seed=100, steps=260)
    # VecEnv surface
    assert ad.num_envs == 12 and ad.observation_space.shape == (297,) and ad.action_space.n == 45
    assert ad.get_attr("num_players") == [2] * 12
    assert ad.get_attr("render_mode", indices=[0, 3]) == [None, None]
    ad.set_attr("my_flag", 7, indices=[1, 2])
    assert ad.get_attr("my_flag", indices=[1, 2]) == [7, 7]
    with pytest.raises(AttributeError):
        ad.get_attr("my_flag")
    assert ad.env_is_wrapped(object) == [False] * 12
    assert ad.get_attr("to_play", indices=0) == [int(ad._last[0][0, 294])]
    assert ad.action_masks().shape == (12, 45) and ad.action_masks().dtype == bool
    with pytest.raises(RuntimeError):
        ad.env_method("get_final_rewards", indices=[0])
    with pytest.raises(AttributeError):
        ad.env_method("no_such_method")
    obs, rew, dones, infos = ad.step(np.zeros(12, np.int64) + ad.action_masks().argmax(1))
    assert infos[-1] is infos[11] and len(infos[2:5]) == 3
    ad.close()
    assert ad.venv.closed


def test_sb3_seed_rules():
    ad = SplendorSB3VecEnv(venv=OracleVectorEnv(3))
    ad._seeds = [5, 9, None]
    with pytest.raises(ValueError):
        ad.reset()


@pytest.mark.gpu
def test_sb3_adapter_over_hip_vector_env_matches_oracle():
    from splendor_gym.vector import SplendorVectorEnv
    n = 64
    _, gpu_trace = run_parity(SplendorVectorEnv(n, device="cuda:0", copy=False), n, seed=7, steps=200)
    _, cpu_trace = run_parity(OracleVectorEnv(n), n, seed=7, steps=200)
    for (a, b, c), (x, y, z) in zip(gpu_trace, cpu_trace):
        assert np.array_equal(a, x) and np.array_equal(b, y) and np.array_equal(c, z)

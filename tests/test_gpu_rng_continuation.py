"""The MT19937 continuation path (csrc/spl_rng.h LaneMT): a deal or token return that needs more
outputs than the register-only stream reaches (454) continues on a full MT19937 state instead of
being refused (the former SPL_F_RNG_LIMIT hole).

  * crafted states (the reference's test style, tests/test_rules.py:37-43) holding hundreds of
    tokens, so that auto_return_tokens (engine/rules.py:150-185) draws far past 454 outputs, stepped
    by every kernel (spl_step, the two-wave and one-wave rollout) against the CPU oracle;
  * the stream-limit test hook lowered so that EVERY deal and every token return runs through the
    continuation: deals, trajectories and rollouts stay bit-exact against the oracle / step chain.
"""
import numpy as np
import pytest

from oracle.oracle import Oracle, OracleVec, table_to_view, view_to_table
from schema import canon

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def engine(n, P, **kw):
    from splendor_gym.device import Engine
    return Engine(n, P, **kw)


def bits_of(mask_i8):
    m = np.asarray(mask_i8).astype(np.uint64)
    return (m << np.arange(45, dtype=np.uint64)).sum(axis=-1).astype(np.uint64)


def crafted(orc, n, P, seed):
    """Initial deals whose player to move holds 50..200 tokens of several colours, and a legal
    action each (takes and reserves end the turn with hundreds of tokens to return)."""
    rs = np.random.default_rng(seed)
    views, acts = [], []
    for i in range(n):
        v = orc.initial_state(P, 500 + i)
        p = v["players"][v["to_play"]]
        k = int(rs.integers(1, 6))
        cols = rs.choice(5, k, replace=False)
        p["tokens"] = [0] * 6
        for c in cols:
            p["tokens"][int(c)] = int(rs.integers(50, 201))
        p["tokens"][5] = int(rs.integers(0, 3))
        legal = [a for a in range(45) if (int(orc.legal(v)) >> a) & 1]
        takes = [a for a in legal if a < 15 or 27 <= a < 42]
        views.append(v)
        acts.append(int(rs.choice(takes if takes else legal)))
    return views, np.array(acts, np.int32)


@pytest.mark.parametrize("P", [2, 4])
def test_token_return_past_the_stream(orc, P):
    import torch
    n = 200
    views, acts = crafted(orc, n, P, 17 + P)
    recs = np.stack([view_to_table(v) for v in views])
    outs = {}
    for mode in ("step", "ws", "one_wave"):
        e = engine(n, P, refill_period=0, pipeline=(mode == "ws"))
        e.reset(seeds=range(n))
        e.upload(recs)
        a = torch.from_numpy(acts).to(e.device)
        if mode == "step":
            e.step(a, autoreset=True, final_obs=True)
        else:
            e.rollout(1, actions=a, next_actions=torch.empty_like(a))
        outs[mode] = (e.obs.cpu().numpy().copy(), e.flags.cpu().numpy().copy(), e.download())
    ref_obs = []
    long_returns = 0
    for i, v in enumerate(views):
        r = orc.env_step(v, int(acts[i]))
        assert r["error"] == 0
        ref_obs.append(r["obs"])
        before = sum(v["players"][v["to_play"]]["tokens"])
        long_returns += before > 300
        for mode in outs:
            if not r["terminated"]:
                assert canon(table_to_view(outs[mode][2][i])) == canon(r["after"]), (mode, i)
    for mode in outs:
        np.testing.assert_array_equal(outs[mode][0], np.stack(ref_obs), err_msg=mode)
        assert not (outs[mode][1] & 0x40).any(), mode  # SPL_F_RNG_LIMIT is never raised
    assert long_returns > 20  # hundreds of returns: far past the 454 streamed outputs


@pytest.fixture()
def low_stream_limit():
    from splendor_gym import _native
    lib = _native.load_library()
    yield lambda k: _native.check(lib, lib.spl_debug_set_stream_limit(k))
    _native.check(lib, lib.spl_debug_set_stream_limit(454))


@pytest.mark.parametrize("P", [2, 3, 4])
def test_deals_through_the_continuation(orc, low_stream_limit, P):
    """Every deal switches to the full-state continuation after 40 (or 1) streamed outputs."""
    for limit in (40, 1):
        low_stream_limit(limit)
        n = 300
        seeds = list(range(9100, 9100 + n))
        e = engine(n, P)
        obs, mask = e.reset(seeds=seeds)
        vec = OracleVec(orc, n, P, seeds)
        np.testing.assert_array_equal(obs.cpu().numpy(), vec.obs)
        recs = e.download()
        for t in range(n):
            assert canon(table_to_view(recs[t])) == canon(vec.table(t)), (limit, t)


def test_trajectories_and_rollout_through_the_continuation(orc, low_stream_limit):
    """Stream limit 3: token returns (auto_return_tokens) and every autoreset / refill deal run the
    continuation inside spl_step and both rollout kernels; outputs stay bit-exact against the oracle
    (spl_step) and against chained steps (rollouts)."""
    import torch
    low_stream_limit(3)
    n, P, plies, seed = 512, 2, 160, 4321
    e = engine(n, P, refill_period=16)
    seeds = [seed + i for i in range(n)]
    e.reset(seeds=seeds)
    vec = OracleVec(orc, n, P, seeds)
    na = torch.zeros(n, dtype=torch.int32, device=e.device)
    e.sample_uniform(out=na, seed=seed, ply=0)
    resets = 0
    for k in range(plies):
        acts = na.cpu().numpy().copy()
        e.step(torch.from_numpy(acts).to(e.device), next_actions=na, policy_seed=seed, ply=k + 1)
        ref = vec.step(acts, want_final=True)
        np.testing.assert_array_equal(e.obs.cpu().numpy(), ref["obs"], err_msg=f"ply {k}")
        np.testing.assert_array_equal(bits_of(e.mask.cpu().numpy()), ref["mask"], err_msg=f"ply {k}")
        np.testing.assert_array_equal(e.flags.cpu().numpy(), ref["flags"], err_msg=f"ply {k}")
        resets += int(ref["terminated"].sum())
    assert resets > 300
    for pipeline, PP in ((True, 2), (False, 2), (True, 4)):
        chain = engine(256, PP, refill_period=16)
        roll = engine(256, PP, refill_period=16, pipeline=pipeline)
        chain.reset(seeds=range(256))
        roll.reset(seeds=range(256))
        a_c = torch.zeros(256, dtype=torch.int32, device=chain.device)
        chain.sample_uniform(out=a_c, seed=3, ply=0)
        a_r = a_c.clone()
        K = 64
        for launch in range(2):
            out = {"obs": torch.empty((K, 256, 297), dtype=torch.int32, device=chain.device),
                   "mask": torch.empty((K, 256, 45), dtype=torch.int8, device=chain.device),
                   "reward": torch.empty((K, 256), dtype=torch.float32, device=chain.device),
                   "terminated": torch.empty((K, 256), dtype=torch.uint8, device=chain.device),
                   "flags": torch.empty((K, 256), dtype=torch.uint8, device=chain.device)}
            nxt = torch.empty_like(a_r)
            roll.rollout(K, actions=a_r, next_actions=nxt, policy_seed=3, ply=1 + K * launch, out=out)
            a_r = nxt
            for k in range(K):
                n2 = torch.empty_like(a_c)
                chain.step(a_c, next_actions=n2, policy_seed=3, ply=1 + K * launch + k)
                a_c = n2
                assert torch.equal(out["obs"][k], chain.obs), (pipeline, PP, launch, k)
                assert torch.equal(out["flags"][k], chain.flags), (pipeline, PP, launch, k)
        assert chain.download().tobytes() == roll.download().tobytes(), (pipeline, PP)

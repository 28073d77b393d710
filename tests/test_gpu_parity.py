"""HIP engine parity: bit-exact against the CPU oracle (itself pinned to the reference by
tests/test_oracle_golden.py) and directly against the reference's own outputs for crafted
states (tests/golden/edge_cases.json).  Every call goes through the C-ABI library."""
import json
import os
import random

import numpy as np
import pytest

from oracle.oracle import Oracle, OracleVec, table_to_view, view_to_table
from schema import canon

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def engine(n, P, **kw):
    from splendor_gym.device import Engine
    return Engine(n, P, **kw)


def bits_of(mask_i8):
    m = np.asarray(mask_i8).astype(np.uint64)
    return (m << np.arange(45, dtype=np.uint64)).sum(axis=-1).astype(np.uint64)


def test_token_lut_matches_cpython():
    e = engine(64, 2)
    lut = e.token_lut()
    assert lut.shape == (128 * 4 * 3 * 16, 4)
    rs = np.random.default_rng(0)
    idx = np.concatenate([np.arange(0, 2048), rs.integers(0, len(lut), 2048)])
    for i in idx:
        i = int(i)
        sb, st, tp, tc = i % 16, 11 + (i // 16) % 3, (i // 48) % 4, i // 192
        seed = (tc * 1315423911) ^ (tp * 2654435761) ^ (st * 97531) ^ (sb * 31337)
        r = random.Random(seed)
        tops = [r.getrandbits(32) >> 29 for _ in range(40)]
        words = [sum(tops[10 * q + k] << (3 * k) for k in range(10)) for q in range(4)]
        assert [int(x) for x in lut[i]] == words, i


@pytest.mark.parametrize("P", [2, 3, 4])
def test_reset_deals(orc, P):
    n = 1000  # not a multiple of 64: exercises the partial last wave
    seeds = list(range(7000, 7000 + n))
    e = engine(n, P)
    obs, mask = e.reset(seeds=seeds)
    vec = OracleVec(orc, n, P, seeds)
    np.testing.assert_array_equal(obs.cpu().numpy(), vec.obs)
    np.testing.assert_array_equal(bits_of(mask.cpu().numpy()), vec.mask)
    recs = e.download()
    for t in range(n):
        assert canon(table_to_view(recs[t])) == canon(vec.table(t)), t


def run_parity(orc, P, n, plies, refill_period, seed, device_policy, check_state_every=50):
    import torch
    e = engine(n, P, refill_period=refill_period)
    seeds = [seed + i for i in range(n)]
    e.reset(seeds=seeds)
    vec = OracleVec(orc, n, P, seeds)
    rs = np.random.default_rng(seed)
    next_actions = torch.zeros(n, dtype=torch.int32, device=e.device)
    e.sample_uniform(out=next_actions, seed=seed, ply=0)
    n_reset = 0
    for k in range(plies):
        if device_policy:
            acts = next_actions.cpu().numpy().copy()
        else:
            acts = np.zeros(n, np.int32)
            for t in range(n):
                legal = np.flatnonzero((int(vec.mask[t]) >> np.arange(45)) & 1)
                acts[t] = rs.choice(legal) if len(legal) else rs.integers(0, 45)
        # inject illegal and (rarely) out-of-range actions: flagged, state unchanged
        inj = rs.random(n)
        acts = np.where(inj < 0.03, rs.integers(0, 45, n), acts)
        acts = np.where(inj > 0.998, rs.choice([-1, 45, 99], n), acts).astype(np.int32)
        e.step(torch.from_numpy(acts).to(e.device), next_actions=next_actions, policy_seed=seed, ply=k + 1)
        ref = vec.step(acts, want_final=True)
        np.testing.assert_array_equal(e.flags.cpu().numpy(), ref["flags"], err_msg=f"flags ply {k}")
        np.testing.assert_array_equal(e.reward.cpu().numpy(), ref["reward"], err_msg=f"reward ply {k}")
        np.testing.assert_array_equal(e.terminated.cpu().numpy(), ref["terminated"], err_msg=f"term ply {k}")
        np.testing.assert_array_equal(e.winner.cpu().numpy(), ref["winner"], err_msg=f"winner ply {k}")
        np.testing.assert_array_equal(e.obs.cpu().numpy(), ref["obs"], err_msg=f"obs ply {k}")
        np.testing.assert_array_equal(bits_of(e.mask.cpu().numpy()), ref["mask"], err_msg=f"mask ply {k}")
        rows = np.flatnonzero(ref["terminated"])
        n_reset += len(rows)
        if len(rows):
            np.testing.assert_array_equal(e.final_obs.cpu().numpy()[rows], ref["final_obs"][rows],
                                          err_msg=f"final obs ply {k}")
        if check_state_every and (k % check_state_every == check_state_every - 1):
            recs = e.download()
            for t in range(0, n, max(1, n // 128)):
                assert canon(table_to_view(recs[t])) == canon(vec.table(t)), (k, t)
    return n_reset


@pytest.mark.parametrize("refill_period", [8, 1, 0])
def test_trajectories_p2_device_policy(orc, refill_period):
    """C2 shape: 2 players, 4096 tables, uniform-random policy drawn on the device; every
    output of every ply compared bit-for-bit with the oracle replaying the same actions.
    The pool refill schedule (every ply / every 8 / inline deals only) must not matter."""
    resets = run_parity(orc, 2, 4096, 240 if refill_period == 8 else 120, refill_period, 1234, True)
    assert resets > 1000


def test_trajectories_c2_2000_plies(orc):
    """SURVEY §8(d) C2 at its specified depth: 2 players, 4 096 tables, 2 000 plies of the device
    uniform-random policy (with injected illegal / out-of-range actions), the default refill period,
    every output of every ply bit-compared with the oracle and the full table state every 250 plies."""
    resets = run_parity(orc, 2, 4096, 2000, 64, 4321, True, check_state_every=250)
    assert resets > 4096 * 2000 // 90  # ~one episode per 77 plies per table


@pytest.mark.parametrize("n", [984, 1000, 520, 4104])
def test_xcd_map_ragged_grids(orc, n):
    """The XCD-contiguous workgroup map (spl_engine.hip wg_block) on grids whose workgroup
    count is a multiple of 8 with a partial last block (984, 1000: 16 workgroups, the last one 24 / 40
    tables; 4104: 72 workgroups at 32 tables per workgroup) and on one that is not (520: 9 workgroups,
    identity map): every ply of k_step_ws bit-compared with the oracle, then a 48-step rollout store
    launch (each rollout kernel shape: auto, two-wave at 64 and 32 tables per workgroup, dealer)
    against the same chain of steps replayed by the oracle."""
    import torch
    run_parity(orc, 2, n, 40, 8, 77 + n, True, check_state_every=20)
    for pipeline in (True, "always", "half", "dealer"):
        e = engine(n, 2, refill_period=16, pipeline=pipeline)
        seeds = [5 + i for i in range(n)]
        e.reset(seeds=seeds)
        vec = OracleVec(orc, n, 2, seeds)
        a = torch.zeros(n, dtype=torch.int32, device=e.device)
        e.sample_uniform(out=a, seed=3, ply=0)
        K = 48
        out = {"obs": torch.empty((K, n, 297), dtype=torch.int32, device=e.device),
               "mask": torch.empty((K, n, 45), dtype=torch.int8, device=e.device),
               "reward": torch.empty((K, n), dtype=torch.float32, device=e.device),
               "terminated": torch.empty((K, n), dtype=torch.uint8, device=e.device),
               "flags": torch.empty((K, n), dtype=torch.uint8, device=e.device),
               "winner": torch.empty((K, n), dtype=torch.int8, device=e.device),
               "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=e.device)}
        acts = torch.empty((K, n), dtype=torch.int32, device=e.device)
        # the actions each step takes are the previous step's next_actions: record them by re-running
        # the device policy stream through a step chain on a twin engine
        twin = engine(n, 2, refill_period=16)
        twin.reset(seeds=seeds)
        ta = a.clone()
        for k in range(K):
            acts[k] = ta
            na = torch.empty_like(ta)
            twin.step(ta, next_actions=na, policy_seed=3, ply=1 + k)
            ta = na
        na = torch.empty_like(a)
        e.rollout(K, actions=a, next_actions=na, policy_seed=3, ply=1, out=out)
        assert torch.equal(na, ta), pipeline
        A = acts.cpu().numpy()
        for k in range(K):
            ref = vec.step(A[k], want_final=True)
            np.testing.assert_array_equal(out["obs"][k].cpu().numpy(), ref["obs"], err_msg=f"{pipeline} obs {k}")
            np.testing.assert_array_equal(bits_of(out["mask"][k].cpu().numpy()), ref["mask"],
                                          err_msg=f"{pipeline} mask {k}")
            np.testing.assert_array_equal(out["reward"][k].cpu().numpy(), ref["reward"], err_msg=f"{pipeline} rew {k}")
            np.testing.assert_array_equal(out["terminated"][k].cpu().numpy(), ref["terminated"])
            rows = np.flatnonzero(ref["terminated"])
            if len(rows):
                np.testing.assert_array_equal(out["final_obs"][k].cpu().numpy()[rows], ref["final_obs"][rows])
        recs = e.download()
        for t in range(n):
            assert canon(table_to_view(recs[t])) == canon(vec.table(t)), (pipeline, t)


@pytest.mark.parametrize("P", [3, 4])
def test_trajectories_multiplayer(orc, P):
    resets = run_parity(orc, P, 1024, 200, 8, 99 * P, False)
    assert resets > 50


def test_edge_cases_against_reference():
    """Crafted and fuzzed states from the REAL reference (make_golden.py): upload, one step
    without autoreset, compare outputs and the resulting state."""
    import torch
    with open(os.path.join(GOLD, "edge_cases.json")) as f:
        cases = json.load(f)
    for P in (2, 3, 4):
        cs = [c for c in cases if c["P"] == P]
        e = engine(len(cs), P)
        e.reset(seeds=list(range(len(cs))))
        recs = np.stack([view_to_table(c["before"]) for c in cs])
        e.upload(recs)
        acts = torch.tensor([c["action"] for c in cs], dtype=torch.int32, device=e.device)
        e.step(acts, autoreset=False)
        flags = e.flags.cpu().numpy()
        obs, mask = e.obs.cpu().numpy(), bits_of(e.mask.cpu().numpy())
        rew, term = e.reward.cpu().numpy(), e.terminated.cpu().numpy()
        after = e.download()
        for i, c in enumerate(cs):
            exp_err = {None: 0, "RuntimeError": 0x08, "ValueError": 0x10}[c["exception"]]
            assert flags[i] & 0x18 == exp_err, c["name"]
            assert canon(table_to_view(after[i])) == canon(c["after"]), c["name"]
            if exp_err:
                continue
            np.testing.assert_array_equal(obs[i], np.array(c["obs"], np.int32), err_msg=c["name"])
            assert int(mask[i]) == c["mask"], c["name"]
            assert rew[i] == np.float32(c["reward"]), c["name"]
            assert term[i] == c["terminated"], c["name"]
            assert flags[i] & 7 == c["flags"], c["name"]


def test_upload_download_roundtrip(orc):
    e = engine(300, 2)
    e.reset(seeds=list(range(300)))
    recs = e.download()
    e.upload(recs)
    again = e.download()
    assert recs.tobytes() == again.tobytes()


def test_sharded_equals_whole():
    """Tables split over two engines (global ids 0..2047 and 2048..4095) evolve exactly as one
    engine of 4096: streams are keyed by global table id (multi-GPU sharding invariance)."""
    import torch
    n, half, plies = 4096, 2048, 150
    whole = engine(n, 2)
    parts = [engine(half, 2, table0=0), engine(half, 2, table0=half)]
    seeds = list(range(n))
    whole.reset(seeds=seeds)
    parts[0].reset(seeds=seeds[:half])
    parts[1].reset(seeds=seeds[half:])
    na_w = torch.zeros(n, dtype=torch.int32, device=whole.device)
    na_p = [torch.zeros(half, dtype=torch.int32, device=whole.device) for _ in parts]
    whole.sample_uniform(out=na_w, seed=5, ply=0)
    for p, na in zip(parts, na_p):
        p.sample_uniform(out=na, seed=5, ply=0)
    for k in range(plies):
        whole.step(na_w.clone(), next_actions=na_w, policy_seed=5, ply=k + 1)
        for p, na in zip(parts, na_p):
            p.step(na.clone(), next_actions=na, policy_seed=5, ply=k + 1)
        got = torch.cat([parts[0].obs, parts[1].obs])
        assert torch.equal(got, whole.obs), k
        assert torch.equal(torch.cat([parts[0].flags, parts[1].flags]), whole.flags), k


def test_unseeded_tables_deal_engine_seed_zero(orc):
    """A table never reset with a seed has no engine-seed stream (zeroed PCG64 record): the
    refill and an unseeded reset must terminate and deal engine seed 0 (splendor_amd.h)."""
    n = 130
    e = engine(n, 2)
    e.refill()             # every table pending and unseeded
    e.reset(seeds=None)    # flips to the pool deal
    want = canon(orc.initial_state(2, 0))
    recs = e.download()
    for t in (0, 64, n - 1):
        assert canon(table_to_view(recs[t])) == want, t
    e.reset(seeds=None)    # pool consumed, not refilled: inline deal, same seed
    recs = e.download()
    assert canon(table_to_view(recs[5])) == want


@pytest.mark.parametrize("P,K,refill_fused,pipeline,R", [(2, 16, True, True, 16), (2, 16, True, False, 16),
                                                          (4, 16, True, True, 16), (4, 16, True, False, 16),
                                                          (4, 16, False, "always", 16), (2, 16, False, True, 16),
                                                          (2, 64, True, True, 64), (3, 16, True, True, 16),
                                                          (3, 16, True, False, 16), (4, 64, True, True, 16),
                                                          (4, 64, True, False, 16), (3, 64, True, "always", 32),
                                                          (4, 16, True, True, 0), (3, 16, True, True, 0),
                                                          (2, 16, True, "always", 16), (4, 64, True, "always", 16),
                                                          (4, 16, True, "always", 0), (2, 16, False, "half", 16),
                                                          (4, 128, True, "dealer", 16), (2, 16, True, "dealer", 0),
                                                          (3, 64, False, "dealer", 32), (4, 64, True, "dealer", 1),
                                                          (4, 128, True, "dealer2", 16), (2, 16, True, "dealer2", 0),
                                                          (3, 64, False, "dealer2", 32), (2, 64, True, "quad", 64),
                                                          (4, 128, True, "quad", 16), (3, 16, True, "quad", 0),
                                                          (2, 16, False, "quad", 16)])
def test_rollout_equals_step_chain(P, K, refill_fused, pipeline, R):
    """spl_rollout(K) is K chained spl_step calls (next_actions fed back, plies ply..ply+K-1):
    every per-step output, the terminal rows of final_obs, episode statistics, the next action
    and the table state match bit for bit, across launches with refills in between — refills
    fused into the rollout launch (each wave at its own step; several per launch when it spans
    several refill periods) or launched after it, or never (R = 0: inline deals once the pool ring is
    spent, through the deal scratch that shares the state slot at 4 players); the two-wave
    pipelined kernel (32 or 64 tables per workgroup), the three-wave dealer variant (the auto choice
    at this size: a third wave deals the refills, spent pools post a batch and wait) or one wave per
    64 tables."""
    _check_rollout_vs_chain(P, K, refill_fused, pipeline, R)


def _check_rollout_vs_chain(P, K, refill_fused, pipeline, R, partner_lead=None, launches=None, n=1024):
    import torch
    seed = 11
    launches = launches or (5 if K <= 16 else 3)
    chain = engine(n, P, refill_period=R)
    fused = engine(n, P, refill_period=R, refill_fused=refill_fused, pipeline=pipeline, partner_lead=partner_lead)
    chain.reset(seeds=range(n))
    fused.reset(seeds=range(n))
    dev = chain.device
    a_c = torch.zeros(n, dtype=torch.int32, device=dev)
    chain.sample_uniform(out=a_c, seed=seed, ply=0)
    a_f = a_c.clone()
    stats = {k: (torch.zeros(n, dtype=torch.float32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev))
             for k in ("c", "f")}
    for launch in range(launches):
        ply0 = 1 + launch * K
        want = []
        for k in range(K):
            na = torch.empty_like(a_c)
            chain.step(a_c, next_actions=na, policy_seed=seed, ply=ply0 + k, ep_return=stats["c"][0],
                       ep_count=stats["c"][1])
            want.append({name: getattr(chain, name).clone() for name in
                         ("obs", "mask", "reward", "terminated", "flags", "winner", "final_obs")})
            a_c = na
        out = {"obs": torch.empty((K, n, 297), dtype=torch.int32, device=dev),
               "mask": torch.empty((K, n, 45), dtype=torch.int8, device=dev),
               "reward": torch.empty((K, n), dtype=torch.float32, device=dev),
               "terminated": torch.empty((K, n), dtype=torch.uint8, device=dev),
               "flags": torch.empty((K, n), dtype=torch.uint8, device=dev),
               "winner": torch.empty((K, n), dtype=torch.int8, device=dev),
               "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev)}
        na = torch.empty_like(a_f)
        fused.rollout(K, actions=a_f, next_actions=na, policy_seed=seed, ply=ply0, out=out,
                      ep_return=stats["f"][0], ep_count=stats["f"][1])
        a_f = na
        for k in range(K):
            for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
                assert torch.equal(out[name][k], want[k][name]), (launch, k, name)
            term = want[k]["terminated"].bool()
            assert torch.equal(out["final_obs"][k][term], want[k]["final_obs"][term]), (launch, k)
        assert torch.equal(a_f, a_c), launch
        assert int(want[-1]["terminated"].sum()) >= 0
    assert torch.equal(stats["c"][0], stats["f"][0]) and torch.equal(stats["c"][1], stats["f"][1])
    assert int(stats["c"][1].sum()) > 0  # episodes finished and autoreset inside the rollouts
    assert chain.download().tobytes() == fused.download().tobytes()
    # overwrite mode: block 0 holds the last step's outputs
    na_c, na_f = torch.empty_like(a_c), torch.empty_like(a_f)
    for k in range(K):
        chain.step(a_c, next_actions=na_c, policy_seed=seed, ply=1000 + k)
        a_c, na_c = na_c, a_c
    fused.rollout(K, actions=a_f, next_actions=na_f, policy_seed=seed, ply=1000)
    for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
        assert torch.equal(getattr(chain, name), getattr(fused, name)), name
    assert torch.equal(a_c, na_f)
    return fused


@pytest.mark.gpu
@pytest.mark.parametrize("P,lead,pipeline", [(4, -1, "dealer2"), (2, -1, "dealer2"), (4, 2, "dealer2"), (3, 1, "dealer2"),
                                             (3, -1, "dealer2"), (2, -1, "always"), (4, -1, "always"),
                                             (2, -1, "quad"), (4, -1, "quad"), (3, -1, "quad"), (2, 2, "quad")])
def test_partner_handoff_equals_step_chain(P, lead, pipeline):
    """The partner hand-off of the six-wave dealer's rollout store (spl_ctx_set_partner_lead; its dealer
    wave polls the flags): with lead -1 every team hands its steps' rows to the same team of the
    neighbouring-XCC workgroup whenever a task slot is free, so the partner's output wave encodes and
    stores many row blocks between its own steps (and the poster claims back what is left at the end);
    every per-step output still equals the chained spl_step bit for bit, and the diagnostic counters
    show the hand-offs happened.  Lead 1-2: hand-offs only when a partner runs ahead (timing-dependent;
    same results either way).  The two-wave kernel ("always") has no partner hand-off since round 5
    (VERDICT r04 item 1): a forced lead is ignored there, no task is handed off; the quad kernel (four
    two-wave teams in one workgroup per CU, its rules waves polling) has it."""
    import ctypes
    from splendor_gym import _native
    st = (ctypes.c_uint64 * 2)()
    probe = engine(128, 2)
    _native.check(probe.lib, probe.lib.spl_debug_partner_stats(st, 1))
    fused = _check_rollout_vs_chain(P, 64, True, pipeline, 16, partner_lead=lead, launches=3)
    name = {"dealer2": f"k_rollout_store_dealer2_{P}p", "quad": f"k_rollout_store_quad_{P}p"}.get(pipeline, f"k_rollout_store_{P}p")
    assert fused.rollout_kernel_name() == name
    _native.check(fused.lib, fused.lib.spl_debug_partner_stats(st, 1))
    if pipeline not in ("dealer2", "quad"):
        assert st[0] == 0 and st[1] == 0, (st[0], st[1])
    elif lead < 0:
        assert st[0] > 0, (st[0], st[1])  # the partners stored handed-off blocks


@pytest.mark.gpu
@pytest.mark.parametrize("pipeline,n", [("dealer2", 1000), ("dealer2", 1156), ("quad", 1000), ("quad", 1156),
                                        ("quad", 1792)])
def test_partner_handoff_ragged_grids_equal_step_chain(pipeline, n):
    """Forced partner hand-off of the multi-team kernels on grids whose last workgroup is partial or
    has no neighbour (dealer2, n = 1000: 8 workgroups of two 64-table teams, the last team ragged;
    1 156: an odd count of 64-table teams; quad, n = 1792: 7 workgroups of four teams, the last without
    a neighbour): those teams keep their rows (pair and neighbour checks), every other team hands off,
    and the outputs equal the chained spl_step."""
    _check_rollout_vs_chain(2, 32, True, pipeline, 16, partner_lead=-1, launches=2, n=n)


@pytest.mark.parametrize("pipeline", [True, "always", False])
def test_rollout_mass_termination_and_long_games(pipeline):
    """Every table of a wave ending in the same step (crafted: one move before the turn limit),
    more than the pipelined kernel hands over per step, and final rows with move_count > 255:
    spl_rollout equals chained spl_step, per-step outputs and final_obs rows."""
    import torch
    n, K, seed = 512, 8, 5
    chain = engine(n, 2, refill_period=K)
    roll = engine(n, 2, refill_period=K, pipeline=pipeline)
    chain.reset(seeds=range(n))
    roll.reset(seeds=range(n))
    dev = chain.device
    a = torch.zeros(n, dtype=torch.int32, device=dev)
    chain.sample_uniform(out=a, seed=seed, ply=0)
    for k in range(7):  # an odd number of plies in (player 1 to move), then craft
        na = torch.empty_like(a)
        chain.step(a, next_actions=na, policy_seed=seed, ply=100 + k)
        a = na
    recs = chain.download()
    odd = (recs["move_count"] % 2) == 1
    # tables with player 1 to move: one move before turn 100 (move_count 197) -> all end next step;
    # every 7th of them far beyond it (crafted move_count > 255: the final row patch)
    recs["move_count"] = np.where(odd, 197, recs["move_count"])
    recs["turn_count"] = np.where(odd, 99, recs["turn_count"])
    far = odd & (np.arange(n) % 7 == 0)
    recs["move_count"] = np.where(far, 301, recs["move_count"])
    recs["turn_count"] = np.where(far, 151, recs["turn_count"])
    chain.upload(recs)
    roll.upload(recs)
    chain.sample_uniform(out=a, seed=seed, ply=0)
    a_r = a.clone()
    want = []
    for k in range(K):
        na = torch.empty_like(a)
        chain.step(a, next_actions=na, policy_seed=seed, ply=1 + k)
        want.append({name: getattr(chain, name).clone() for name in
                     ("obs", "mask", "reward", "terminated", "flags", "winner", "final_obs")})
        a = na
    out = {"obs": torch.empty((K, n, 297), dtype=torch.int32, device=dev),
           "mask": torch.empty((K, n, 45), dtype=torch.int8, device=dev),
           "reward": torch.empty((K, n), dtype=torch.float32, device=dev),
           "terminated": torch.empty((K, n), dtype=torch.uint8, device=dev),
           "flags": torch.empty((K, n), dtype=torch.uint8, device=dev),
           "winner": torch.empty((K, n), dtype=torch.int8, device=dev),
           "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev)}
    na = torch.empty_like(a_r)
    roll.rollout(K, actions=a_r, next_actions=na, policy_seed=seed, ply=1, out=out)
    assert int(want[0]["terminated"].sum()) > 64  # whole waves ended at once
    assert int(want[0]["final_obs"][:, 295].max()) > 255
    for k in range(K):
        for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
            assert torch.equal(out[name][k], want[k][name]), (k, name)
        term = want[k]["terminated"].bool()
        assert torch.equal(out["final_obs"][k][term], want[k]["final_obs"][term]), k
    assert torch.equal(na, a)
    assert chain.download().tobytes() == roll.download().tobytes()


def test_rollout_store_delegation_equals_undelegated():
    """Rollout-store delegation (the odd workgroup of each pair hands every 4th step's rows to its
    even partner; spl_ctx_set_rollout_delegation) changes nothing: 11 workgroups (five pairs and an
    unpaired last one), crafted tables with move_count > 255 (their delegated steps are stored by
    the producer itself), several eager launches, then hipGraph replays of one captured launch
    (launch epochs counted on the device), against the same rollouts without delegation."""
    import torch
    n, K, seed, R = 64 * 11, 24, 3, 8
    ref = engine(n, 2, refill_period=R, pipeline="always", delegation=0)
    dlg = engine(n, 2, refill_period=R, pipeline="always", delegation=4)
    ref.reset(seeds=range(n))
    dlg.reset(seeds=range(n))
    recs = ref.download()
    big = np.arange(n) % 5 == 0
    recs["move_count"] = np.where(big, 300 + 2 * (recs["move_count"] % 2), recs["move_count"])
    ref.upload(recs)
    dlg.upload(recs)
    dev = ref.device
    a_r = torch.zeros(n, dtype=torch.int32, device=dev)
    ref.sample_uniform(out=a_r, seed=seed, ply=0)
    a_d = a_r.clone()

    def outs():
        return {"obs": torch.full((K, n, 297), -1, dtype=torch.int32, device=dev),
                "mask": torch.empty((K, n, 45), dtype=torch.int8, device=dev),
                "reward": torch.empty((K, n), dtype=torch.float32, device=dev),
                "terminated": torch.empty((K, n), dtype=torch.uint8, device=dev),
                "flags": torch.empty((K, n), dtype=torch.uint8, device=dev),
                "winner": torch.empty((K, n), dtype=torch.int8, device=dev),
                "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev)}

    def same(o_r, o_d, tag):
        for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
            assert torch.equal(o_r[name], o_d[name]), (tag, name)
        term = o_r["terminated"].bool()
        assert torch.equal(o_r["final_obs"][term], o_d["final_obs"][term]), tag

    saw_big = False
    for launch in range(3):
        o_r, o_d = outs(), outs()
        na_r, na_d = torch.empty_like(a_r), torch.empty_like(a_d)
        ref.rollout(K, actions=a_r, next_actions=na_r, policy_seed=seed, ply=1 + K * launch, out=o_r)
        dlg.rollout(K, actions=a_d, next_actions=na_d, policy_seed=seed, ply=1 + K * launch, out=o_d)
        same(o_r, o_d, launch)
        saw_big = saw_big or bool((o_r["obs"][:, :, 295] > 255).any())
        assert torch.equal(na_r, na_d)
        a_r, a_d = na_r, na_d
    assert saw_big  # the producer's own-store path ran
    assert ref.download().tobytes() == dlg.download().tobytes()
    # graph replays of one captured launch: the kernel arguments repeat, the epochs do not
    o_d, na_d = outs(), torch.empty_like(a_d)
    torch.cuda.synchronize(dev)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            dlg.rollout(K, actions=a_d, next_actions=na_d, policy_seed=seed, ply=500, out=o_d)
    for rep in range(2):
        o_d["obs"].fill_(-1)
        g.replay()
        o_r, na_r = outs(), torch.empty_like(a_r)
        ref.rollout(K, actions=a_r, next_actions=na_r, policy_seed=seed, ply=500, out=o_r)
        torch.cuda.synchronize(dev)
        same(o_r, o_d, ("replay", rep))
        a_r.copy_(na_r)
        a_d.copy_(na_d)


@pytest.mark.parametrize("players", [3, 4])
def test_rollout_store_delegation_multiplayer(players):
    """Delegation at 3 and 4 players (more state words staged per table): two launches of a
    6-workgroup rollout store equal the undelegated ones, outputs and final state."""
    import torch
    n, K, seed, R = 64 * 6, 24, 5, 8
    ref = engine(n, players, refill_period=R, pipeline="always", delegation=0)
    dlg = engine(n, players, refill_period=R, pipeline="always", delegation=4)
    ref.reset(seeds=range(n))
    dlg.reset(seeds=range(n))
    dev = ref.device
    a_r = torch.zeros(n, dtype=torch.int32, device=dev)
    ref.sample_uniform(out=a_r, seed=seed, ply=0)
    a_d = a_r.clone()

    def outs():
        return {"obs": torch.full((K, n, 297), -1, dtype=torch.int32, device=dev),
                "mask": torch.empty((K, n, 45), dtype=torch.int8, device=dev),
                "reward": torch.empty((K, n), dtype=torch.float32, device=dev),
                "terminated": torch.empty((K, n), dtype=torch.uint8, device=dev),
                "flags": torch.empty((K, n), dtype=torch.uint8, device=dev),
                "winner": torch.empty((K, n), dtype=torch.int8, device=dev),
                "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev)}

    for launch in range(2):
        o_r, o_d = outs(), outs()
        na_r, na_d = torch.empty_like(a_r), torch.empty_like(a_d)
        ref.rollout(K, actions=a_r, next_actions=na_r, policy_seed=seed, ply=1 + K * launch, out=o_r)
        dlg.rollout(K, actions=a_d, next_actions=na_d, policy_seed=seed, ply=1 + K * launch, out=o_d)
        for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
            assert torch.equal(o_r[name], o_d[name]), (launch, name)
        term = o_r["terminated"].bool()
        assert torch.equal(o_r["final_obs"][term], o_d["final_obs"][term]), launch
        assert torch.equal(na_r, na_d)
        a_r, a_d = na_r, na_d
    assert ref.download().tobytes() == dlg.download().tobytes()


def test_dual_step_vector_env_matches_per_env_wrappers():
    """DualStepVectorEnv (fused device greedy_v1 opponent) == per-env DualStepNativeWrapper over
    SplendorEnv with the host greedy_opponent_v1, including the PPO loop's reset after done; the
    optional step counter (spl_dual_io_t.step_counter) advances by one per dual step."""
    import torch
    from splendor_gym.envs import SplendorEnv
    from splendor_gym.opponents import greedy_opponent_v1
    from splendor_gym.selfplay import DualStepVectorEnv
    from splendor_gym.wrappers import DualStepNativeWrapper
    n, steps, seed = 6, 150, 40
    counter = torch.full((1,), 7, dtype=torch.int64, device="cuda")
    vec = DualStepVectorEnv(n, opponent="greedy_v1", step_counter=counter)
    obs_v, info_v = vec.reset(seed=seed)
    envs = [DualStepNativeWrapper(SplendorEnv(), opponent_policy=greedy_opponent_v1, random_starts=False)
            for _ in range(n)]
    per = [w.reset(seed=seed + i) for i, w in enumerate(envs)]
    rs = np.random.default_rng(3)
    ended = 0
    for k in range(steps):
        acts = []
        for i in range(n):
            legal = np.flatnonzero(per[i][1]["action_mask"])
            acts.append(int(rs.choice(legal)) if len(legal) else 0)
        assert np.array_equal(info_v["action_mask"].cpu().numpy(), np.stack([p[1]["action_mask"] for p in per]))
        ao, ar, oo, orr, done, info_v = vec.dual_step(torch.tensor(acts, dtype=torch.int32, device=vec.device))
        for i, w in enumerate(envs):
            a_obs, a_rew, o_obs, o_rew, d, inf = w.dual_step(acts[i])
            assert bool(done[i]) == bool(d), (k, i)
            assert float(ar[i]) == pytest.approx(a_rew) and float(orr[i]) == pytest.approx(o_rew), (k, i)
            assert np.array_equal(oo[i].cpu().numpy(), o_obs), (k, i)  # post-turn (final) observation
            if d:
                ended += 1
                assert np.array_equal(info_v["final_observation"][i].cpu().numpy(), a_obs)
                per[i] = w.reset()  # ppo_splendor.py:246-256
            else:
                per[i] = (a_obs, inf)
            assert np.array_equal(ao[i].cpu().numpy(), per[i][0]), (k, i)
    assert ended >= n  # every table finished at least one game and was re-dealt
    assert int(counter.item()) == 7 + steps


def test_dual_step_callable_opponent_and_illegal_actions():
    """The callable-opponent path (two spl_step launches, the second gated, then spl_dual_finish)
    equals the fused device-opponent path table for table, including illegal and out-of-range
    agent actions: those leave the table unchanged, the opponent does not move, and info reports
    illegal_action with the -0.01 step reward (envs/splendor_env.py:62-66)."""
    import torch
    from splendor_gym.opponents import greedy_opponent_v1
    from splendor_gym.selfplay import DualStepVectorEnv

    def host_greedy(obs, mask):
        o, m = obs.cpu().numpy(), mask.cpu().numpy()
        return torch.tensor([greedy_opponent_v1(o[i], {"action_mask": m[i]}) for i in range(len(o))],
                            dtype=torch.int32, device=obs.device)

    n, seed = 96, 70
    dev = DualStepVectorEnv(n, opponent="greedy_v1")
    cal = DualStepVectorEnv(n, opponent=host_greedy)
    _, info_d = dev.reset(seed=seed)
    _, info_c = cal.reset(seed=seed)
    rs = np.random.default_rng(9)
    seen_illegal = seen_done = 0
    for k in range(120):
        mask = info_d["action_mask"].cpu().numpy()
        acts = []
        for i in range(n):
            legal = np.flatnonzero(mask[i])
            u = rs.random()
            if u < 0.05:
                acts.append(int(rs.choice([-1, 45, 99])))
            elif u < 0.12 and len(legal) < 45:
                acts.append(int(rs.choice(np.setdiff1d(np.arange(45), legal))))
            else:
                acts.append(int(rs.choice(legal)) if len(legal) else 0)
        before = dev.eng.obs.clone()
        a = torch.tensor(acts, dtype=torch.int32, device=dev.device)
        od, ard, ood, ord_, dd, info_d = dev.dual_step(a)
        oc, arc, ooc, orc_, dc, info_c = cal.dual_step(a.clone())
        for x, y in ((od, oc), (ard, arc), (ood, ooc), (ord_, orc_), (dd, dc)):
            assert torch.equal(x, y), k
        for key in ("action_mask", "final_observation", "opponent_action", "game_ended_on", "agent_step_reward",
                    "illegal_action", "draw", "turn_limit"):
            assert torch.equal(info_d[key], info_c[key]), (k, key)
        bad = np.array([not (0 <= x < 45) or mask[i][x] == 0 for i, x in enumerate(acts)])
        ill = info_d["illegal_action"].cpu().numpy()
        oob = np.array([not (0 <= x < 45) for x in acts])
        assert np.array_equal(ill, bad & ~oob & (mask.sum(axis=1) > 0)), k
        unchanged = bad & (mask.sum(axis=1) > 0)
        assert (info_d["opponent_action"].cpu().numpy()[unchanged] == -1).all()
        assert torch.equal(od[torch.from_numpy(unchanged).to(od.device)],
                           before[torch.from_numpy(unchanged).to(od.device)])
        r = info_d["agent_step_reward"].cpu().numpy()
        assert np.allclose(r[ill], -0.01)
        seen_illegal += int(ill.sum())
        seen_done += int(dd.sum())
    assert seen_illegal > 50 and seen_done > n


def test_batched_eval_matches_reference_eval_suite():
    """splendor_gym.evaluation.eval_vs_opponent == the reference eval_suite.eval_vs_opponent
    (tests/golden/eval.json) for deterministic agents against greedy_opponent_v1."""
    from splendor_gym.evaluation import eval_vs_opponent, first_legal_policy, last_legal_policy
    with open(os.path.join(GOLD, "eval.json")) as f:
        cases = json.load(f)
    agents = {"first_legal": first_legal_policy, "last_legal": last_legal_policy}
    for c in cases:
        got = eval_vs_opponent(agents[c["agent"]], opponent=c["opponent"], n_games=c["n_games"], seed=c["seed"])
        assert got.pop("unfinished") == 0
        want = c["result"]
        for k in ("n", "wins", "losses", "draws"):
            assert got[k] == want[k], (c["agent"], c["seed"], k, got, want)
        for k in ("win_rate", "win_rate_ci95", "avg_turns", "avg_prestige", "illegal_action_rate"):
            assert got[k] == pytest.approx(want[k], abs=1e-12), (c["agent"], c["seed"], k, got, want)


@pytest.mark.parametrize("policy", [1, 2])
def test_device_scripted_policies(orc, policy):
    """SPL_POLICY_GREEDY_V1 equals the host greedy_opponent_v1 on every table; every
    SPL_POLICY_BASIC_PRIORITY choice lies in the reference's preferred set (its random tie-breaks
    are Philox draws, eval_suite.py:32-78)."""
    import torch
    from splendor_gym.opponents import greedy_opponent_v1
    n = 2048
    e = engine(n, 2)
    e.reset(seeds=range(100, 100 + n))
    a = torch.zeros(n, dtype=torch.int32, device=e.device)
    nxt = torch.zeros_like(a)
    e.sample_uniform(out=a, seed=9, ply=0)
    for k in range(60):
        e.step(a, next_actions=nxt, policy=policy, policy_seed=9, ply=k + 1)
        obs, mask, got = e.obs.cpu().numpy(), e.mask.cpu().numpy(), nxt.cpu().numpy()
        for i in range(0, n, 7):
            info = {"action_mask": mask[i]}
            legal = np.flatnonzero(mask[i])
            if policy == 1:
                assert got[i] == greedy_opponent_v1(obs[i], info), (k, i)
                continue
            if len(legal) == 0:
                assert got[i] == 0
                continue
            vis = legal[(legal >= 15) & (legal <= 26)]
            if len(vis):
                pts = np.array([obs[i][32 + (x - 15) * 13 + 2] for x in vis])
                allowed = vis[pts == pts.max()]
            else:
                allowed = next(legal[(legal >= lo) & (legal <= hi)] for lo, hi in ((42, 44), (0, 9), (10, 14), (27, 41), (0, 44))
                               if len(legal[(legal >= lo) & (legal <= hi)]))
            assert got[i] in allowed, (k, i, got[i], allowed)
        e.sample_uniform(out=a, seed=11, ply=k)  # keep the tables moving with uniform play


def test_fused_gate_equals_spl_dual_gate():
    """spl_step_args_t.gate_* (the dual step's gate inside the opponent's spl_step) equals
    spl_dual_gate followed by a plain spl_step: the same gated actions written back, the same
    outputs and table states, with ended, illegal and out-of-range agent moves mixed in."""
    import ctypes
    import torch
    from splendor_gym import _native
    n, seed = 1000, 21
    a, b = engine(n, 2), engine(n, 2)
    a.reset(seeds=range(seed, seed + n))
    b.reset(seeds=range(seed, seed + n))
    dev = a.device
    rs = np.random.default_rng(4)
    z = lambda dt: torch.zeros(n, dtype=dt, device=dev)
    small_a, small_b = (z(torch.float32), z(torch.uint8), z(torch.uint8), z(torch.int8)), \
        (z(torch.float32), z(torch.uint8), z(torch.uint8), z(torch.int8))
    gated = 0
    for k in range(80):
        mask = a.mask.cpu().numpy()
        acts = [int(rs.choice(np.flatnonzero(m))) if m.any() and rs.random() > 0.1 else int(rs.integers(-2, 50))
                for m in mask]
        act = torch.tensor(acts, dtype=torch.int32, device=dev)
        a.step(act, autoreset=False, final_obs=False, small=small_a)
        b.step(act.clone(), autoreset=False, final_obs=False, small=small_b)
        opp = torch.tensor([int(rs.choice(np.flatnonzero(m))) if m.any() else 0 for m in a.mask.cpu().numpy()],
                           dtype=torch.int32, device=dev)
        oa, ob = opp.clone(), opp.clone()
        with torch.cuda.device(dev):
            _native.check(b.lib, b.lib.spl_dual_gate(n, small_b[1].data_ptr(), small_b[2].data_ptr(), ob.data_ptr(),
                                                     b.stream()))
        b.step(ob, autoreset=2, final_obs=True)
        a.step(oa, autoreset=2, final_obs=True, gate=(small_a[1], small_a[2]))
        assert torch.equal(oa, ob), k
        gated += int((oa == -1).sum())
        for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (k, name)
        term = a.terminated.bool()
        assert torch.equal(a.final_obs[term], b.final_obs[term]), k
    assert a.download().tobytes() == b.download().tobytes()
    assert gated > 100

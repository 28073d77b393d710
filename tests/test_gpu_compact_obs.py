"""Compact observation rows (spl_step_args_t.obs_u8, spl_act_args_t.obs_u8): the agent's move of a
batched dual step writes the opponent's observation as 300-byte rows (the 297 values, move_count
>> 8, two zero bytes) for the pool kernel instead of int32 [n][297] rows.

  * the rows carry exactly the int32 observation spl_step writes for the same state (natural
    play, terminal and re-dealt tables, crafted move_count > 255), byte for byte, and the step's
    other outputs and the table state are the same either way;
  * the fp32 actor (grouped pool kernel, its narrow tails, and spl_policy_act) reads them into the
    same logits and actions as the int32 rows."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def engine(n, players=2):
    from splendor_gym.device import Engine
    e = Engine(n, players)
    return e


def as_obs(rows):
    """int32 [n, 297] observation from compact rows."""
    import torch
    o = rows[:, :297].to(torch.int32)
    o[:, 295] += 256 * rows[:, 297].to(torch.int32)
    return o


@pytest.mark.parametrize("players", [2, 4])
def test_compact_rows_equal_int32_obs(players):
    import torch
    n, seed = 1000, 3  # a ragged last workgroup
    a, b = engine(n, players), engine(n, players)
    a.reset(seeds=range(n))
    b.reset(seeds=range(n))
    dev = a.device
    rows = torch.full((n, 300), 0xAB, dtype=torch.uint8, device=dev)
    act = torch.zeros(n, dtype=torch.int32, device=dev)
    a.sample_uniform(out=act, seed=seed, ply=0)
    for k in range(60):
        na, nb = torch.empty_like(act), torch.empty_like(act)
        a.step(act, next_actions=na, policy_seed=seed, ply=k + 1)
        b.step(act, next_actions=nb, policy_seed=seed, ply=k + 1, obs_u8=rows)
        assert torch.equal(as_obs(rows), a.obs), k
        assert int(rows[:, 298:].abs().sum()) == 0 and int(rows[:, 297].max()) == 0, k
        for name in ("mask", "reward", "terminated", "flags", "winner"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (k, name)
        assert torch.equal(na, nb), k
        act = na
    assert a.download().tobytes() == b.download().tobytes()
    # crafted long games: move_count > 255 on every third table
    recs = a.download()
    big = np.arange(n) % 3 == 0
    recs["move_count"] = np.where(big, 300 + (recs["move_count"] % 2), recs["move_count"])
    a.upload(recs)
    b.upload(recs)
    na, nb = torch.empty_like(act), torch.empty_like(act)
    a.step(act, next_actions=na, policy_seed=seed, ply=99, autoreset=False)
    b.step(act, next_actions=nb, policy_seed=seed, ply=99, autoreset=False, obs_u8=rows)
    assert int(a.obs[:, 295].max()) > 255
    assert torch.equal(as_obs(rows), a.obs)


def test_pool_kernel_reads_compact_rows_like_int32_rows():
    """Grouped greedy (13 networks, full workgroups and narrow tails) and spl_policy_act on the
    same states: identical logits-derived actions from either observation form."""
    import torch
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    from splendor_gym.policy import ActorCritic
    n = 4096 + 77
    a, b = engine(n), engine(n)
    a.reset(seeds=range(10, 10 + n))
    b.reset(seeds=range(10, 10 + n))
    dev = a.device
    rows = torch.zeros((n, 300), dtype=torch.uint8, device=dev)
    act = torch.zeros(n, dtype=torch.int32, device=dev)
    a.sample_uniform(out=act, seed=1, ply=0)
    for k in range(25):
        na = torch.empty_like(act)
        a.step(act, next_actions=na, policy_seed=1, ply=k + 1)
        b.step(act, next_actions=torch.empty_like(act), policy_seed=1, ply=k + 1, obs_u8=rows)
        act = na
    torch.manual_seed(0)
    agent = ActorCritic().to(dev).eval()
    pool = OpponentPool(agent, pool_size=12, p_current=0.25, seed=5)
    for i in range(12):
        torch.manual_seed(100 + i)
        pool.add_snapshot(ActorCritic().to(dev).eval())
    group = torch.randint(0, 13, (n,), dtype=torch.int32, device=dev)
    want = pool.act(a.obs, a.mask, group)
    got = pool.act(rows, b.mask, group)
    assert torch.equal(want, got)
    f = FusedActorCritic(agent)
    w2 = f.greedy(a.obs, a.mask)
    g2 = f.greedy(rows, b.mask)
    assert torch.equal(w2, g2)


@pytest.mark.parametrize("players", [2, 4])
def test_step_writes_both_forms(players):
    """spl_step with obs AND obs_u8 (ABI 8, Engine.step(keep_obs=True)): the int32 rows exactly as a
    step without the copy writes them, the compact rows their byte form (crafted move_count > 255
    included), every other output and the state the same."""
    import torch
    from splendor_gym.selfplay import compact_rows
    n, seed = 1000, 5
    a, b = engine(n, players), engine(n, players)
    a.reset(seeds=range(n))
    b.reset(seeds=range(n))
    dev = a.device
    rows = torch.full((n, 300), 0xCD, dtype=torch.uint8, device=dev)
    act = torch.zeros(n, dtype=torch.int32, device=dev)
    a.sample_uniform(out=act, seed=seed, ply=0)
    for k in range(40):
        na, nb = torch.empty_like(act), torch.empty_like(act)
        a.step(act, next_actions=na, policy_seed=seed, ply=k + 1)
        b.step(act, next_actions=nb, policy_seed=seed, ply=k + 1, obs_u8=rows, keep_obs=True)
        assert torch.equal(a.obs, b.obs), k
        assert torch.equal(as_obs(rows), a.obs), k
        assert torch.equal(rows, compact_rows(a.obs, torch.empty_like(rows))), k
        for name in ("mask", "reward", "terminated", "flags", "winner", "final_obs"):
            assert torch.equal(getattr(a, name), getattr(b, name)), (k, name)
        assert torch.equal(na, nb), k
        act = na
    recs = a.download()
    big = np.arange(n) % 3 == 1
    recs["move_count"] = np.where(big, 260 + (recs["move_count"] % 5), recs["move_count"])
    a.upload(recs)
    b.upload(recs)
    na, nb = torch.empty_like(act), torch.empty_like(act)
    a.step(act, next_actions=na, policy_seed=seed, ply=77, autoreset=False)
    b.step(act, next_actions=nb, policy_seed=seed, ply=77, autoreset=False, obs_u8=rows, keep_obs=True)
    assert int(a.obs[:, 295].max()) > 255
    assert torch.equal(a.obs, b.obs) and torch.equal(as_obs(rows), a.obs)


def test_dual_step_agent_compact_rows_follow_the_observation():
    """DualStepVectorEnv(agent_obs_u8=True): after reset and after every dual step the env's compact
    rows are the byte form of the int32 observation it returns, and the fused actor reads either form
    into the same actions."""
    import torch
    from splendor_gym.fused_policy import FusedActorCritic
    from splendor_gym.policy import ActorCritic
    from splendor_gym.selfplay import DualStepVectorEnv
    n = 3000
    env = DualStepVectorEnv(n, opponent="greedy_v1", agent_obs_u8=True)
    obs, info = env.reset(seed=21)
    torch.manual_seed(4)
    f = FusedActorCritic(ActorCritic().to(env.device).eval())
    for k in range(30):
        assert torch.equal(as_obs(env.agent_obs_u8), obs), k
        mask = info["action_mask"]
        a32, lp32, _, v32 = f.act(obs, mask, seed=3, ply=k)
        a8, lp8, _, v8 = f.act(env.agent_obs_u8, mask, seed=3, ply=k)
        assert torch.equal(a32, a8) and torch.equal(lp32, lp8) and torch.equal(v32, v8), k
        obs, _, _, _, done, info = env.dual_step(a32)

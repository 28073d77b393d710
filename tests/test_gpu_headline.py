"""Full-size and configuration-5 checks on the GPU:

  * the exact headline variant of bench.py (2 players, 65 536 tables, spl_rollout of K = 128 steps,
    pool refill every 64 steps fused into the launch, the quad kernel k_rollout_store_quad_2p — four
    two-wave teams in one 512-thread workgroup per CU, partner hand-off at lead 4 — per-step rollout
    store with non-temporal stores), with the hand-off forced too, and the two-wave kernel
    (k_rollout_store_2p, four workgroups per CU), equal chained spl_step launches bit for bit, and a
    256-table subset of the chain is replayed through the CPU oracle;
  * 4-player sharding invariance (two shards == one engine);
  * BASELINE config 5: batched self-play with the fused fp32 ActorCritic as agent AND opponent
    (DualStepVectorEnv) equals the same loop driven by the torch fp32 module, table by table —
    with random-init networks and with the reference's trained checkpoint.
Reference: scripts/random_rollout.py:13-28, envs/splendor_env.py:51-90, ppo_splendor.py:219-297."""
import numpy as np
import pytest

from oracle.oracle import Oracle, OracleVec

pytestmark = pytest.mark.gpu


def engine(n, P, **kw):
    from splendor_gym.device import Engine
    return Engine(n, P, **kw)


def bits_of(mask_i8):
    m = np.asarray(mask_i8).astype(np.uint64)
    return (m << np.arange(45, dtype=np.uint64)).sum(axis=-1).astype(np.uint64)


def store(K, n, dev):
    import torch
    return {"obs": torch.empty((K, n, 297), dtype=torch.int32, device=dev),
            "mask": torch.empty((K, n, 45), dtype=torch.int8, device=dev),
            "reward": torch.empty((K, n), dtype=torch.float32, device=dev),
            "terminated": torch.empty((K, n), dtype=torch.uint8, device=dev),
            "flags": torch.empty((K, n), dtype=torch.uint8, device=dev),
            "winner": torch.empty((K, n), dtype=torch.int8, device=dev),
            "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev)}


@pytest.mark.parametrize("P,n,R,lead,pipeline", [(2, 65536, 64, None, True), (2, 65536, 64, -1, "always"),
                                                 (2, 65536, 64, None, "quad"), (2, 65536, 64, -1, "quad"),
                                                 (4, 32768, 16, None, True), (4, 32768, 16, -1, True),
                                                 (2, 32768, 64, -1, "dealer2")])
def test_headline_rollout_65536_equals_step_chain_and_oracle(P, n, R, lead, pipeline):
    """bench.py's headline (2p x 65 536: the auto choice, the quad kernel — four two-wave teams in one
    workgroup per CU — with fused refills; and the two-wave kernel at four workgroups per CU, "always")
    and C4's per-GPU share (4p x 32 768 of 262 144 on 8 GPUs: the six-wave dealer, one workgroup per CU)
    at full size: two 128-step rollout launches equal the spl_step chain bit for bit; every 256th table
    is replayed through the CPU oracle.  lead -1 forces the partner hand-off
    whenever a task slot is free: the six-wave dealer and the quad kernel (one
    workgroup per CU, 4 teams: the headline's 65 536 tables in 256 workgroups) then hand rows between
    every pair of workgroups with the most slot reuse their rings allow (dealer2 also at 2p x 32 768),
    and the two-wave kernel ("always", four workgroups per CU), which has no partner hand-off since
    round 5, must hand off nothing."""
    import ctypes
    import torch
    from splendor_gym import _native
    K, seed, launches = 128, 0, 2
    chain = engine(n, P, refill_period=R)
    roll = engine(n, P, refill_period=R, refill_fused=True, pipeline=pipeline, partner_lead=lead)  # bench.py defaults
    want = {"always": "k_rollout_store_2p", "quad": f"k_rollout_store_quad_{P}p",
            "dealer2": f"k_rollout_store_dealer2_{P}p"}.get(pipeline, roll.rollout_kernel_name())
    assert roll.rollout_kernel_name() == want
    multi = want.startswith(("k_rollout_store_dealer2", "k_rollout_store_quad"))  # the partner hand-off runs
    pst = (ctypes.c_uint64 * 2)()
    _native.check(roll.lib, roll.lib.spl_debug_partner_stats(pst, 1))
    chain.reset(seeds=range(n))
    roll.reset(seeds=range(n))
    dev = chain.device
    a_c = torch.zeros(n, dtype=torch.int32, device=dev)
    chain.sample_uniform(out=a_c, seed=seed, ply=0)
    a_r = a_c.clone()
    st = {k: (torch.zeros(n, dtype=torch.float32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev))
          for k in "cr"}
    sub = np.arange(0, n, 256)  # the oracle replays these tables
    vec = OracleVec(Oracle(), len(sub), P, [int(t) for t in sub])
    out = store(K, n, dev)
    for launch in range(launches):
        ply0 = 1 + launch * K
        na = torch.empty_like(a_r)
        roll.rollout(K, actions=a_r, next_actions=na, policy_seed=seed, ply=ply0, out=out,
                     ep_return=st["r"][0], ep_count=st["r"][1])
        a_r = na
        for k in range(K):
            acts = a_c[sub].cpu().numpy().copy()
            na = torch.empty_like(a_c)
            chain.step(a_c, next_actions=na, policy_seed=seed, ply=ply0 + k, ep_return=st["c"][0],
                       ep_count=st["c"][1])
            for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
                assert torch.equal(out[name][k], getattr(chain, name)), (launch, k, name)
            term = chain.terminated.bool()
            assert torch.equal(out["final_obs"][k][term], chain.final_obs[term]), (launch, k)
            ref = vec.step(acts, want_final=True)
            np.testing.assert_array_equal(chain.obs[sub].cpu().numpy(), ref["obs"], err_msg=f"{launch} {k}")
            assert np.array_equal(bits_of(chain.mask[sub].cpu().numpy()), ref["mask"]), (launch, k)
            assert np.array_equal(chain.reward[sub].cpu().numpy(), ref["reward"]), (launch, k)
            assert np.array_equal(chain.flags[sub].cpu().numpy(), ref["flags"]), (launch, k)
            a_c = na
        assert torch.equal(a_r, a_c), launch
    assert torch.equal(st["c"][0], st["r"][0]) and torch.equal(st["c"][1], st["r"][1])
    assert int(st["c"][1].sum()) > (100_000 if n == 65536 else 50_000 if P == 2 else 200_000)  # one episode per ~77 (2p) / ~29 (4p) plies
    assert chain.download().tobytes() == roll.download().tobytes()
    _native.check(roll.lib, roll.lib.spl_debug_partner_stats(pst, 0))
    if multi and lead == -1:
        assert pst[0] > 1000, (pst[0], pst[1])  # many row blocks were stored by the partner
    elif not multi:
        assert pst[0] == 0 and pst[1] == 0, (pst[0], pst[1])


def test_sharded_equals_whole_4p():
    """4 players: two shards (global ids 0..1023, 1024..2047) evolve exactly as one engine of 2048,
    through the rollout kernel and its fused refills (every 16 steps at 4 players)."""
    import torch
    n, half, K, launches = 2048, 1024, 64, 3
    whole = engine(n, 4)
    parts = [engine(half, 4, table0=0), engine(half, 4, table0=half)]
    whole.reset(seeds=range(n))
    parts[0].reset(seeds=range(half))
    parts[1].reset(seeds=range(half, n))
    a_w = torch.zeros(n, dtype=torch.int32, device=whole.device)
    a_p = [torch.zeros(half, dtype=torch.int32, device=whole.device) for _ in parts]
    whole.sample_uniform(out=a_w, seed=9, ply=0)
    for p, a in zip(parts, a_p):
        p.sample_uniform(out=a, seed=9, ply=0)
    for launch in range(launches):
        ow, op = store(K, n, whole.device), [store(K, half, whole.device) for _ in parts]
        na = torch.empty_like(a_w)
        whole.rollout(K, actions=a_w, next_actions=na, policy_seed=9, ply=1 + K * launch, out=ow)
        a_w = na
        for i, p in enumerate(parts):
            na = torch.empty_like(a_p[i])
            p.rollout(K, actions=a_p[i], next_actions=na, policy_seed=9, ply=1 + K * launch, out=op[i])
            a_p[i] = na
        for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
            assert torch.equal(torch.cat([op[0][name], op[1][name]], dim=1), ow[name]), (launch, name)
        assert torch.equal(torch.cat(a_p), a_w)
    assert whole.download().tobytes() == np.concatenate([p.download() for p in parts]).tobytes()


@pytest.mark.parametrize("weights", ["random", "trained"])
def test_selfplay_fused_fp32_actor_matches_torch(weights):
    """Config 5 (ppo_splendor.py:219-297 with the frozen-opponent dual step): 4096 tables x 120
    dual steps, agent = greedy fused fp32 actor, opponent = greedy fused fp32 frozen actor, against
    the same loop with the torch fp32 modules.  Every table must match step for step (obs, masks,
    rewards, done, opponent actions), except tables where one of the two sides met a NEAR TIE — top
    two legal logits within 1e-5 of each other, where the two fp32 summation orders may pick
    different actions; those tables leave the comparison (at most 1 % of them)."""
    import torch
    from splendor_gym.fused_policy import FusedActorCritic
    from splendor_gym.policy import ActorCritic
    from splendor_gym.selfplay import DualStepVectorEnv
    N, steps = 4096, 120
    torch.manual_seed(7)
    agent = ActorCritic().cuda().eval()
    opp = ActorCritic().cuda().eval()
    if weights == "trained":  # the reference's checkpoint for both sides
        import os
        from safetensors.torch import load_file
        sd = load_file(os.path.join(os.path.dirname(__file__), "golden", "ppo_splendor_latest.safetensors"), device="cuda")
        agent.load_state_dict(sd)
        opp.load_state_dict(sd)
    fa = FusedActorCritic(agent, with_critic=True)   # precision fp32
    fo = FusedActorCritic(opp, with_critic=False)
    rec = {}

    def torch_opponent(obs, mask):
        with torch.no_grad():
            lg = opp.actor(obs.float())
        rec["opp_logits"], rec["opp_mask"] = lg, mask.clone()
        return torch.argmax(lg.masked_fill(mask < 1, float("-inf")), dim=-1).to(torch.int32)

    envF = DualStepVectorEnv(N, opponent=fo.opponent())
    envT = DualStepVectorEnv(N, opponent=torch_opponent)
    oF, iF = envF.reset(seed=100)
    oT, iT = envT.reset(seed=100)
    tainted = torch.zeros(N, dtype=torch.bool, device=oF.device)

    def near_tie(logits, mask, rows):
        m = logits[rows].masked_fill(mask[rows] < 1, float("-inf"))
        top2 = torch.topk(m, 2, dim=-1).values
        return ((top2[:, 0] - top2[:, 1]) <= 1e-5).all().item()

    done_total = 0
    for k in range(steps):
        ok = ~tainted
        assert torch.equal(oF[ok], oT[ok]), k
        assert torch.equal(iF["action_mask"][ok], iT["action_mask"][ok]), k
        aF = fa.greedy(oF, iF["action_mask"])
        with torch.no_grad():
            lgT = agent.actor(oT.float())
        aT = torch.argmax(lgT.masked_fill(iT["action_mask"] < 1, float("-inf")), dim=-1).to(torch.int32)
        diff = (aF != aT) & ok
        if diff.any():
            assert near_tie(lgT, iT["action_mask"], diff), k
            tainted |= diff
        oF, rF, _, orF, dF, iF = envF.dual_step(aF)
        oT, rT, _, orT, dT, iT = envT.dual_step(aT)
        ok = ~tainted
        oppF, oppT = iF["opponent_action"], iT["opponent_action"]
        odiff = (oppF != oppT) & ok
        if odiff.any():
            assert near_tie(rec["opp_logits"], rec["opp_mask"], odiff), k
            tainted |= odiff
            ok = ~tainted
        assert torch.equal(rF[ok], rT[ok]) and torch.equal(orF[ok], orT[ok]), k
        assert torch.equal(dF[ok], dT[ok]), k
        assert torch.equal(iF["final_observation"][ok & dF], iT["final_observation"][ok & dT]), k
        done_total += int(dF[ok].sum())
    assert tainted.float().mean().item() <= 0.01, int(tainted.sum())
    assert done_total > 1000  # many games finished and were re-dealt inside the loop


def test_config5_pool_selfplay_at_per_gpu_size_matches_torch():
    """BASELINE config 5 at its per-GPU size (65 536 tables): the fused loop —
    agent = fused fp32 ActorCritic (exact fp32 operands), opponent = OpponentPool with 12 frozen snapshots + the current
    policy drawn per episode (spl_policy_act_grouped) — against the same loop with the torch fp32
    modules (each table's opponent = the network the pool drew for its episode), 40 dual steps.  Per
    table: agent and opponent actions, rewards, done and the next observations equal, except tables
    where either side met a near tie (top two legal logits within 1e-5; at most 1 % leave the
    comparison).  The agent's sampling launch (k_act32<true, true>, the bench's config-5 kernel) is
    run on the same observations every step and its critic value checked against torch (1e-5)."""
    import os
    import torch
    from safetensors.torch import load_file
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    from splendor_gym.policy import ActorCritic
    from splendor_gym.selfplay import DualStepVectorEnv
    N, steps = 65536, 40
    sd = load_file(os.path.join(os.path.dirname(__file__), "golden", "ppo_splendor_latest.safetensors"), device="cuda")
    torch.manual_seed(5)

    def net(noise):
        m = ActorCritic().cuda().eval()
        m.load_state_dict(sd)
        if noise:
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(noise * torch.randn_like(p))
        return m

    agent = net(0.0)
    snaps = [net(0.02) for _ in range(12)]
    pool = OpponentPool(agent, pool_size=12, p_current=0.25, seed=99)
    for m in snaps:
        pool.add_snapshot(m)
    nets = {0: agent}
    nets.update({slot: m for slot, m in zip(pool.pool, snaps)})
    fa = FusedActorCritic(agent, precision="fp32")
    envF = DualStepVectorEnv(N, opponent=pool, opponent_obs=False)
    cur = {}

    def torch_pool(obs, mask):
        groups = cur["groups"]
        act = torch.zeros(obs.shape[0], dtype=torch.int32, device=obs.device)
        lg_all = torch.empty(obs.shape[0], 45, device=obs.device)
        with torch.no_grad():
            for g in torch.unique(groups).tolist():
                rows = groups == g
                lg = nets[g].actor(obs[rows].float())
                lg_all[rows] = lg
                act[rows] = torch.argmax(lg.masked_fill(mask[rows] < 1, float("-inf")), dim=-1).to(torch.int32)
        cur["opp_logits"], cur["opp_mask"] = lg_all, mask.clone()
        return act

    envT = DualStepVectorEnv(N, opponent=torch_pool, opponent_obs=False)
    oF, iF = envF.reset(seed=7)
    oT, iT = envT.reset(seed=7)
    tainted = torch.zeros(N, dtype=torch.bool, device=oF.device)

    def near_tie(logits, mask, rows):
        m = logits[rows].masked_fill(mask[rows] < 1, float("-inf"))
        top2 = torch.topk(m, 2, dim=-1).values
        return ((top2[:, 0] - top2[:, 1]) <= 1e-5).all().item()

    done_total = 0
    max_rel = 0.0  # the agent's logits against torch fp32, over every untainted table of every step
    for k in range(steps):
        ok = ~tainted
        assert torch.equal(oF[ok], oT[ok]) and torch.equal(iF["action_mask"][ok], iT["action_mask"][ok]), k
        with torch.no_grad():
            _, _, _, value = fa.act(oF, iF["action_mask"], seed=3, ply=k)
            vT = agent.get_value(oF.float())
            lgT = agent.actor(oT.float())
        assert torch.allclose(value, vT, rtol=1e-5, atol=1e-5), k
        aF, lgF = fa.greedy(oF, iF["action_mask"], want_logits=True)
        okr = ~tainted
        max_rel = max(max_rel, ((lgF[okr] - lgT[okr]).abs() / (lgT[okr].abs() + 1)).max().item())
        aT = torch.argmax(lgT.masked_fill(iT["action_mask"] < 1, float("-inf")), dim=-1).to(torch.int32)
        diff = (aF != aT) & ok
        if diff.any():
            assert near_tie(lgT, iT["action_mask"], diff), k
            tainted |= diff
        oF, rF, _, orF, dF, iF = envF.dual_step(aF)
        cur["groups"] = iF["episode_opponent_index"].clone()  # the network each table's opponent played
        oT, rT, _, orT, dT, iT = envT.dual_step(aT)
        ok = ~tainted
        odiff = (iF["opponent_action"] != iT["opponent_action"]) & ok
        if odiff.any():
            assert near_tie(cur["opp_logits"], cur["opp_mask"], odiff), k
            tainted |= odiff
            ok = ~tainted
        assert torch.equal(rF[ok], rT[ok]) and torch.equal(orF[ok], orT[ok]) and torch.equal(dF[ok], dT[ok]), k
        done_total += int(dF[ok].sum())
    # the precision of the credited config-5 line, recorded (exact fp32 operands)
    print("config5_precision", {"max_logit_rel_err_vs_torch_fp32": max_rel,
                                "near_tie_tainted_fraction": tainted.float().mean().item(), "tables": N,
                                "dual_steps": steps, "precision": fa.precision})
    assert max_rel <= 1e-5, max_rel
    assert tainted.float().mean().item() <= 0.01, int(tainted.sum())
    assert len(torch.unique(cur["groups"])) == 13  # the current policy and all 12 snapshots played
    assert done_total > 0  # episodes ended, re-dealt and drew their next opponents inside the loop
    envF.close()
    envT.close()

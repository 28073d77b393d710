"""The batched opponent pool of config-5 self-play (ppo_splendor.py:137-143 opponent_supplier,
:366-370 snapshot pool): per-table networks in one grouped launch (spl_policy_act_grouped), the
per-table opponent draw (spl_dual_draw_opponents), and DualStepVectorEnv with an OpponentPool against
per-env DualStepNativeWrapper loops whose opponent_supplier makes the same draws (a host Philox
restatement below) — wrappers/dual_step_native.py:45-79, 90-193."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M32 = 0xFFFFFFFF


def philox4x32(ctr, key):
    """Philox4x32-10 (csrc/spl_rng.h) on Python ints: ctr 4 words, key 2 words."""
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0, p1 = 0xD2511F53 * c0, 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
        k0, k1 = (k0 + 0x9E3779B9) & M32, (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3


def host_draw(seed, table, episode, pool_slots, p_current):
    """The group spl_dual_draw_opponents gives `table` for its `episode`-th draw."""
    r = philox4x32((table & M32, table >> 32, episode & M32, 0x6F70706F), (seed & M32, seed >> 32))
    u = np.float32(r[0] >> 8) * np.float32(1.0 / 16777216.0)
    if not pool_slots or u < np.float32(p_current):
        return 0
    return pool_slots[(r[1] * len(pool_slots)) >> 32]


def models(k, seed=0):
    import torch
    from splendor_gym.policy import ActorCritic
    torch.manual_seed(seed)
    return [ActorCritic().cuda().eval() for _ in range(k)]


def states(n, seed=5, plies=10):
    import torch
    from splendor_gym.device import Engine
    e = Engine(n, 2)
    e.reset(seeds=range(seed, seed + n))
    a = torch.zeros(n, dtype=torch.int32, device=e.device)
    e.sample_uniform(out=a, seed=seed, ply=0)
    for k in range(plies):
        e.step(a, next_actions=a, policy_seed=seed, ply=k + 1)
    return e.obs.clone(), e.mask.clone()


def test_grouped_act_equals_each_network():
    """Tables spread over 4 networks (current + 3 snapshots) by an arbitrary per-table index: every
    table's action equals that network's own FusedActorCritic greedy action, bit for bit."""
    import torch
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    ms = models(4, seed=3)
    pool = OpponentPool(ms[0], pool_size=3)
    for m in ms[1:]:
        pool.add_snapshot(m)
    assert pool.pool == [1, 2, 3]
    n = 5000
    obs, mask = states(n)
    g = torch.randint(0, 4, (n,), dtype=torch.int32, device=obs.device)
    g[:700] = 2  # a large group, a partial workgroup at the end of each group
    act = pool.act(obs, mask, g)
    for i, m in enumerate(ms):
        want = FusedActorCritic(m, with_critic=False).greedy(obs, mask)
        sel = g == i
        assert torch.equal(act[sel], want[sel]), i
    g2 = torch.full((n,), -1, dtype=torch.int32, device=obs.device)  # outside the images: untouched
    out = torch.full((n,), 77, dtype=torch.int32, device=obs.device)
    pool.act(obs, mask, g2, out=out)
    assert (out == 77).all()


@pytest.mark.parametrize("n", [5000, 65536])
def test_grouped_sampling_and_logits_equal_each_network(n):
    """spl_policy_act_grouped in SAMPLE mode with logits: full 128-table workgroups (k_act32) and the
    16-table tail workgroups (k_act32_narrow, hidden units split over the waves, weights from global
    memory) give every table exactly its own network's logits, action and log-prob — the draw is
    keyed by the table id, so it equals the per-network launch's."""
    import ctypes
    import torch
    from splendor_gym import _native
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    ms = models(5, seed=8)
    pool = OpponentPool(ms[0], pool_size=4)
    for m in ms[1:]:
        pool.add_snapshot(m)
    obs, mask = states(n, seed=2)
    g = torch.randint(0, 5, (n,), dtype=torch.int32, device=obs.device)
    act = torch.empty(n, dtype=torch.int32, device=obs.device)
    lp = torch.empty(n, dtype=torch.float32, device=obs.device)
    ent = torch.empty(n, dtype=torch.float32, device=obs.device)
    lg = torch.empty(n, 45, dtype=torch.float32, device=obs.device)
    nb = int(pool.lib.spl_policy_group_scratch_bytes(n, pool.n_images))
    scratch = torch.zeros(nb, dtype=torch.uint8, device=obs.device)
    a = _native.ActArgs(obs=obs.data_ptr(), mask=mask.data_ptr(), action=act.data_ptr(), logprob=lp.data_ptr(),
                        entropy=ent.data_ptr(), value=None, logits=lg.data_ptr(), seed=41, ply=3, ply_base=None,
                        table0=0, mode=_native.ACT_SAMPLE, image=_native.PREC_FP32 << 1)
    _native.check(pool.lib, pool.lib.spl_policy_act_grouped(pool.images.data_ptr(), pool.image_bytes, pool.n_images,
                                                            g.data_ptr(), scratch.data_ptr(), n, ctypes.byref(a),
                                                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    for i, m in enumerate(ms):
        f = FusedActorCritic(m, with_critic=False)
        wa, wl, we, _, wlg = f.act(obs, mask, seed=41, ply=3, want_logits=True)
        sel = g == i
        assert torch.equal(lg[sel], wlg[sel]), i
        assert torch.equal(act[sel], wa[sel]) and torch.equal(lp[sel], wl[sel]) and torch.equal(ent[sel], we[sel]), i


def test_draw_matches_host_and_statistics():
    import torch
    from splendor_gym.fused_policy import OpponentPool
    (m,) = models(1)
    pool = OpponentPool(m, pool_size=12, p_current=0.25, seed=77)
    n = 1 << 16
    grp = torch.zeros(n, dtype=torch.int32, device="cuda")
    ep = torch.zeros(n, dtype=torch.int32, device="cuda")
    pool.draw(grp, ep, table0=1000)
    assert (grp == 0).all()  # empty pool: always the current policy
    for _ in range(14):
        pool.add_snapshot()  # ring of 14 snapshot slots, pool keeps the last 12
    assert len(pool.pool) == 12 and pool.pool == list(range(3, 15))
    draw = (torch.arange(n, device="cuda") % 3 == 0).to(torch.uint8)
    pool.draw(grp, ep, draw, table0=1000)
    g = grp.cpu().numpy()
    e = ep.cpu().numpy()
    assert (e == 1 + (np.arange(n) % 3 == 0)).all()
    sel = np.arange(n) % 3 == 0
    frac_cur = (g[sel] == 0).mean()
    assert abs(frac_cur - 0.25) < 4 * np.sqrt(0.25 * 0.75 / sel.sum())
    counts = np.bincount(g[sel], minlength=15)[3:15]
    assert counts.min() > 0.6 * counts.mean()
    for t in list(range(0, 60, 3)) + [n - 4]:
        assert g[t] == host_draw(77, 1000 + t, 1, pool.pool, 0.25), t
    assert (g[~sel] == 0).all()


def test_pool_self_play_matches_per_env_wrappers():
    """DualStepVectorEnv(opponent=OpponentPool) == per-env DualStepNativeWrapper loops whose
    opponent_supplier draws the same network for each episode (host_draw), each network played by
    its own single-table FusedActorCritic greedy call, with the PPO loop's reset after done."""
    import torch
    from splendor_gym.envs import SplendorEnv
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    from splendor_gym.selfplay import DualStepVectorEnv
    from splendor_gym.wrappers import DualStepNativeWrapper
    ms = models(3, seed=11)
    pool = OpponentPool(ms[0], pool_size=2, p_current=0.4, seed=5)
    pool.add_snapshot(ms[1])
    pool.add_snapshot(ms[2])
    fused = {0: FusedActorCritic(ms[0], with_critic=False), 1: FusedActorCritic(ms[1], with_critic=False),
             2: FusedActorCritic(ms[2], with_critic=False)}
    n, steps, seed = 256, 140, 300  # >= 256 tables

    def greedy_of(net):
        def policy(obs, info):
            o = torch.as_tensor(obs, dtype=torch.int32, device="cuda").reshape(1, 297).contiguous()
            k = torch.as_tensor(info["action_mask"], dtype=torch.int8, device="cuda").reshape(1, 45).contiguous()
            return int(fused[net].greedy(o, k)[0].item())
        return policy

    def supplier_for(i):
        count = [0]

        def supplier():
            g = host_draw(5, i, count[0], pool.pool, 0.4)
            count[0] += 1
            supplier.groups.append(g)
            return greedy_of(g)
        supplier.groups = []
        return supplier

    vec = DualStepVectorEnv(n, opponent=pool)
    obs_v, info_v = vec.reset(seed=seed)
    sups = [supplier_for(i) for i in range(n)]
    envs = [DualStepNativeWrapper(SplendorEnv(), opponent_policy=None, opponent_supplier=sups[i], random_starts=True)
            for i in range(n)]
    per = [w.reset(seed=seed + i) for i, w in enumerate(envs)]
    assert info_v["opponent_index"].cpu().tolist() == [s.groups[0] for s in sups]
    ended = 0
    for k in range(steps):
        acts = [int(np.flatnonzero(p[1]["action_mask"])[-1]) if p[1]["action_mask"].any() else 0 for p in per]
        ao, ar, oo, orr, done, info_v = vec.dual_step(torch.tensor(acts, dtype=torch.int32, device=vec.device))
        for i, w in enumerate(envs):
            a_obs, a_rew, o_obs, o_rew, d, inf = w.dual_step(acts[i])
            assert bool(done[i]) == bool(d), (k, i)
            assert float(ar[i]) == pytest.approx(a_rew) and float(orr[i]) == pytest.approx(o_rew), (k, i)
            if d:
                ended += 1
                per[i] = w.reset()
            else:
                per[i] = (a_obs, inf)
            assert np.array_equal(ao[i].cpu().numpy(), per[i][0]), (k, i)
        assert info_v["opponent_index"].cpu().tolist() == [s.groups[-1] for s in sups], k
    assert ended >= n
    assert len({g for s in sups for g in s.groups}) == 3  # all three networks played


def test_snapshot_in_play_is_not_overwritten():
    """a snapshot that left the pool must keep its weights while a table's running episode
    still plays it; add_snapshot skips busy slots (and grows the ring when all are busy)."""
    import torch
    from splendor_gym.fused_policy import OpponentPool
    ms = models(6, seed=21)
    pool = OpponentPool(ms[0], pool_size=1, p_current=0.0, seed=1)  # ring of 3 snapshot slots
    playing = torch.zeros(8, dtype=torch.int32, device="cuda")
    pool.track(playing)
    pool.add_snapshot(ms[1])
    first = pool.pool[0]
    playing[3] = first  # table 3's episode plays the first snapshot
    img = pool.images[first * pool.image_bytes:(first + 1) * pool.image_bytes].clone()
    for m in ms[2:]:
        pool.add_snapshot(m)  # the first leaves the pool at once (pool_size 1)
        assert first not in pool.pool
        assert torch.equal(pool.images[first * pool.image_bytes:(first + 1) * pool.image_bytes], img)
    assert pool.n_images == 1 + 1 + 2  # one busy slot fits the ring: no growth needed
    # every non-member slot busy: the ring grows instead of overwriting
    playing[:3] = torch.tensor([s for s in range(1, pool.n_images) if s not in pool.pool and s != first][:3],
                               dtype=torch.int32)
    n0 = pool.n_images
    pool.add_snapshot(ms[1])
    assert pool.n_images == n0 + 1 and pool.pool[-1] == n0
    assert torch.equal(pool.images[first * pool.image_bytes:(first + 1) * pool.image_bytes], img)
    playing.zero_()
    pool.add_snapshot(ms[2])  # nothing busy: the ring position moves on, reusing freed slots
    assert pool.pool[-1] != n0


def test_grouped_calls_reuse_their_scratch():
    """Back-to-back grouped calls on ONE scratch block with different groupings (and group counts of
    zero): the placing kernel derives each call's group starts itself and its last workgroup zeroes
    the counts, cursors and ticket for the next call — every call must still give each table its own
    network's action."""
    import torch
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    ms = models(4, seed=21)
    pool = OpponentPool(ms[0], pool_size=3)
    for m in ms[1:]:
        pool.add_snapshot(m)
    n = 3000
    obs, mask = states(n, seed=5)
    want = [FusedActorCritic(m, with_critic=False).greedy(obs, mask) for m in ms]
    gen = torch.Generator(device="cpu").manual_seed(3)
    for call in range(4):
        hi = 4 if call != 2 else 2  # call 2 leaves groups 2 and 3 empty
        g = torch.randint(0, hi, (n,), generator=gen, dtype=torch.int32).to(obs.device)
        out = pool.act(obs, mask, g)
        for i in range(4):
            sel = g == i
            assert torch.equal(out[sel], want[i][sel]), (call, i)


def test_grouped_act_at_the_maximum_network_count():
    """A pool at its largest (pool_size 61: 64 images, the grouping kernels' LDS tables and the
    act launch's counter reset at their bounds): every table's action equals its network's own."""
    import torch
    from splendor_gym.fused_policy import FusedActorCritic, OpponentPool
    ms = models(4, seed=31)
    pool = OpponentPool(ms[0], pool_size=61)
    assert pool.n_images == pool.MAX_IMAGES
    for i in range(61):  # the snapshots cycle through three networks
        pool.add_snapshot(ms[1 + i % 3])
    assert len(pool.pool) == 61
    slots = [0] + list(pool.pool)  # image slot of the current policy, then of each snapshot
    net_of = {0: 0} | {slot: 1 + i % 3 for i, slot in enumerate(pool.pool)}
    n = 6000
    obs, mask = states(n, seed=9)
    want = [FusedActorCritic(m, with_critic=False).greedy(obs, mask) for m in ms]
    gen = torch.Generator(device="cpu").manual_seed(11)
    for call in range(2):
        pick = torch.randint(0, len(slots), (n,), generator=gen)
        g = torch.tensor(slots, dtype=torch.int32)[pick].to(obs.device)
        out = pool.act(obs, mask, g)
        gi = g.cpu().numpy()
        for slot in slots:
            sel = torch.from_numpy(gi == slot).to(obs.device)
            if sel.any():
                assert torch.equal(out[sel], want[net_of[slot]][sel]), (call, slot)

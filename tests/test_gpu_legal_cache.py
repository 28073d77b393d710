"""The legal-mask cache (ABI 9; csrc/spl_layout.h).

Every kernel that stores table state also stores legal_moves of that state (engine/rules.py:40-93)
tagged with its context, or "unknown" (tag 0: a crafted upload); spl_step answers the pre-step
check of envs/splendor_env.py:55-66 (any legal move? is the action legal?) from it instead of
evaluating legal_moves.  A stale entry would silently change which moves count as illegal, so:
  * after every writer (reset, step, each rollout kernel shape, refill, upload) the cache equals
    spl_legal of the stored state and carries the context's tag, or tag 0 after an upload;
  * chains that mix writers (rollout launches of every shape between spl_step calls) equal a pure
    spl_step chain bit for bit;
  * a crafted upload followed by a step is judged on the NEW state (an action legal only before
    the edit is illegal after it, and the reverse), as the oracle says;
  * a new card table (another context) never reuses the old context's masks.
"""
import numpy as np
import pytest

from oracle.oracle import Oracle, table_to_view

pytestmark = pytest.mark.gpu


def engine(n, P, **kw):
    from splendor_gym.device import Engine
    return Engine(n, P, **kw)


def bits_of(mask_i8):
    m = np.asarray(mask_i8).astype(np.uint64)
    return (m << np.arange(45, dtype=np.uint64)).sum(axis=-1).astype(np.uint64)


def cache_of(e):
    """(mask u64 [n], tag u32 [n]) read from the arena's legal-mask region: the last 2n u32 words of
    spl_arena_bytes, each plane 256-byte aligned (spl_layout.h arena_layout)."""
    import torch
    e.torch.cuda.synchronize(e.device)
    n = e.n
    off = e.arena.numel() - (8 * n + 255) // 256 * 256
    w = e.arena[off:off + 8 * n].view(torch.int32).cpu().numpy().view(np.uint32)
    lo, hi = w[:n].astype(np.uint64), w[n:].astype(np.uint64)
    return lo | ((hi & np.uint64(0x1FFF)) << np.uint64(32)), (hi >> np.uint64(16)).astype(np.uint32)


def check_cache(e, where, unknown=()):
    """The cache equals spl_legal of every stored non-terminal state, all under one nonzero tag
    (the context's), except tables in `unknown` (tag 0)."""
    import torch
    got, tag = cache_of(e)
    ref = bits_of(e.legal(out=torch.empty((e.n, 45), dtype=torch.int8, device=e.device)).cpu().numpy())
    recs = e.download()
    term = (recs["game_over"] != 0) & (recs["to_play"] == 0)
    known = np.ones(e.n, bool)
    known[list(unknown)] = False
    assert (tag[~known] == 0).all(), where
    tags = set(tag[known].tolist())
    assert len(tags) == 1 and 0 not in tags, (where, sorted(tags)[:4])
    live = known & ~term
    bad = np.flatnonzero(got[live] != ref[live])
    assert bad.size == 0, (where, np.flatnonzero(live)[bad[:8]])
    return tags.pop()


@pytest.mark.parametrize("P,pipeline", [(2, "quad"), (2, "always"), (2, False), (4, "dealer2"), (3, "dealer"),
                                        (4, "quad")])
def test_every_writer_leaves_the_legal_mask_of_the_stored_state(P, pipeline):
    import torch
    n, seed = 1024, 5
    e = engine(n, P, refill_period=16, pipeline=pipeline)
    e.reset(seeds=range(n))
    tag = check_cache(e, "reset(seed)")
    a = torch.zeros(n, dtype=torch.int32, device=e.device)
    e.sample_uniform(out=a, seed=seed, ply=0)
    for k in range(40):  # spl_step with autoreset and the device policy (several episodes end)
        na = torch.empty_like(a)
        e.step(a, next_actions=na, policy_seed=seed, ply=1 + k)
        a = na
    assert check_cache(e, "step") == tag
    na = torch.empty_like(a)
    e.rollout(32, actions=a, next_actions=na, policy_seed=seed, ply=100)
    assert check_cache(e, f"rollout {pipeline}") == tag
    e.refill()
    e.reset(seeds=None)  # pool flip
    assert check_cache(e, "reset()") == tag
    mask = torch.zeros(n, dtype=torch.uint8, device=e.device)
    mask[::3] = 1
    e.reset(seeds=range(n), mask=mask)  # partial reset: the other tables keep their state and entry
    assert check_cache(e, "partial reset") == tag
    recs = e.download(7, 2)
    e.upload(recs, first=7)
    check_cache(e, "upload", unknown=(7, 8))
    e.step(e.legal().to(torch.int32).argmax(dim=1).to(torch.int32))
    assert check_cache(e, "step after upload") == tag


@pytest.mark.parametrize("P,pipeline,K", [(2, "quad", 16), (2, "always", 16), (2, False, 8), (4, "dealer2", 16),
                                          (3, "dealer", 8), (2, "dealer2", 8)])
def test_chains_mixing_rollouts_and_steps_equal_the_step_chain(P, pipeline, K):
    """rollout(K) launches of each kernel shape alternated with K spl_step calls (each step's pre-check
    then reads the mask the rollout stored) equal 2K-step spl_step chains bit for bit."""
    import torch
    n, seed = 1024, 3
    chain = engine(n, P, refill_period=16)
    mixed = engine(n, P, refill_period=16, pipeline=pipeline)
    chain.reset(seeds=range(n))
    mixed.reset(seeds=range(n))
    a_c = torch.zeros(n, dtype=torch.int32, device=chain.device)
    chain.sample_uniform(out=a_c, seed=seed, ply=0)
    a_m = a_c.clone()
    ply = 1
    for rnd in range(3):
        for k in range(K):
            na = torch.empty_like(a_c)
            chain.step(a_c, next_actions=na, policy_seed=seed, ply=ply + k)
            a_c = na
        na = torch.empty_like(a_m)
        mixed.rollout(K, actions=a_m, next_actions=na, policy_seed=seed, ply=ply)
        a_m = na
        assert torch.equal(a_m, a_c), rnd
        ply += K
        for k in range(K):
            nc, nm = torch.empty_like(a_c), torch.empty_like(a_m)
            chain.step(a_c, next_actions=nc, policy_seed=seed, ply=ply + k)
            mixed.step(a_m, next_actions=nm, policy_seed=seed, ply=ply + k)
            for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
                assert torch.equal(getattr(chain, name), getattr(mixed, name)), (rnd, k, name)
            a_c, a_m = nc, nm
        ply += K
    assert chain.download().tobytes() == mixed.download().tobytes()


def test_crafted_upload_then_step_is_judged_on_the_new_state():
    """Tables stepped (cache written), then edited through upload so that the action legal BEFORE
    the edit is illegal after it (table 0) and an action illegal before is legal after (table 1):
    the step flags and rewards follow the new state, and the whole step equals the oracle's."""
    import torch
    from splendor_gym import _native
    from schema import canon
    o = Oracle()
    n = 64
    e = engine(n, 2, refill_period=0)
    e.reset(seeds=range(n))
    a = torch.zeros(n, dtype=torch.int32, device=e.device)
    e.sample_uniform(out=a, seed=1, ply=0)
    e.step(a, autoreset=False)
    before = e.legal().cpu().numpy().copy()
    recs = e.download(0, 2)
    # table 0: the bank is emptied, so every take is illegal; pick a take legal before
    take0 = int(np.flatnonzero(before[0][:10])[0])
    recs[0]["bank"][:5] = 0
    # table 1: the mover gets enough tokens of every colour to buy board slot 0 (action 15)
    assert before[1][15] == 0  # the mover of table 1 holds nothing yet
    tp = int(recs[1]["to_play"])
    recs[1]["players"][tp]["tokens"][:6] = [7, 7, 7, 7, 7, 0]
    recs[1]["bank"][:5] = 0
    e.upload(recs, first=0)
    acts = torch.tensor([take0, 15] + [0] * (n - 2), dtype=torch.int32, device=e.device)
    views = [table_to_view(r) for r in e.download(0, 2)]
    e.step(acts, autoreset=False)
    flags = e.flags.cpu().numpy()
    assert flags[0] & _native.F_ILLEGAL and float(e.reward[0]) == pytest.approx(-0.01)
    assert not flags[1] & _native.F_ILLEGAL
    after = e.download(0, 2)
    for i, act in enumerate((take0, 15)):
        ref = o.env_step(views[i], act)
        np.testing.assert_array_equal(e.obs[i].cpu().numpy(), ref["obs"])
        assert canon(table_to_view(after[i])) == canon(ref["after"]), i


def test_a_new_card_table_does_not_reuse_the_old_contexts_masks():
    """The cache is tagged per card table: after set_card_table the old entries are not this context's,
    so the next step evaluates legal_moves under the edited table (a card made free is buyable)."""
    import torch
    from splendor_gym import _native
    from splendor_gym.engine.state import load_tables
    n = 64
    e = engine(n, 2, refill_period=0)
    e.reset(seeds=range(n))
    _, tag0 = cache_of(e)
    recs = e.download(0, 1)
    card = int(recs[0]["board"][0])
    cards, _ = load_tables()
    cards = np.array(cards, np.int32).copy()
    cards[card, 3:8] = 0  # board slot 0's card costs nothing: buying it (action 15) is legal
    before = e.legal().cpu().numpy()[0].copy()
    assert before[15] == 0
    e.set_card_table(cards)
    _, tag1 = cache_of(e)
    assert (tag1 == tag0).all()  # nothing rewritten by the switch itself
    acts = torch.zeros(n, dtype=torch.int32, device=e.device)
    acts[0] = 15
    e.step(acts, autoreset=False)
    assert not int(e.flags[0]) & _native.F_ILLEGAL
    _, tag2 = cache_of(e)
    assert (tag2 != tag0).all() and len(set(tag2.tolist())) == 1


def test_equal_card_tables_share_the_tag_and_an_edit_back_trusts_it_again():
    """The tag belongs to the card table's contents (card_table_tag in spl_engine.hip): a second engine on the
    canonical table carries the same tag, an edited table another, and switching back to the canonical
    table (a new context) trusts the entries the first context wrote — and they are still exact."""
    from splendor_gym.engine.state import load_tables
    n = 256
    e = engine(n, 2, refill_period=0)
    e.reset(seeds=range(n))
    tag0 = check_cache(e, "reset")
    f = engine(64, 2, refill_period=0)
    f.reset(seeds=range(64))
    assert check_cache(f, "second engine, canonical table") == tag0
    cards, _ = load_tables()
    cards = np.array(cards, np.int32).copy()
    cards[0, 3] += 1  # one cost edited: a different table
    e.set_card_table(cards)
    e.step(e.sample_uniform(seed=3, ply=1), autoreset=False)
    tag_edit = check_cache(e, "step under the edited table")
    assert tag_edit not in (0, tag0)
    e.set_card_table(None)  # back to the canonical table: a new context with the canonical tag
    e.step(e.sample_uniform(seed=3, ply=2), autoreset=False)
    assert check_cache(e, "step back under the canonical table") == tag0


@pytest.mark.parametrize("P,n,other", [(2, 4096, 1), (2, 65536, 1), (4, 2048, 1), (3, 1000, 1),
                                       (2, 4096, 2), (2, 65536, 2), (4, 2048, 2), (3, 1000, 2)])
def test_step_shapes_are_bit_identical(P, n, other):
    """spl_step's kernel shapes (spl_ctx_set_step_tail: 0 two waves; 1 three, the tail wave evaluating the
    new state's legal mask, storing the mask block, drawing the fused policy's action and writing the
    legal-mask cache; 2 two waves with the output wave doing that between its row stores) give the same
    outputs bit for bit, step by step, with autoreset, final observations and the device policy."""
    import torch
    seed = 9
    two = engine(n, P, refill_period=16, step_tail=0)
    three = engine(n, P, refill_period=16, step_tail=other)
    for e in (two, three):
        e.reset(seeds=range(n))
    a2 = torch.zeros(n, dtype=torch.int32, device=two.device)
    two.sample_uniform(out=a2, seed=seed, ply=0)
    a3 = a2.clone()
    for k in range(48):
        n2, n3 = torch.empty_like(a2), torch.empty_like(a3)
        two.step(a2, next_actions=n2, policy_seed=seed, ply=k + 1)
        three.step(a3, next_actions=n3, policy_seed=seed, ply=k + 1)
        for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
            assert torch.equal(getattr(two, name), getattr(three, name)), (k, name)
        term = two.terminated.bool()
        assert torch.equal(two.final_obs[term], three.final_obs[term]), k
        assert torch.equal(n2, n3), k
        a2, a3 = n2, n3
    assert two.download().tobytes() == three.download().tobytes()
    assert check_cache(two, "two waves") == check_cache(two, "two waves")
    check_cache(three, "three waves")

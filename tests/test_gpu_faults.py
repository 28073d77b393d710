"""A lost hand-off in the dealer rollout is reported, not silent.

The three-wave dealer variant of spl_rollout (k_rollout_*_dealer_<P>p) hands off through LDS counters
with bounded waits.  spl_debug_set_spin_limit(0) makes the first wait that has to wait run out, which
must fault the launch loudly: SPL_F_FAULT in the flags of the steps that were not stored, the launch's
serial in the context's host-mapped fault word (spl_ctx_faults), LaunchFault from Engine and from
SplendorVectorEnv — and after a reset + clear_faults the engine runs bit-exact again.
"""
import pytest

pytestmark = pytest.mark.gpu


def _out(torch, K, n, dev):
    return {"obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev),
            "mask": torch.zeros((K, n, 45), dtype=torch.int8, device=dev),
            "reward": torch.zeros((K, n), dtype=torch.float32, device=dev),
            "terminated": torch.zeros((K, n), dtype=torch.uint8, device=dev),
            "flags": torch.zeros((K, n), dtype=torch.uint8, device=dev),
            "winner": torch.zeros((K, n), dtype=torch.int8, device=dev),
            "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev)}


def _forced_fault_rollout(eng, K, a, na, out):
    """One rollout launch with the hand-off spin limit at 0 (restored afterwards)."""
    import torch
    from splendor_gym import _native
    lib = eng.lib
    _native.check(lib, lib.spl_debug_set_spin_limit(0))
    try:
        eng.rollout(K, actions=a, next_actions=na, policy_seed=1, ply=1, out=out)
        torch.cuda.synchronize(eng.device)
    finally:
        _native.check(lib, lib.spl_debug_set_spin_limit(-1))


@pytest.mark.parametrize("P,pipeline,lead", [(2, "dealer", None), (4, "dealer", None), (4, "dealer2", None),
                                              (4, "dealer2", -1), (2, "dealer2", -1)])
def test_dealer_handoff_timeout_is_reported_and_recoverable(P, pipeline, lead):
    """... and with the six-wave dealer's partner hand-off forced (lead -1): a faulting
    output wave posts DONE and stores the rows of the steps it had handed to its partner and the partner
    had not taken, so EVERY step whose flags lack SPL_F_FAULT holds the rows a clean launch writes."""
    import torch
    from splendor_gym import _native
    from splendor_gym.device import Engine
    n, K = 1024, 16
    dev = torch.device("cuda", torch.cuda.current_device())
    # the clean launch from the same deals (three-wave dealer, no partner hand-off)
    clean = Engine(n, P, refill_period=16, pipeline="dealer")
    clean.reset(seeds=range(n))
    a_c = torch.zeros(n, dtype=torch.int32, device=dev)
    clean.sample_uniform(out=a_c, seed=1, ply=0)
    out_c = _out(torch, K, n, dev)
    clean.rollout(K, actions=a_c, next_actions=torch.empty_like(a_c), policy_seed=1, ply=1, out=out_c)
    eng = Engine(n, P, refill_period=16, pipeline=pipeline, partner_lead=lead)
    assert eng.rollout_kernel_name(per_step=True) == f"k_rollout_store_{pipeline}_{P}p"
    eng.reset(seeds=range(n))
    a = torch.zeros(n, dtype=torch.int32, device=dev)
    na = torch.empty_like(a)
    eng.sample_uniform(out=a, seed=1, ply=0)
    assert eng.faults() == 0
    out = _out(torch, K, n, dev)
    _forced_fault_rollout(eng, K, a, na, out)
    f = eng.faults()
    assert f != 0 and f == int(eng.lib.spl_ctx_launches(eng.ctx)), "the faulting launch's serial is reported"
    faulted = (out["flags"] & _native.F_FAULT) != 0
    assert bool(faulted.any()), "steps that were not stored carry SPL_F_FAULT"
    # a faulted workgroup marks every step from the one it did not store on, for all its tables
    first = faulted.to(torch.int32).argmax(dim=0)
    tail = torch.arange(K, device=dev)[:, None] >= first[None, :]
    assert bool((faulted == (tail & faulted.any(dim=0)[None, :])).all())
    # every step not flagged was stored, whoever stored its rows
    ok = ~faulted
    for name in ("obs", "mask", "reward", "terminated", "winner"):
        assert torch.equal(out[name][ok], out_c[name][ok]), name
    assert torch.equal(out["flags"][ok], out_c["flags"][ok])
    clean.close()
    # Engine reports it loudly on the next use, without a synchronisation of its own
    with pytest.raises(_native.LaunchFault):
        eng.rollout(K, actions=a, next_actions=na, policy_seed=1, ply=1 + K, out=out)
    with pytest.raises(_native.LaunchFault):
        eng.download(0, 1)
    # recovery: reset every table, clear, and the engine matches a fresh one bit for bit
    eng.reset(seeds=range(n))
    eng.clear_faults()
    assert eng.faults() == 0
    ref = Engine(n, P, refill_period=16, pipeline="dealer")  # the three-wave variant as the reference
    ref.reset(seeds=range(n))
    a_r = torch.zeros_like(a)
    ref.sample_uniform(out=a_r, seed=1, ply=0)
    a.copy_(a_r)
    out_r = _out(torch, K, n, dev)
    out.update(_out(torch, K, n, dev))
    na_r = torch.empty_like(a)
    eng.rollout(K, actions=a, next_actions=na, policy_seed=1, ply=1, out=out)
    ref.rollout(K, actions=a_r, next_actions=na_r, policy_seed=1, ply=1, out=out_r)
    torch.cuda.synchronize(dev)
    assert eng.faults() == 0 and ref.faults() == 0
    for name in ("obs", "mask", "reward", "terminated", "flags", "winner"):
        assert torch.equal(out[name], out_r[name]), name
    assert not bool(((out["flags"] & _native.F_FAULT) != 0).any())
    assert torch.equal(na, na_r)
    assert eng.download().tobytes() == ref.download().tobytes()


def test_vector_env_raises_on_a_faulted_launch():
    """SplendorVectorEnv checks its engine's fault word on every step (no sync) and raises; reset() is
    the recovery: it re-deals every table, clears the fault and reports its serial in
    info["recovered_fault"], and the env steps cleanly afterwards."""
    import torch
    from splendor_gym import _native
    from splendor_gym.vector import SplendorVectorEnv
    n, K = 1024, 16
    for mode in ("sync", "deferred"):
        env = SplendorVectorEnv(n, num_players=4, check_actions=mode)
        # the auto rollout shape at this size is the dealer variant (<= 2 workgroups per CU)
        assert "dealer" in env.engine.rollout_kernel_name(per_step=True)
        env.reset(seed=0)
        acts = env.sample_actions(seed=2)
        env.step(acts)  # a clean step
        a = torch.zeros(n, dtype=torch.int32, device=env.device)
        env.engine.sample_uniform(out=a, seed=3, ply=0)
        _forced_fault_rollout(env.engine, K, a, torch.empty_like(a), _out(torch, K, n, env.device))
        serial = env.engine.faults()
        assert serial != 0
        with pytest.raises(_native.LaunchFault):
            env.step(env.sample_actions(seed=4))
        _, info = env.reset(seed=0)
        assert info["recovered_fault"] == serial and env.engine.faults() == 0
        obs, rew, term, trunc, info = env.step(env.sample_actions(seed=5))
        assert env.engine.faults() == 0 and "recovered_fault" not in info
        env.close()

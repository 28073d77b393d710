"""Child process of tests/test_gpu_bounds_check.py: runs parity workloads on the BOUNDS-CHECK build
of the engine (SPLENDOR_AMD_LIB -> libsplendor_amd_checked.so) and prints the recorded invariant
violations as JSON.  Test infrastructure only."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd"), os.path.join(HERE, "golden")]

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.oracle import Oracle, OracleVec, view_to_table  # noqa: E402
from splendor_gym import _native  # noqa: E402
from splendor_gym.device import Engine  # noqa: E402


def main():
    lib = _native.load_library()
    flags = ctypes.c_uint32()
    _native.check(lib, lib.spl_debug_bounds_flags(ctypes.byref(flags), 1))
    orc = Oracle()
    out = {"steps": 0}
    # 2 players: device policy with injected illegal / out-of-range actions, autoreset, refills
    n, seed = 1024, 77
    e = Engine(n, 2, refill_period=8)
    e.reset(seeds=range(seed, seed + n))
    vec = OracleVec(orc, n, 2, list(range(seed, seed + n)))
    rs = np.random.default_rng(seed)
    na = torch.zeros(n, dtype=torch.int32, device=e.device)
    e.sample_uniform(out=na, seed=seed, ply=0)
    for k in range(150):
        acts = na.cpu().numpy().copy()
        inj = rs.random(n)
        acts = np.where(inj < 0.03, rs.integers(0, 45, n), acts)
        acts = np.where(inj > 0.995, rs.choice([-1, 45, 99], n), acts).astype(np.int32)
        e.step(torch.from_numpy(acts).to(e.device), next_actions=na, policy_seed=seed, ply=k + 1)
        ref = vec.step(acts, want_final=True)
        assert np.array_equal(e.obs.cpu().numpy(), ref["obs"]), k
        out["steps"] += n
    # every rollout kernel at 2 / 3 / 4 players, per-step store and in place, fused refills
    # (the quad and six-wave dealer kernels with the partner hand-off forced: lead -1; the quad kernel's
    # barrier count is checked per wave, BC_BARRIER)
    for P, pipe, lead in ((2, True, None), (2, False, None), (3, True, None), (4, True, None), (4, "half", None),
                          (2, "always", None), (4, "dealer", None), (2, "quad", -1), (4, "dealer2", -1)):
        r = Engine(512, P, pipeline=pipe, partner_lead=lead)
        r.reset(seeds=range(512))
        a = torch.zeros(512, dtype=torch.int32, device=r.device)
        r.sample_uniform(out=a, seed=1, ply=0)
        K = 64
        store = {"obs": torch.empty((K, 512, 297), dtype=torch.int32, device=r.device),
                 "mask": torch.empty((K, 512, 45), dtype=torch.int8, device=r.device),
                 "reward": torch.empty((K, 512), dtype=torch.float32, device=r.device),
                 "terminated": torch.empty((K, 512), dtype=torch.uint8, device=r.device),
                 "flags": torch.empty((K, 512), dtype=torch.uint8, device=r.device)}
        for launch in range(3):
            nxt = torch.empty_like(a)
            r.rollout(K, actions=a, next_actions=nxt, policy_seed=1, ply=1 + K * launch,
                      out=store if launch % 2 == 0 else None)
            a = nxt
            out["steps"] += 512 * K
    # crafted reference edge cases, then hundreds-of-tokens returns through the continuation
    with open(os.path.join(HERE, "golden", "edge_cases.json")) as f:
        cases = json.load(f)
    for P in (2, 3, 4):
        cs = [c for c in cases if c["P"] == P]
        ee = Engine(len(cs), P)
        ee.reset(seeds=range(len(cs)))
        ee.upload(np.stack([view_to_table(c["before"]) for c in cs]))
        ee.step(torch.tensor([c["action"] for c in cs], dtype=torch.int32, device=ee.device), autoreset=True)
    _native.check(lib, lib.spl_debug_set_stream_limit(2))
    d = Engine(700, 3)
    d.reset(seeds=range(700))
    a = torch.zeros(700, dtype=torch.int32, device=d.device)
    d.sample_uniform(out=a, seed=2, ply=0)
    for k in range(60):
        d.step(a, next_actions=a, policy_seed=2, ply=k + 1)
    _native.check(lib, lib.spl_debug_set_stream_limit(454))
    torch.cuda.synchronize()
    _native.check(lib, lib.spl_debug_bounds_flags(ctypes.byref(flags), 0))
    out["flags"] = int(flags.value)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

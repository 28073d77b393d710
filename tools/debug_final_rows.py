"""Diagnose a final_obs mismatch between spl_rollout and the spl_step chain (prints the differing
rows / columns and the terminal-row counts of their waves).  Debug aid, GPU only."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "splendor-gym_amd")]

import torch  # noqa: E402
from splendor_gym.device import Engine  # noqa: E402

P, K, R, n, seed = 2, 16, 16, 1024, 11
pipeline = sys.argv[1] if len(sys.argv) > 1 else True
chain = Engine(n, P, refill_period=R)
fused = Engine(n, P, refill_period=R, refill_fused=True, pipeline=pipeline)
print("kernel", fused.rollout_kernel_name())
chain.reset(seeds=range(n))
fused.reset(seeds=range(n))
dev = chain.device
a_c = torch.zeros(n, dtype=torch.int32, device=dev)
chain.sample_uniform(out=a_c, seed=seed, ply=0)
a_f = a_c.clone()
bad = 0
for launch in range(5):
    ply0 = 1 + launch * K
    want = []
    for k in range(K):
        na = torch.empty_like(a_c)
        chain.step(a_c, next_actions=na, policy_seed=seed, ply=ply0 + k)
        want.append({x: getattr(chain, x).clone() for x in ("terminated", "final_obs", "obs")})
        a_c = na
    out = {"obs": torch.empty((K, n, 297), dtype=torch.int32, device=dev),
           "mask": torch.empty((K, n, 45), dtype=torch.int8, device=dev),
           "reward": torch.empty((K, n), dtype=torch.float32, device=dev),
           "terminated": torch.empty((K, n), dtype=torch.uint8, device=dev),
           "flags": torch.empty((K, n), dtype=torch.uint8, device=dev),
           "winner": torch.empty((K, n), dtype=torch.int8, device=dev),
           "final_obs": torch.zeros((K, n, 297), dtype=torch.int32, device=dev)}
    na = torch.empty_like(a_f)
    fused.rollout(K, actions=a_f, next_actions=na, policy_seed=seed, ply=ply0, out=out)
    a_f = na
    for k in range(K):
        term = want[k]["terminated"].bool()
        rows = term.nonzero().flatten()
        d = out["final_obs"][k][rows] != want[k]["final_obs"][rows]
        if d.any():
            rr = rows[d.any(dim=1)].tolist()
            waves = {}
            for t in rows.tolist():
                waves[t // 64] = waves.get(t // 64, 0) + 1
            print(f"launch {launch} step {k}: {len(rr)} of {len(rows)} terminal rows differ; per-wave terminal counts "
                  f"{sorted(waves.items())[:20]}")
            for t in rr[:6]:
                i = rows.tolist().index(t)
                cols = d[i].nonzero().flatten().tolist()
                print(f"  table {t} (wave {t // 64}, rank in wave {sum(1 for x in rows.tolist() if x // 64 == t // 64 and x < t)}):"
                      f" cols {cols[:20]} rollout {out['final_obs'][k][t][cols[:20]].tolist()} "
                      f"chain {want[k]['final_obs'][t][cols[:20]].tolist()}")
            bad += 1
print("bad steps", bad)

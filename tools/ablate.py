"""Ablation timing of k_step: build variants of the engine with one phase compiled out
(-DSPL_ABL=<bits>, see spl_engine.hip) and time each in its own process (HIP events around
each eager launch, 2p x 65536 tables, device random policy, refill every 16).

    python tools/ablate.py [--build-only] [--run] [--rollout] [variant ...]
--rollout times k_rollout launches (16 steps each) instead of k_step.
Outputs are wrong in ablated builds by design; only timings are meaningful.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "splendor-gym_amd", "csrc")
OUTD = os.path.join(REPO, "splendor-gym_amd", "ablate")
IO = 1 | 2 | 4 | 8 | 16 | 32  # every compute phase compiled out: loads + stores only
VARIANTS = {"full": 0, "no_legal_pre": 1, "no_apply": 2, "no_legal_post": 4, "no_final": 8, "no_reset": 16,
            "no_encode": 32, "no_store": 64, "no_encode_store": 96, "only_io": IO,
            "only_io_no_mask": IO | 128, "only_io_no_small": IO | 256, "only_io_no_tab": IO | 512,
            "only_io_no_obs": IO | 1024, "only_obs": IO | 128 | 256 | 512, "only_obs_noload": IO | 128 | 256 | 512 | 2048,
            "no_noble": 8192, "no_toklim": 4096, "no_obs_store": 1024, "no_compute": 2 | 4 | 32}


def build():
    os.makedirs(OUTD, exist_ok=True)
    names = [a for a in sys.argv[1:] if not a.startswith("--")] or list(VARIANTS)
    for name in names:
        bits = VARIANTS[name]
        out = os.path.join(OUTD, f"lib_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", f"-DSPL_ABL={bits}",
                        "-shared", "-o", out, *[os.path.join(CSRC, f) for f in ("spl_engine.hip", "spl_policy.hip", "spl_policy32.hip", "spl_dual.hip")]], check=True)


CHILD = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
T = 65536
e = Engine(T, 2, device="cuda:0", refill_period=0)
e.reset(seeds=range(T))
buf = [torch.zeros(T, dtype=torch.int32, device=e.device) for _ in range(2)]
e.sample_uniform(out=buf[0], seed=1, ply=0)
times = []
for k in range(320):
    a, b = buf[k & 1], buf[(k & 1) ^ 1]
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record(); e.step(a, next_actions=b, policy_seed=1, ply=k + 1); s1.record()
    if (k + 1) % 16 == 0: e.refill()
    times.append((s0, s1))
torch.cuda.synchronize()
ms = [x.elapsed_time(y) for x, y in times[64:]]
print(json.dumps({"avg_us": 1000 * sum(ms) / len(ms), "min_us": 1000 * min(ms)}))
'''


CHILD_ROLLOUT = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
T, K = 65536, 16
e = Engine(T, 2, device="cuda:0", refill_period=0)
e.reset(seeds=range(T))
buf = [torch.zeros(T, dtype=torch.int32, device=e.device) for _ in range(2)]
e.sample_uniform(out=buf[0], seed=1, ply=0)
times = []
for it in range(24):
    a, b = buf[it & 1], buf[(it & 1) ^ 1]
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record(); e.rollout(K, actions=a, next_actions=b, policy_seed=1, ply=1 + K * it); s1.record()
    if (it + 1) % 4 == 0: e.refill()
    times.append((s0, s1))
torch.cuda.synchronize()
ms = [x.elapsed_time(y) / K for x, y in times[8:]]
print(json.dumps({"avg_us_per_step": 1000 * sum(ms) / len(ms), "min_us_per_step": 1000 * min(ms)}))
'''


def run():
    res = {}
    child = CHILD_ROLLOUT if "--rollout" in sys.argv else CHILD
    names = [a for a in sys.argv[1:] if not a.startswith("--")] or list(VARIANTS)
    for name in names:
        env = dict(os.environ, SPLENDOR_AMD_LIB=os.path.join(OUTD, f"lib_{name}.so"))
        r = subprocess.run([sys.executable, "-c", child, REPO], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            print(name, "FAILED", r.stderr[-500:])
            return 1
        res[name] = json.loads(r.stdout.strip().splitlines()[-1])
        print(name, res[name], flush=True)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    if "--run" not in sys.argv:
        build()
    if "--build-only" not in sys.argv:
        sys.exit(run())

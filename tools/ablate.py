"""Ablation timing of k_step_ws: build variants of the engine with one phase compiled out
(-DSPL_ABL=<bits>, see spl_engine.hip) and time each in its own process (HIP events around
each eager launch, 2p tables, device random policy, refill every 16).

    python tools/ablate.py [--build-only] [--run] [--rollout] [--tables 16384,65536] [--rounds R] [variant ...]
--rollout times k_rollout launches (16 steps each) instead of k_step.  --rounds R alternates the
variants R times (one process per variant and round) so box drift hits every arm alike.
Only spl_engine.hip is recompiled per variant; the other objects come from csrc/obj (run `make` first).
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
            "no_noble": 8192, "no_toklim": 4096, "no_obs_store": 1024, "no_compute": 2 | 4 | 32,
            "no_deck_gather": 16384, "no_lut_gather": 32768, "no_gathers": 16384 | 32768, "no_mask_store": 128,
            "no_final_legal_post": 8 | 4}


def _build_one(name, src):
    bits = VARIANTS[name]
    out = os.path.join(OUTD, f"lib_{name}.so")
    obj = os.path.join(OUTD, "obj", f"spl_engine_{name}.o")
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950"]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, f"-DSPL_ABL={bits}", "-c", "-o", obj,
                    os.path.join(src, "spl_engine.hip")], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-shared", "-o", out, obj,
                    *[os.path.join(CSRC, "obj", f + ".o") for f in ("spl_policy", "spl_policy32", "spl_dual")]], check=True)
    return name


def build():
    """Compile the variants in parallel (one hipcc each, at most 8 at once) from a snapshot of the
    sources, so csrc/ can be edited while they build."""
    import shutil
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(os.path.join(OUTD, "obj"), exist_ok=True)
    src = os.path.join(OUTD, "obj", "src")
    shutil.rmtree(src, ignore_errors=True)
    shutil.copytree(CSRC, os.path.join(src, "pkg", "csrc"), ignore=shutil.ignore_patterns("obj"))  # ../../include
    shutil.copytree(os.path.join(REPO, "include"), os.path.join(src, "include"))
    names = [a for a in sys.argv[1:] if not a.startswith("--") and a in VARIANTS] or list(VARIANTS)
    with ThreadPoolExecutor(max_workers=int(os.environ.get("ABL_JOBS", "8"))) as ex:
        for name in ex.map(lambda n: _build_one(n, os.path.join(src, "pkg", "csrc")), names):
            print("built", name, flush=True)


CHILD = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
T = int(sys.argv[2])
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
ms = sorted(x.elapsed_time(y) for x, y in times[64:])
print(json.dumps({"median_us": round(1000 * ms[len(ms) // 2], 2), "avg_us": round(1000 * sum(ms) / len(ms), 2),
                  "min_us": round(1000 * ms[0], 2)}))
'''


CHILD_ROLLOUT = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
T, K = int(sys.argv[2]), 16
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


def opt(flag, default):
    return sys.argv[sys.argv.index(flag) + 1] if flag in sys.argv else default


def run():
    res = {}
    child = CHILD_ROLLOUT if "--rollout" in sys.argv else CHILD
    names = [a for a in sys.argv[1:] if not a.startswith("--") and a in VARIANTS] or list(VARIANTS)
    sizes = [int(x) for x in opt("--tables", "65536").split(",")]
    for rnd in range(int(opt("--rounds", "1"))):
        for T in sizes:
            for name in names:
                env = dict(os.environ, SPLENDOR_AMD_LIB=os.path.join(OUTD, f"lib_{name}.so"))
                r = subprocess.run([sys.executable, "-c", child, REPO, str(T)], env=env, capture_output=True, text=True,
                                   timeout=300)
                if r.returncode != 0:
                    print(name, T, "FAILED", r.stderr[-500:])
                    return 1
                res.setdefault(f"{name}|T{T}", []).append(json.loads(r.stdout.strip().splitlines()[-1]))
                print(rnd, T, name, res[f"{name}|T{T}"][-1], flush=True)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    if "--run" not in sys.argv:
        build()
    if "--build-only" not in sys.argv:
        sys.exit(run())

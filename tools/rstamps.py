"""Per-step timeline of k_rollout from register-held s_memrealtime stamps (diagnostic build).

    python tools/rstamps.py [--build-only | --run]
Stamps per step k (lane k of each wave): 0 step start, 1 rules done, 2 previous step's obs tail
issued, 3 obs rows encoded, 4 this step's stores issued; 5 = wave end.  Reports medians over waves
of each phase's duration and of the step period (start k+1 - start k), in microseconds.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "splendor-gym_amd", "ablate", "lib_stamps.so")

CHILD = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
T, K = 65536, 16
e = Engine(T, 2, device="cuda:0", refill_period=0)
e.lib.spl_debug_set_rollout_stamps.argtypes = [ctypes.c_void_p]
e.lib.spl_debug_set_stamps.argtypes = [ctypes.c_void_p]
step_st = torch.zeros((T // 64) * 16, dtype=torch.int64, device=e.device)  # k_step stamp points inside step_rules
_native.check(e.lib, e.lib.spl_debug_set_stamps(step_st.data_ptr()))
e.reset(seeds=range(T))
buf = [torch.zeros(T, dtype=torch.int32, device=e.device) for _ in range(2)]
e.sample_uniform(out=buf[0], seed=1, ply=0)
st = torch.zeros((T // 64) * 16 * 6, dtype=torch.int64, device=e.device)
_native.check(e.lib, e.lib.spl_debug_set_rollout_stamps(st.data_ptr()))
out = []
for it in range(12):
    e.rollout(K, actions=buf[it & 1], next_actions=buf[(it & 1) ^ 1], policy_seed=1, ply=1 + K * it)
    if (it + 1) % 4 == 0: e.refill()
    if it >= 8:
        torch.cuda.synchronize()
        out.append(st.view(-1, 16, 6).cpu().tolist())
print(json.dumps(out))
'''


def main():
    if "--run" not in sys.argv:
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-DSPL_STAMPS",
                        "-shared", "-o", LIB, *[os.path.join(REPO, "splendor-gym_amd", "csrc", f)
                                                  for f in ("spl_engine.hip", "spl_policy.hip", "spl_policy32.hip", "spl_dual.hip")]],
                       check=True)
        if "--build-only" in sys.argv:
            return 0
    env = dict(os.environ, SPLENDOR_AMD_LIB=LIB)
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True, text=True, timeout=600)
    if r.returncode:
        print(r.stderr[-2000:])
        return 1
    import numpy as np
    runs = np.array(json.loads(r.stdout.strip().splitlines()[-1]), dtype=np.int64)  # [run, wave, step, 6]
    us = lambda x: x * 0.01  # 100 MHz ticks
    t0 = runs[..., 0, 0].min(axis=1)[:, None, None]
    a = runs[..., :5] - t0[..., None]
    names = ["rules", "prev obs tail issued", "final+reset+encode", "sample+stores issued"]
    print("median over waves and launches, microseconds")
    print(f"{'step':>4s} {'start':>8s} " + " ".join(f"{n:>22s}" for n in names) + f" {'period':>8s}")
    for k in range(16):
        st = a[:, :, k, :]
        d = [np.median(us(st[..., i + 1] - st[..., i])) for i in range(4)]
        per = np.median(us(a[:, :, k + 1, 0] - st[..., 0])) if k < 15 else float("nan")
        print(f"{k:4d} {np.median(us(st[..., 0])):8.2f} " + " ".join(f"{x:22.2f}" for x in d) + f" {per:8.2f}")
    end = us(runs[:, :, 0, 5] - t0[:, :, 0])
    print(f"wave end: median {np.median(end):.1f} us, max {end.max():.1f} us; first step start spread "
          f"p90-p10 {np.percentile(us(a[:, :, 0, 0]), 90) - np.percentile(us(a[:, :, 0, 0]), 10):.2f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())

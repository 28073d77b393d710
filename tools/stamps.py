"""Per-phase timeline of k_step from in-kernel s_memrealtime stamps (diagnostic build only).

    python tools/stamps.py            # build lib_stamps.so (-DSPL_STAMPS) and run on the GPU
Lane 0 of every wave stamps 12 phase boundaries (see STAMP(i) in spl_engine.hip); we report, per
phase, the median and max over waves of the time since the kernel's first stamp (10 ns ticks).
Stamped builds fence the scheduler around each stamp: read the SHARES, not the absolute length.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("STAMP_LIB", os.path.join(REPO, "splendor-gym_amd", "ablate", "lib_stamps.so"))
NAMES = ["start", "loaded+prefetched", "pre-apply", "applied", "step logic", "final obs", "reset done",
         "encoded", "barrier", "obs stored", "mask+final stored", "end"]

CHILD = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
T = 65536
e = Engine(T, 2, device="cuda:0", refill_period=0)
e.lib.spl_debug_set_stamps.argtypes = [ctypes.c_void_p]
e.reset(seeds=range(T))
buf = [torch.zeros(T, dtype=torch.int32, device=e.device) for _ in range(2)]
e.sample_uniform(out=buf[0], seed=1, ply=0)
st = torch.zeros((T // 64) * 16, dtype=torch.int64, device=e.device)
_native.check(e.lib, e.lib.spl_debug_set_stamps(st.data_ptr()))
out = []
for k in range(96):
    e.step(buf[k & 1], next_actions=buf[(k & 1) ^ 1], policy_seed=1, ply=k + 1)
    if (k + 1) % 16 == 0: e.refill()
    if k >= 80:
        torch.cuda.synchronize()
        out.append(st.view(-1, 16).cpu().tolist())
print(json.dumps(out))
'''


def main():
    if "--run" not in sys.argv:
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        extra = os.environ.get("STAMP_DEFS", "").split()  # e.g. STAMP_DEFS=-DSPL_ABL=4096
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-DSPL_STAMPS",
                        *extra, "-shared", "-o", LIB, *[os.path.join(REPO, "splendor-gym_amd", "csrc", f)
                        for f in ("spl_engine.hip", "spl_policy.hip", "spl_policy32.hip", "spl_dual.hip")]],
                       check=True)
        if "--build-only" in sys.argv:
            return 0
    env = dict(os.environ, SPLENDOR_AMD_LIB=LIB)
    r = subprocess.run([sys.executable, "-c", CHILD, REPO], env=env, capture_output=True, text=True, timeout=600)
    if r.returncode:
        print(r.stderr[-2000:])
        return 1
    runs = json.loads(r.stdout.strip().splitlines()[-1])
    import numpy as np
    rows = []
    for run in runs:
        a = np.array(run, dtype=np.int64)[:, :len(NAMES)]
        t0 = a[:, 0].min()
        rows.append(a - t0)
    a = np.concatenate(rows).astype(np.float64) * 0.01  # 100 MHz ticks -> microseconds
    print(f"{'phase':22s} {'median us':>10s} {'p90 us':>8s} {'max us':>8s}   (since kernel start, {len(a)} wave-samples)")
    for i, nm in enumerate(NAMES):
        col = a[:, i][a[:, i] >= 0]
        print(f"{i:2d} {nm:19s} {np.median(col):10.2f} {np.percentile(col, 90):8.2f} {col.max():8.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())

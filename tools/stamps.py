"""Per-phase timeline of k_step from in-kernel s_memrealtime stamps (diagnostic build only).

    python tools/stamps.py            # build lib_stamps.so (-DSPL_STAMPS) and run on the GPU
    (STAMP_T: tables, default 65536; --build-only here, --run on the box)
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
# k_step_ws (the default spl_step kernel): stamps per wave, wave 0 = rules, wave 1 = output
WS_RULES = ["start", "past hand-off 0", "rules done", "state to LDS (reset done)", "past hand-off 2 (row halves)", "legal mask",
            "end (mask, small outputs, state stored)", "final rows stored (before 5)", "mask block issued (before 6)"]
WS_OUT = ["start", "tables staged", "past hand-off 0", "past hand-off 1", "past hand-off 2 (rows encoded)", "final rows done",
          "obs stores issued", "end", "early board stores issued"]

CHILD = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
T = int(os.environ.get("STAMP_T", "65536"))
e = Engine(T, 2, device="cuda:0", refill_period=0, step_tail=0)  # the two-wave shape this parser reads
e.lib.spl_debug_set_stamps.argtypes = [ctypes.c_void_p]
e.reset(seeds=range(T))
buf = [torch.zeros(T, dtype=torch.int32, device=e.device) for _ in range(2)]
e.sample_uniform(out=buf[0], seed=1, ply=0)
st = torch.zeros((T // 64) * 3 * 16, dtype=torch.int64, device=e.device)  # room for three waves per workgroup
_native.check(e.lib, e.lib.spl_debug_set_stamps(st.data_ptr()))
out = []
for k in range(96):
    e.step(buf[k & 1], next_actions=buf[(k & 1) ^ 1], policy_seed=1, ply=k + 1)
    if (k + 1) % 16 == 0: e.refill()
    if k >= 80:
        torch.cuda.synchronize()
        out.append(st.view(-1, 16)[: (T // 64) * 2].cpu().tolist())
        st.zero_()
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
    a = np.array(runs, dtype=np.int64)  # [run, wave slot, 16]
    ws = (a[0, :, 0] != 0).sum() > a.shape[1] // 2  # k_step_ws stamps two waves per 64 tables
    if not ws:
        a = a[:, : a.shape[1] // 2]
    rows = []
    for run in a:
        t0 = run[run[:, 0] > 0, 0].min()
        rows.append(np.where(run > 0, run - t0, -1))
    a = np.stack(rows).astype(np.float64)
    a = np.where(a >= 0, a * 0.01, np.nan)  # 100 MHz ticks -> microseconds since the kernel's first stamp
    groups = [("k_step", NAMES, a.reshape(-1, 16))] if not ws else [
        ("k_step_ws rules wave", WS_RULES, a[:, 0::2].reshape(-1, 16)), ("k_step_ws output wave", WS_OUT, a[:, 1::2].reshape(-1, 16))]
    for title, names, m in groups:
        print(f"{title}: {'phase':26s} {'median us':>10s} {'p90 us':>8s} {'max us':>8s}   ({len(m)} wave-samples)")
        for i, nm in enumerate(names):
            col = m[:, i][~np.isnan(m[:, i])]
            if col.size == 0:
                continue
            print(f"{i:2d} {nm:26s} {np.median(col):10.2f} {np.percentile(col, 90):8.2f} {col.max():8.2f}")
    if ws:  # the rules wave's tail by its terminal-row count (slot 9: rows | deferred-mask lanes << 8)
        raw = np.array(runs, dtype=np.int64)[:, 0::2, 9].reshape(-1)
        fin, dfr = raw & 255, raw >> 8
        r = a[:, 0::2]
        tail = (r[:, :, 7] - r[:, :, 4]).reshape(-1)
        lm = (r[:, :, 5] - r[:, :, 7]).reshape(-1)
        end = r[:, :, 6].reshape(-1)
        for n in range(0, 8):
            sel = fin == n
            if sel.sum() == 0:
                continue
            print(f"rules waves with {n} terminal rows: {sel.sum():6d}, final rows {np.nanmedian(tail[sel]):.2f} us, "
                  f"legal mask {np.nanmedian(lm[sel]):.2f} us (deferred lanes {np.median(dfr[sel]):.0f}), "
                  f"end median {np.nanmedian(end[sel]):.2f} max {np.nanmax(end[sel]):.2f}")
    if ws:  # per XCC (workgroup i runs on XCC i % 8): the rules wave's hand-off 1 and the output wave's end
        wg = np.arange(a.shape[1] // 2) % 8
        for title, idx, ph in (("rules: past hand-off 1", 0, 4), ("output: end", 1, WS_OUT.index("end"))):
            v = a[:, idx::2, ph]
            print(f"{title} by XCC median/p99: " + " | ".join(
                f"{np.nanmedian(v[:, wg == x]):.1f}/{np.nanpercentile(v[:, wg == x], 99):.1f}" for x in range(8)))
    return 0


if __name__ == "__main__":
    sys.exit(main())

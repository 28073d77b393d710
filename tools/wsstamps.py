"""Per-step timeline of the two-wave rollout kernel k_rollout_ws from register-held
s_memrealtime stamps (diagnostic build -DSPL_STAMPS; not the product library).

    python tools/wsstamps.py [--build-only | --run] [--inplace] [--lib PATH]
    (WS_P / WS_T: players and tables, default 2 and 65536; 4 x 32768 runs the dealer variant)
Rules wave stamps per step: 0 start, 1 rules done, 2 hand-off written, 3 past the barrier.
Output wave: 0 past the barrier, 1 rows encoded (incl. terminal rows), 2 obs stores issued,
3 mask + small outputs issued.  Medians over workgroups and launches, microseconds.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "splendor-gym_amd", "ablate", "lib_wsstamps.so")

CHILD = r'''
import sys, os, ctypes, json
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "splendor-gym_amd")]
import torch
from splendor_gym import _native
from splendor_gym.device import Engine
inplace = sys.argv[2] == "1"
T, K, P = int(os.environ.get("WS_T", "65536")), 64, int(os.environ.get("WS_P", "2"))
lead = os.environ.get("WS_LEAD")  # partner hand-off lead of the six-wave dealer (None = library default)
e = Engine(T, P, device="cuda:0", refill_period={2: 64, 3: 32, 4: 16}[P], partner_lead=None if lead is None else int(lead))
e.lib.spl_debug_set_ws_stamps.argtypes = [ctypes.c_void_p]
e.reset(seeds=range(T))
buf = [torch.zeros(T, dtype=torch.int32, device=e.device) for _ in range(2)]
e.sample_uniform(out=buf[0], seed=1, ply=0)
e.lib.spl_debug_set_ws_hwid.argtypes = [ctypes.c_void_p]
hw = torch.zeros((T // 64) * 2 * 2, dtype=torch.int32, device=e.device)
_native.check(e.lib, e.lib.spl_debug_set_ws_hwid(hw.data_ptr()))
e.lib.spl_debug_set_ws_clk.argtypes = [ctypes.c_void_p]
clk = torch.zeros((T // 64) * 4, dtype=torch.int64, device=e.device)
_native.check(e.lib, e.lib.spl_debug_set_ws_clk(clk.data_ptr()))
wend = torch.zeros((T // 64) * 2, dtype=torch.int64, device=e.device)
e.lib.spl_debug_set_ws_end.argtypes = [ctypes.c_void_p]  # a 64-bit pointer, not a C int
_native.check(e.lib, e.lib.spl_debug_set_ws_end(wend.data_ptr()))
deleg = os.environ.get("WS_DELEG")
if deleg is not None:
    _native.check(e.lib, e.lib.spl_ctx_set_rollout_delegation(e.ctx, int(deleg)))
st = torch.zeros((T // 64) * 2 * 64 * 11, dtype=torch.int64, device=e.device)
_native.check(e.lib, e.lib.spl_debug_set_ws_stamps(st.data_ptr()))
store = None if inplace else dict(
    obs=torch.empty((K, T, 297), dtype=torch.int32, device=e.device),
    mask=torch.empty((K, T, 45), dtype=torch.int8, device=e.device),
    reward=torch.empty((K, T), dtype=torch.float32, device=e.device),
    terminated=torch.empty((K, T), dtype=torch.uint8, device=e.device),
    flags=torch.empty((K, T), dtype=torch.uint8, device=e.device),
    winner=torch.empty((K, T), dtype=torch.int8, device=e.device),
    final_obs=torch.empty((K, T, 297), dtype=torch.int32, device=e.device))
out = []
for it in range(6):
    e.rollout(K, actions=buf[it & 1], next_actions=buf[(it & 1) ^ 1], policy_seed=1, ply=1 + K * it, out=store)
    if it >= 3:
        torch.cuda.synchronize()
        out.append(st.view(-1, 2, 64, 11).cpu().numpy().tolist())
        hws = hw.view(-1, 2, 2).cpu().numpy().tolist()
        clks = clk.view(-1, 4).cpu().numpy().tolist()
        ends = wend.view(-1, 2).cpu().numpy().tolist()
print(json.dumps(ends))
print(json.dumps(clks))
print(json.dumps(hws))
print(json.dumps(out))
'''


def main():
    lib = LIB
    if "--lib" in sys.argv:
        lib = sys.argv[sys.argv.index("--lib") + 1]
    if "--run" not in sys.argv:
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        extra = os.environ.get("STAMP_DEFS", "").split()  # e.g. STAMP_DEFS=-DSPL_ABL=49152
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-DSPL_STAMPS", "-w",
                        *extra, "-shared", "-o", lib, *[os.path.join(REPO, "splendor-gym_amd", "csrc", f)
                                                  for f in ("spl_engine.hip", "spl_policy.hip", "spl_policy32.hip", "spl_dual.hip")]],
                       check=True)
        if "--build-only" in sys.argv:
            return 0
    env = dict(os.environ, SPLENDOR_AMD_LIB=lib)
    r = subprocess.run([sys.executable, "-c", CHILD, REPO, "1" if "--inplace" in sys.argv else "0"], env=env,
                       capture_output=True, text=True, timeout=600)
    if r.returncode:
        print(r.stderr[-2000:])
        return 1
    import numpy as np
    runs = np.array(json.loads(r.stdout.strip().splitlines()[-1]), dtype=np.int64)  # [run, wg, wave, step, 4]
    hws = np.array(json.loads(r.stdout.strip().splitlines()[-2]), dtype=np.int64)  # [wg, wave, 2] (last launch)
    clks = np.array(json.loads(r.stdout.strip().splitlines()[-3]), dtype=np.float64)  # [wg, 4]
    ends = np.array(json.loads(r.stdout.strip().splitlines()[-4]), dtype=np.float64)  # [wg, 2] (last launch)
    ghz = (clks[:, 2] - clks[:, 0]) / ((clks[:, 3] - clks[:, 1]) * 10.0)  # s_memtime ticks per ns
    us = lambda x: x * 0.01  # 100 MHz ticks
    t0 = runs[:, :, 0, 0, 0].min(axis=1)[:, None, None]
    a = runs - t0[..., None, None]
    R, O = a[:, :, 0], a[:, :, 1]  # [run, wg, step, 4]
    print("median over workgroups and launches, microseconds (K = 64 steps)")
    print(f"{'step':>4s} | rules: {'rules':>6s} {'tail':>6s} {'wait':>6s} | output: {'encode':>6s} {'obs st':>6s} "
          f"{'mask':>6s} {'wait':>6s} | {'period':>6s}")
    rows = []
    for k in range(64):
        r = [np.median(us(R[..., k, i + 1] - R[..., k, i])) for i in range(3)]
        o = [np.median(us(O[..., k, i + 1] - O[..., k, i])) for i in range(3)]
        ow = np.median(us(O[..., k + 1, 0] - O[..., k, 3])) if k < 63 else float("nan")
        per = np.median(us(R[..., k + 1, 0] - R[..., k, 0])) if k < 63 else float("nan")
        rows.append(r + o + [ow, per])
        if k < 4 or k % 8 == 0 or k == 63:
            print(f"{k:4d} | rules: {r[0]:6.2f} {r[1]:6.2f} {r[2]:6.2f} | output: {o[0]:6.2f} {o[1]:6.2f} {o[2]:6.2f} "
                  f"{ow:6.2f} | {per:6.2f}")
    m = np.nanmean(np.array(rows[4:63]), axis=0)
    print("mean of steps 4..62: rules %.2f tail %.2f wait %.2f | encode %.2f obs %.2f mask %.2f wait %.2f | period %.2f"
          % tuple(m))
    end = us(a[:, :, 1, 63, 3])
    print(f"output wave last step done: median {np.median(end):.1f} us, max {end.max():.1f} us")
    print("end percentiles p10/p50/p90/p99/max: " + " ".join(f"{np.percentile(end, q):.0f}" for q in (10, 50, 90, 99, 100)))
    nwg = end.shape[1]
    xcd = np.arange(nwg) % 8
    print("mean end by blockIdx % 8: " + " ".join(f"{end[:, xcd == x].mean():.0f}" for x in range(8)))
    print("mean end by blockIdx // 128: " + " ".join(f"{end[:, (np.arange(nwg) // 128) == g].mean():.0f}" for g in range(nwg // 128)))
    hwid, xcc = hws[..., 0] & 0xFFFFFFFF, hws[..., 1]
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 15
    se = (hwid >> 13) & 7
    e_last = end[-1]
    print("XCC of wg (blockIdx % 8 -> xcc):", [int(np.bincount(xcc[np.arange(nwg) % 8 == x, 0] & 15).argmax()) for x in range(8)])
    print("mean end by XCC: " + " ".join(f"{e_last[(xcc[:, 0] & 15) == x].mean():.0f}" for x in range(8)))
    print("mean step-0 start by XCC: " + " ".join(f"{us(R[-1, (xcc[:, 0] & 15) == x, 0, 0]).mean():.1f}" for x in range(8)))
    print("s_memtime rate (GHz) by XCC: " + " ".join(f"{ghz[(xcc[:, 0] & 15) == x].mean():.3f}" for x in range(8)))
    pair = simd[:, 0] * 4 + simd[:, 1]
    print("(rules SIMD, output SIMD) counts / mean end: " + "; ".join(
        f"({p // 4},{p % 4}) {int((pair == p).sum())} {e_last[pair == p].mean():.0f}" for p in range(16) if (pair == p).any()))
    # rules waves sharing a SIMD with another rules wave of the same CU
    key = (xcc[:, 0] & 15) * 10000 + se[:, 0] * 1000 + cu[:, 0] * 10 + simd[:, 0]
    _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    nr = cnt[inv]
    print("rules waves per SIMD (of each WG's rules wave): " + "; ".join(
        f"{c} -> {int((nr == c).sum())} WGs, mean end {e_last[nr == c].mean():.0f}" for c in sorted(set(nr.tolist()))))
    print("first 8 WGs hwid:", [(int(xcc[i, 0] & 15), int(se[i, 0]), int(cu[i, 0]), int(simd[i, 0]), int(simd[i, 1])) for i in range(8)])
    # rules-wave sub-phases (stamps 4-7; 4/5 only on lanes' steps that apply an action, so a
    # missing stamp reads as 0 and those steps are skipped)
    ok = (R[..., 4:63, 4] > 0) & (R[..., 4:63, 5] > 0) & (R[..., 4:63, 6] > 0)
    ok = ok & (R[..., 4:63, 8] > 0) & (R[..., 4:63, 9] > 0) & (R[..., 4:63, 10] > 0)
    sub = {"pre (to apply)": (R[..., 4:63, 4] - R[..., 4:63, 0]), "apply": (R[..., 4:63, 5] - R[..., 4:63, 4]),
           "  action": (R[..., 4:63, 8] - R[..., 4:63, 4]), "  noble": (R[..., 4:63, 9] - R[..., 4:63, 8]),
           "  token limit": (R[..., 4:63, 10] - R[..., 4:63, 9]), "  end of turn": (R[..., 4:63, 5] - R[..., 4:63, 10]),
           "post (term/reward)": (R[..., 4:63, 6] - R[..., 4:63, 5]), "legal mask": (R[..., 4:63, 1] - R[..., 4:63, 6]),
           "refill/final/autoreset": (R[..., 4:63, 7] - R[..., 4:63, 1]), "policy+prefetch+LDS": (R[..., 4:63, 2] - R[..., 4:63, 7])}
    print("rules-wave sub-phases, steps 4..62, median/mean us: " + "; ".join(
        f"{k} {np.median(us(v[ok])):.2f}/{us(v[ok]).mean():.2f}" for k, v in sub.items()))
    xs = xcc[:, 0] & 15
    for par in (0, 1):  # even / odd XCCs: where the rules wave's extra time goes
        sel = (xs % 2 == par)[None, :, None] & ok
        print(f"  {'even' if par == 0 else 'odd '} XCCs sub-phase means: " + "; ".join(
            f"{k.strip()} {us(v[sel]).mean():.2f}" for k, v in sub.items()))
    raw = os.environ.get("WS_RAW")
    if raw:  # the raw stamps for offline analysis
        np.savez_compressed(raw, runs=runs, hws=hws, clks=clks, ends=ends)
    # per XCC (from HW_ID/XCC_ID): where the rules wave's time goes
    xcd = xcc[:, 0] & 15  # the XCC each stamp slot's rules wave ran on (last launch; the map is static)
    rs = us(R[..., 4:63, 1] - R[..., 4:63, 0])  # [run, wg, step]
    tl = us(R[..., 4:63, 2] - R[..., 4:63, 1])
    enc = us(O[..., 4:63, 1] - O[..., 4:63, 0])
    ost = us(O[..., 4:63, 2] - O[..., 4:63, 1])
    rw = us(R[..., 4:63, 3] - R[..., 4:63, 2])
    ow = us(O[..., 5:64, 0] - O[..., 4:63, 3])
    per = us(R[..., 5:64, 0] - R[..., 4:63, 0])
    for name, v in (("rules", rs), ("tail", tl), ("rules wait", rw), ("out encode", enc), ("out obs st", ost),
                    ("out wait", ow), ("period", per)):
        print(f"per-step {name:10s} by XCC mean/p90/p99: " + " | ".join(
            f"{v[:, xcd == x].mean():.2f}/{np.percentile(v[:, xcd == x], 90):.1f}/{np.percentile(v[:, xcd == x], 99):.1f}"
            for x in range(8)))
    # per-workgroup: total rules-wave busy time vs barrier waits; slowest 1% vs median
    busy = us((R[..., :, 2] - R[..., :, 0]).sum(axis=-1))
    slow = end >= np.percentile(end, 99)
    print(f"rules busy per launch: median {np.median(busy):.0f} us, slowest-1% WGs {busy[slow].mean():.0f} us")
    st = us(R[..., 1, 0] - 0)
    print(f"rules wave step-0 start: median {np.median(us(R[..., 0, 0])):.1f}, slowest-1% WGs {us(R[..., 0, 0])[slow].mean():.1f} us")
    worst = np.argmax(np.array([us(R[..., k, 2] - R[..., k, 0])[slow].mean() for k in range(64)]))
    print(f"slowest-1% WGs: per-step rules busy at k={worst}: {us(R[..., worst, 2] - R[..., worst, 0])[slow].mean():.1f} us; "
          f"sum of per-step periods excluding the max step {np.sort(us(np.diff(R[..., :, 0], axis=-1))[slow], axis=-1)[:, :-1].sum(axis=-1).mean():.0f} us")
    # output waves of the last launch: last step issued, and the wave's end (delegated blocks included,
    # its stores completed)
    e0 = runs[-1, :, 0, 0, 0].min()
    le, fe = us(ends[:, 0] - e0), us(ends[:, 1] - e0)
    wgx = np.arange(len(fe)) % 8
    print("output wave, last launch: last step issued mean/max %.0f/%.0f us; wave end (stores done) mean/p99/max "
          "%.0f/%.0f/%.0f us" % (le.mean(), le.max(), fe.mean(), np.percentile(fe, 99), fe.max()))
    print("  wave end mean by blockIdx %% 8: " + " ".join(f"{fe[wgx == x].mean():.0f}" for x in range(8)))
    print("  last step mean by blockIdx %% 8: " + " ".join(f"{le[wgx == x].mean():.0f}" for x in range(8)))
    return 0


if __name__ == "__main__":
    sys.exit(main())

"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel and record the per-launch HBM
traffic of the step and rollout kernels for bench.py's roofline.traffic.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> profiles/pmc_summary.json \
        --players 2 --tables 65536 --rollout-steps 128

Every kernel of the run is keyed by its name (the identifier before the argument list, e.g.
k_rollout_store_2p, k_step_ws_2p, k_refill) plus the workload: `<kernel>|T<tables>|K<steps per
launch>`.  Entries of other workloads already in the output file are kept, so one file holds the
2p headline, the 3p/4p lines and C4's 4p x 32768 share side by side.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB.  WRITE_SIZE is exact
for 16 B/lane streaming stores (the observation blocks, >99 % of these kernels' writes).  On gfx950
FETCH_SIZE counts half the bytes of a 16 B/lane coalesced read; these kernels read 4 B/lane state
planes and 4-16 B gathers, outside that calibration, so FETCH_SIZE is reported uncorrected (reads
are < 1 % of the rollout's traffic).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

STEP_KERNELS = ("k_step", "k_rollout")  # kernels whose traffic bench.py reports


def base_name(kernel_name):
    """'void spl::k_rollout_store_2p(spl::KArena, ...)' -> 'k_rollout_store_2p'."""
    m = re.search(r"(?:\w+::)*(\w+)\s*[<(]", kernel_name)
    return m.group(1) if m else kernel_name.split("(")[0].strip()


def load(pmc_dir):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [value per dispatch]
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "**", "*counter_collection.csv"), recursive=True)):
        acc = defaultdict(float)  # (kernel, dispatch, counter) -> summed value
        times = {}
        for r in csv.DictReader(open(f)):
            k = base_name(r["Kernel_Name"])
            key = (k, int(r["Dispatch_Id"]), r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            times[(k, int(r["Dispatch_Id"]))] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (k, d, c), v in acc.items():
            per[k][c].append(v)
        for (k, d), t in times.items():
            dur[k].append(t)
    return per, dur


def derive(mean, durs):
    d = {"counters_mean_per_dispatch": mean}
    if durs:
        d["duration_us_mean"] = sum(durs) / len(durs) / 1e3
    if "GRBM_GUI_ACTIVE" in mean and durs:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md DVFS note)
        d["clock_ghz_est"] = mean["GRBM_GUI_ACTIVE"] / 8 / (sum(durs) / len(durs))
    if mean.get("SQ_WAVE_CYCLES") and mean.get("SQ_WAVES"):
        d["wave_cycles_each"] = 4 * mean["SQ_WAVE_CYCLES"] / mean["SQ_WAVES"]  # quad-cycles -> cycles
        for part in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if part in mean:
                d[part + "_frac"] = mean[part] / mean["SQ_WAVE_CYCLES"]
    if mean.get("SQ_WAVES"):
        for ins in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                    "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
            if ins in mean:
                d[ins + "_per_wave"] = mean[ins] / mean["SQ_WAVES"]
    if "FETCH_SIZE" in mean:
        d["fetch_bytes"] = mean["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in mean:
        d["write_bytes"] = mean["WRITE_SIZE"] * 1024
    if "fetch_bytes" in d and "write_bytes" in d:
        d["hbm_bytes_per_launch"] = round(d["fetch_bytes"] + d["write_bytes"])
    if "TCC_EA0_RDREQ" in mean:
        d["rdreq_bytes_64B"] = mean["TCC_EA0_RDREQ"] * 64
        d["wrreq_bytes_64B"] = mean.get("TCC_EA0_WRREQ", 0) * 64
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--tables", type=int, required=True)
    ap.add_argument("--players", type=int, required=True)
    ap.add_argument("--rollout-steps", type=int, default=128, help="env steps per rollout launch in the run")
    a = ap.parse_args()
    per, dur = load(a.pmc_dir)
    summary = {"entries": {}}
    if os.path.exists(a.out):
        with open(a.out) as f:
            summary = json.load(f)
        summary.setdefault("entries", {})
    for k, cs in per.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        steps = a.rollout_steps if k.startswith("k_rollout") else 1
        key = f"{k}|T{a.tables}|K{steps}"
        e = summary["entries"].get(key, {})
        # passes of one run add counters; a later run of the same workload replaces them
        if e.get("source") != a.pmc_dir:
            e = {}
        old_mean = e.get("counters_mean_per_dispatch", {})
        old_mean.update(mean)
        e = derive(old_mean, dur.get(k, []))
        e.update(kernel=k, players=a.players, tables=a.tables, steps_per_launch=steps, source=a.pmc_dir,
                 dispatches_per_pass=max(len(v) for v in cs.values()))
        summary["entries"][key] = e
    summary["hbm_bytes_note"] = ("FETCH_SIZE + WRITE_SIZE (KiB x 1024) per launch: WRITE_SIZE exact for the 16 B/lane "
                                 "block stores; FETCH_SIZE uncorrected (4 B/lane reads, outside the guide's 16 B/lane "
                                 "calibration; < 1 % of the rollout's bytes)")
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    for key, e in sorted(summary["entries"].items()):
        if e.get("source") == a.pmc_dir:
            print(key, {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in e.items()
                        if kk not in ("counters_mean_per_dispatch", "source")})


if __name__ == "__main__":
    main()

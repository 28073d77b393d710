"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel and write the per-launch HBM
traffic of the step and rollout kernels for bench.py's roofline.traffic.

    python tools/pmc_summary.py gpurun_out/pmc_<tag> profiles/pmc_summary.json [--tables 65536 --players 2]

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts exactly half the bytes of a wide (16 B/lane) coalesced read and other widths
are uncalibrated.  The step kernel's reads are 4 B/lane planes + 4 B gathers, so we report the
raw FETCH_SIZE bytes and, separately, the TCC_EA0_RDREQ x 64 B / WRREQ x 64 B request bytes.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(pmc_dir):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [value per dispatch]
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        acc = defaultdict(float)  # (kernel, dispatch, counter) -> summed value
        times = {}
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            k = next((kk for kk in ("k_step", "k_rollout", "k_refill") if kk in name), name)
            key = (k, int(r["Dispatch_Id"]), r["Counter_Name"])
            acc[key] += float(r["Counter_Value"])
            times[(k, int(r["Dispatch_Id"]))] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (k, d, c), v in acc.items():
            per[k][c].append(v)
        for (k, d), t in times.items():
            dur[k].append(t)
    return per, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--tables", type=int, default=65536)
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--rollout-steps", type=int, default=64, help="env steps per k_rollout launch in the run")
    ap.add_argument("--rollout-key", default="k_rollout_store",
                    help="name under which the rollout kernel's traffic is recorded: k_rollout_store (bench "
                         "--outputs store, per-step blocks) or k_rollout (--outputs inplace)")
    ap.add_argument("--merge", action="store_true",
                    help="update the kernels of this run in an existing summary instead of replacing it")
    a = ap.parse_args()
    per, dur = load(a.pmc_dir)
    summary = {"tables": a.tables, "players": a.players, "kernels": {}, "hbm_bytes_per_launch": {},
               "steps_per_launch": {}, "sources": {}}
    if a.merge and os.path.exists(a.out):
        with open(a.out) as f:
            old = json.load(f)
        assert old.get("tables") == a.tables and old.get("players") == a.players, "merge: other workload"
        for key in ("kernels", "hbm_bytes_per_launch", "steps_per_launch", "sources"):
            summary[key].update(old.get(key, {}))
    for k, cs in per.items():
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"counters_mean_per_dispatch": mean, "dispatches_per_pass": max(len(v) for v in cs.values())}
        if "GRBM_GUI_ACTIVE" in mean and dur.get(k):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md DVFS note)
            d["clock_ghz_est"] = mean["GRBM_GUI_ACTIVE"] / 8 / (sum(dur[k]) / len(dur[k]))
        if "SQ_WAVE_CYCLES" in mean and "SQ_WAVES" in mean and mean["SQ_WAVES"]:
            d["wave_cycles_each"] = 4 * mean["SQ_WAVE_CYCLES"] / mean["SQ_WAVES"]  # quad-cycles -> cycles
            for part in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if part in mean:
                    d[part + "_frac"] = mean[part] / mean["SQ_WAVE_CYCLES"]
            for ins in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                        "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
                if ins in mean:
                    d[ins + "_per_wave"] = mean[ins] / mean["SQ_WAVES"]
        if mean.get("SQC_ICACHE_REQ"):
            d["icache_hit_rate"] = mean.get("SQC_ICACHE_HITS", 0) / mean["SQC_ICACHE_REQ"]
            d["icache_misses_per_wave"] = mean.get("SQC_ICACHE_MISSES", 0) / max(mean.get("SQ_WAVES", 1), 1)
        if mean.get("SQ_IFETCH"):
            d["ifetch_per_wave"] = mean["SQ_IFETCH"] / max(mean.get("SQ_WAVES", 1), 1)
            if "SQ_IFETCH_LEVEL" in mean:
                d["ifetch_level_avg"] = mean["SQ_IFETCH_LEVEL"] / mean["SQ_IFETCH"]
        if "FETCH_SIZE" in mean:
            d["fetch_bytes"] = mean["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in mean:
            d["write_bytes"] = mean["WRITE_SIZE"] * 1024
        if "TCC_EA0_RDREQ" in mean:
            d["rdreq_bytes_64B"] = mean["TCC_EA0_RDREQ"] * 64
            d["wrreq_bytes_64B"] = mean.get("TCC_EA0_WRREQ", 0) * 64
        name = a.rollout_key if k == "k_rollout" else k
        summary["kernels"][name] = d
        summary["sources"][name] = a.pmc_dir
        if name in ("k_step", a.rollout_key) and "fetch_bytes" in d and "write_bytes" in d:
            summary["hbm_bytes_per_launch"][name] = round(d["fetch_bytes"] + d["write_bytes"])
            summary["steps_per_launch"][name] = 1 if name == "k_step" else a.rollout_steps
    summary["hbm_bytes_note"] = ("FETCH_SIZE + WRITE_SIZE (KiB x 1024) per launch, uncorrected: the kernels' reads "
                                 "are 4-byte-per-lane planes and gathers, outside the guide's 16 B/lane calibration")
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    print(json.dumps({k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()
                          if kk != "counters_mean_per_dispatch"} for k, v in summary["kernels"].items()}, indent=1))
    print("hbm_bytes_per_launch", summary["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()

"""Average a rocprofv3 kernel trace over bench.py's TIMED launches only.

    python tools/trace_timed.py TRACE_CSV BENCH_STDERR [--out JSON]

bench.py prints a JSON line at the start and end of every timed region (region_mark: the region's
name, the kernel it times, how many launches of it the region holds, and CLOCK_BOOTTIME /
CLOCK_MONOTONIC stamps).  rocprofv3 --kernel-trace writes every dispatch with start/end timestamps.
For each region this picks the dispatches of its kernel that ran between the region's edges (trying
both clocks: the one that yields exactly the planned number of launches is used) and reports their
min / median / max / mean duration beside the all-launch average of that kernel (what the
--stats summary row shows, warm-up launches included).  VERDICT r03 item 1.
"""
import argparse
import csv
import json
import statistics
import sys


def load_trace(path):
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("KernelName") or ""
            try:
                t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            except (KeyError, ValueError):
                continue
            rows.append((name, t0, t1))
    return rows


def load_regions(path):
    regions, open_ = [], {}
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line.startswith("{") or "timed_region" not in line:
                continue
            try:
                rec = json.loads(line)
            except ValueError:
                continue
            if rec["edge"] == "start":
                open_[rec["timed_region"]] = rec
            elif rec["timed_region"] in open_:
                st = open_.pop(rec["timed_region"])
                regions.append({"name": st["timed_region"], "kernel": st.get("kernel"), "launches": st.get("launches"),
                                "boottime": (st["boottime_ns"], rec["boottime_ns"]),
                                "monotonic": (st["monotonic_ns"], rec["monotonic_ns"])})
    return regions


def matches(name, kernel):
    """rocprofv3 names carry the namespace and argument list: 'spl::k_rollout_store_2p(spl::KArena, ...)',
    'void splp32::k_act32<true, true>(unsigned char const*, ...)'."""
    base = name.split("(")[0].replace("void ", "").strip()
    return base == kernel or base.endswith("::" + kernel)


def summarise(trace, regions):
    out = {}
    for reg in regions:
        k = reg["kernel"]
        if not k:
            continue
        every = [(t1 - t0) / 1e3 for n, t0, t1 in trace if matches(n, k)]
        pick, clock = None, None
        for c in ("boottime", "monotonic"):
            a, b = reg[c]
            sel = [(t1 - t0) / 1e3 for n, t0, t1 in trace if matches(n, k) and t0 >= a and t1 <= b]
            if sel and (pick is None or len(sel) == reg["launches"]):
                pick, clock = sel, c
                if len(sel) == reg["launches"]:
                    break
        rec = {"kernel": k, "planned_launches": reg["launches"], "all_launches": len(every),
               "all_avg_us": round(statistics.fmean(every), 2) if every else None}
        if pick:
            rec.update(timed_launches=len(pick), clock=clock, timed_avg_us=round(statistics.fmean(pick), 2),
                       timed_median_us=round(statistics.median(pick), 2), timed_min_us=round(min(pick), 2),
                       timed_max_us=round(max(pick), 2))
        out[reg["name"]] = rec
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("stderr")
    ap.add_argument("--out")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    res = {"source": a.source, "regions": summarise(load_trace(a.trace), load_regions(a.stderr))}
    txt = json.dumps(res, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    print(txt)
    if not res["regions"]:
        sys.exit(1)


if __name__ == "__main__":
    main()

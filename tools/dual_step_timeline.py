"""Per-kernel timeline of config-5 dual steps from a rocprofv3 kernel-trace CSV of
tools/bench_selfplay.py: each dual step starts at the agent's k_act32<true, true> launch.
    python tools/dual_step_timeline.py run_kernel_trace.csv [--first 40] [--count 4]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--first", type=int, default=40)
    ap.add_argument("--count", type=int, default=4)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_act32<true, true>" in r["Kernel_Name"]]
    print(f"rocprofv3 --kernel-trace of tools/bench_selfplay.py --opponent pool: dual steps {a.first}.."
          f"{a.first + a.count - 1} of {len(starts) - 1} (time from the step's first launch, duration, gap, kernel)")
    for k in range(a.first, min(a.first + a.count, len(starts) - 1)):
        i0, i1 = starts[k], starts[k + 1]
        t0, prev = int(rows[i0]["Start_Timestamp"]), None
        for r in rows[i0:i1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev) / 1e3 if prev is not None else 0.0
            print(f"step {k} {(s - t0) / 1e3:8.2f} dur {(e - s) / 1e3:8.2f} gap {gap:6.2f}  {r['Kernel_Name'][:80]}")
            prev = e
        print(f"step {k} period {(int(rows[i1]['Start_Timestamp']) - t0) / 1e3:.2f} us")


if __name__ == "__main__":
    main()

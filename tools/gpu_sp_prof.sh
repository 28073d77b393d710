# rocprofv3 kernel stats of the config-5 self-play loop (pool and frozen opponents)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for opp in pool frozen; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sp_$opp -o run -- \
      python3 tools/bench_selfplay.py --opponent $opp > gpurun_out/sp_prof_$opp.json 2> gpurun_out/sp_prof_err.txt || { tail -20 gpurun_out/sp_prof_err.txt; exit 1; }
  python3 - $opp <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/prof_sp_{sys.argv[1]}/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(sys.argv[1], r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Percentage"])
PY
done

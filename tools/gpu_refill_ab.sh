# rollout kernel time with the refill fused vs a separate k_refill launch (rocprof kernel stats)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for R in fused separate; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_refill_$R -o run -- \
    python3 bench.py --no-cpu-baseline --only --mode rollout --outputs store --refill $R --steps 512 --warmup 128 \
    > gpurun_out/refill_$R.json 2> gpurun_out/refill_$R.err || { tail -20 gpurun_out/refill_$R.err; exit 1; }
  python3 - "$R" <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/prof_refill_{sys.argv[1]}/run_kernel_stats.csv")):
    if "k_rollout" in r["Name"] or "k_refill" in r["Name"]:
        print(sys.argv[1], r["Name"][:60], r["Calls"], r["AverageNs"])
PY
done

# instruction-cache counters of the rollout kernel, per-step store vs in place
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in store inplace; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES SQ_WAVE_CYCLES \
      --kernel-include-regex "k_rollout" --output-format csv -d gpurun_out/ic_$V -o run -- \
      python3 bench.py --no-cpu-baseline --only --mode rollout --outputs $V --steps 128 --warmup 128 > gpurun_out/ic_$V.log 2>&1 || { tail -5 gpurun_out/ic_$V.log; exit 1; }
  python3 - $V <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f"gpurun_out/ic_{sys.argv[1]}/run_counter_collection.csv")):
    acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
d = {k: acc[k] / max(1, len({1})) for k in acc}
print(sys.argv[1], {k: round(v) for k, v in acc.items()}, "rows", dict(n))
PY
done

#!/bin/bash
# Kernel-trace durations of ablation builds (tools/ablate.py variants), one rocprofv3 run each.
set -o pipefail
TAG=${1:-r01}
shift
OUT=gpurun_out/ablate_trace_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "k_step" --output-format csv \
      -d $OUT/$v -o run -- python3 tools/ablate.py --run $v > $OUT/$v.log 2>&1 || { echo "variant $v failed"; exit 1; }
  python3 - "$OUT/$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(f[0])):
    if "k_step" in r["Name"]:
        print(f"{sys.argv[2]:20s} k_step calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1000:7.2f} us  min {float(r['MinNs'])/1000:7.2f} us")
PY
done

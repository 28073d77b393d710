#!/bin/bash
# Parameter sweep of the headline bench (rollout launch length K, refill placement); one JSON line each.
set -o pipefail
TAG=${1:-sw}
O=gpurun_out
mkdir -p $O
: > $O/sweep_$TAG.jsonl
for cfg in "16 separate" "16 fused" "32 fused" "64 separate" "64 fused"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --only --rollout-k $1 --refill $2 >> $O/sweep_$TAG.jsonl 2>> $O/sweep_$TAG.err || { echo "fail $cfg"; exit 1; }
done
python - <<PY
import json
for l in open("$O/sweep_$TAG.jsonl"):
    d=json.loads(l); c=d["config"]; r=d["roofline"]
    print(c["rollout_steps_per_launch"], c["refill"], f'{d["value"]:.4e}', r["kernel_avg_us"], r["frac"], d["error_flags"], d["episodes"])
PY

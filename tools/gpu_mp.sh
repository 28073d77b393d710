#!/bin/bash
# 3-4 player rollout kernels: parity of both rollout kernels, then bench lines per kernel choice.
set -o pipefail
TAG=${1:-mp}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "rollout" > $O/pt_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/pt_$TAG.log; exit 1; }
tail -1 $O/pt_$TAG.log
: > $O/mp_$TAG.jsonl
IFS=',' read -ra CFG_LIST <<< "${CFGS:-4 65536 auto,4 65536 off,3 65536 auto,3 65536 off,4 32768 auto,3 32768 auto,2 65536 auto}"
for cfg in "${CFG_LIST[@]}"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu-baseline --only --players $1 --tables $2 --pipeline $3 >> $O/mp_$TAG.jsonl 2>> $O/mp_$TAG.err || { echo "fail $cfg"; exit 1; }
done
python - <<PY
import json
for l in open("$O/mp_$TAG.jsonl"):
    d=json.loads(l); c=d["config"]; r=d["roofline"]
    print(c["players"], c["tables_per_gpu"], c["pipeline"], c["refill_every"], f'{d["value"]:.4e}', r["kernel_avg_us"], r["frac"], d["error_flags"])
PY

#!/bin/bash
# The driver's bench command three times (timed-region diagnostics on stderr).
set -o pipefail
O=gpurun_out
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/dc_$i.json 2> $O/dc_$i.err || { tail -20 $O/dc_$i.err; exit 1; }
  grep "rollout_store.*timed region" $O/dc_$i.err
  python3 -c "import json;d=json.load(open('$O/dc_$i.json'));print(d['value'], d['roofline']['kernel_avg_us'])"
done

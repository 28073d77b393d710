#!/bin/bash
# Rollout launch length A/B: K = 64 vs 128 steps per spl_rollout launch (store headline), two passes.
set -o pipefail
O=gpurun_out
mkdir -p $O
for pass in 1 2; do
  for k in 64 128; do
    timeout -k 10 200 python3 bench.py --only --no-cpu-baseline --steps 512 --warmup 128 --rollout-k $k > $O/rk_$k.json 2> $O/rk_$k.err || { tail -5 $O/rk_$k.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/rk_$k.json'));print('pass $pass K=$k', d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'])"
  done
done

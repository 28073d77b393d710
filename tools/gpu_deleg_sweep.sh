#!/bin/bash
# Rollout-store delegation period sweep (bench.py --only, 512 timed steps), two passes.
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/deleg_sweep.txt
for pass in 1 2; do
  for d in 0 4 5 6 8 12; do
    timeout -k 10 120 python3 bench.py --only --no-cpu-baseline --steps 512 --warmup 128 --delegation $d > $O/deleg_$d.json 2> $O/deleg_$d.err || { tail -5 $O/deleg_$d.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/deleg_$d.json'));print('pass $pass deleg $d', d['value'], d['roofline']['kernel_avg_us'])" | tee -a $O/deleg_sweep.txt
  done
done

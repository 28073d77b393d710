#!/bin/bash
# Sensitivity of the rollout-store kernel to the rules work: bench.py --only (store headline) on
# -DSPL_ABL builds (splendor-gym_amd/ablate/lib_<v>.so; wrong trajectories by design), two passes.
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/abl_store.txt
for pass in 1 2; do
  for v in $VARIANTS; do
    SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_$v.so timeout -k 10 120 python3 bench.py --only --no-cpu-baseline --steps 256 --warmup 128 > $O/abl_$v.json 2> $O/abl_$v.err || { tail -5 $O/abl_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/abl_$v.json'));print('pass $pass $v', d['value'], d['roofline']['kernel_avg_us'])" | tee -a $O/abl_store.txt
  done
done

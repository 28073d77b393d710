#!/bin/bash
# Step-mode A/B of library variants (ablate/lib_<v>.so): bench.py --only --mode step, two passes.
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/step_var.txt
for pass in 1 2; do
  for v in $VARIANTS; do
    SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_$v.so timeout -k 10 120 python3 bench.py --only --mode step --no-cpu-baseline --steps 1024 --warmup 128 > $O/sv_$v.json 2> $O/sv_$v.err || { tail -5 $O/sv_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/sv_$v.json'));print('pass $pass $v', d['value'], d['roofline']['kernel_avg_us'], d['roofline'].get('eager_launch_us'))" | tee -a $O/step_var.txt
  done
done

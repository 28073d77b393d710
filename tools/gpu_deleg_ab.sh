#!/bin/bash
# Delegation payload A/B: parity tests of the rollout kernels on the in-tree library, then the store
# headline on ablate/lib_old.so vs lib_new.so (two passes) and the new library at other periods.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/deleg_tests.log 2>&1 || { tail -30 $O/deleg_tests.log; exit 1; }
tail -1 $O/deleg_tests.log
: > $O/deleg_ab.txt
for pass in 1 2; do
  for v in old new; do
    SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_$v.so timeout -k 10 120 python3 bench.py --only --no-cpu-baseline --steps 512 --warmup 128 > $O/dab_$v.json 2> $O/dab_$v.err || { tail -5 $O/dab_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/dab_$v.json'));print('pass $pass $v', d['value'], d['roofline']['kernel_avg_us'])" | tee -a $O/deleg_ab.txt
  done
done
for d in 4 5 8; do
  timeout -k 10 120 python3 bench.py --only --no-cpu-baseline --steps 512 --warmup 128 --delegation $d > $O/dab_d$d.json 2> $O/dab_d$d.err || { tail -5 $O/dab_d$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/dab_d$d.json'));print('new deleg $d', d['value'], d['roofline']['kernel_avg_us'])" | tee -a $O/deleg_ab.txt
done

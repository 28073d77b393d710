#!/bin/bash
# Self-play A/B of library variants (ablate/lib_<v>.so): tools/bench_selfplay.py (pool and frozen),
# two passes; then the policy and opponent-pool GPU tests on the in-tree library.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_opponent_pool.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/spv_tests.log 2>&1 || { tail -30 $O/spv_tests.log; exit 1; }
tail -1 $O/spv_tests.log
: > $O/sp_var.txt
for pass in 1 2; do
  for v in $VARIANTS; do
    for opp in pool frozen; do
      SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_$v.so timeout -k 10 200 python3 tools/bench_selfplay.py --opponent $opp > $O/spv_$v.json 2> $O/spv_$v.err || { tail -5 $O/spv_$v.err; exit 1; }
      python3 -c "import json;d=json.load(open('$O/spv_$v.json'));print('pass $pass $v $opp', d['value'], d['ms_per_dual_step'])" | tee -a $O/sp_var.txt
    done
  done
done

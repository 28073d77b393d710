#!/bin/bash
# A/B of fp32 actor builds (VARIANTS, splendor-gym_amd/ablate/lib_pol_<v>.so): bench_policy twice each,
# alternating, then the policy GPU tests against each variant library.
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/pol_ab.txt
for pass in 1 2; do
  for v in $VARIANTS; do
    SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_pol_$v.so timeout -k 10 300 python tools/bench_policy.py --iters 20 --fused-only > $O/pol_$v.json 2> $O/pol_$v.err || { tail -20 $O/pol_$v.err; exit 1; }
    echo "pass $pass $v $(cat $O/pol_$v.json)" | tee -a $O/pol_ab.txt
  done
done
for v in $TEST_VARIANTS; do
  SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_pol_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pol_tests_$v.log 2>&1 || { tail -30 $O/pol_tests_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pol_tests_$v.log)" | tee -a $O/pol_ab.txt
done

#!/bin/bash
# GPU session for the fused policy kernel: its tests, then the microbench.
set -o pipefail
TAG=${1:-p}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_policy.py -x -q > $OUT/pytest_policy_$TAG.log 2>&1 || { echo "policy tests failed"; tail -40 $OUT/pytest_policy_$TAG.log; exit 1; }
tail -2 $OUT/pytest_policy_$TAG.log
timeout -k 10 300 python tools/bench_policy.py > $OUT/bench_policy_$TAG.json 2> $OUT/bench_policy_$TAG.err || { echo "bench failed"; tail -20 $OUT/bench_policy_$TAG.err; exit 1; }
cat $OUT/bench_policy_$TAG.json

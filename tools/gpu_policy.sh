#!/bin/bash
# GPU session for the fused policy kernel: its tests, the microbench, the config-5 self-play bench.
set -o pipefail
TAG=${1:-p}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_parity.py -x -q -k "policy or greedy or sample or refresh or dual or selfplay or fused" --timeout 200 --timeout-method thread > $OUT/pytest_policy_$TAG.log 2>&1 || { echo "policy tests failed"; tail -40 $OUT/pytest_policy_$TAG.log; exit 1; }
tail -2 $OUT/pytest_policy_$TAG.log
timeout -k 10 300 python tools/bench_policy.py > $OUT/bench_policy_$TAG.json 2> $OUT/bench_policy_$TAG.err || { echo "bench failed"; tail -20 $OUT/bench_policy_$TAG.err; exit 1; }
cat $OUT/bench_policy_$TAG.json
timeout -k 10 300 python tools/bench_selfplay.py > $OUT/sp_$TAG.json 2> $OUT/sp_$TAG.err || { tail -20 $OUT/sp_$TAG.err; exit 1; }
cat $OUT/sp_$TAG.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_pol_$TAG -o run -- python3 tools/bench_policy.py --fused-only --iters 20 > /dev/null 2>&1 || { echo "rocprof failed"; exit 1; }
grep -h 'k_act' $OUT/prof_pol_$TAG/run_kernel_stats.csv

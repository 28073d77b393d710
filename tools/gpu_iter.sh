#!/bin/bash
# Iteration check on one GPU: parity suite, headline sweep (rollout K, refill placement), rollout
# stamp timeline.  Stops at the first failing step.
set -o pipefail
TAG=${1:-it}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pt_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $O/pt_$TAG.log; exit 1; }
tail -1 $O/pt_$TAG.log
bash tools/gpu_sweep.sh $TAG || exit 1
[ "${STAMPS:-0}" = "1" ] && timeout -k 10 200 python tools/rstamps.py --run > $O/rstamps_$TAG.txt 2>&1 && cat $O/rstamps_$TAG.txt; true

#!/bin/bash
# Round-3 check of the narrow-tail grouped actor and the k_step_ws terminal-row change: the new
# opponent-pool tests first (tight limit), the full GPU suite, then step mode and config 5.
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_opponent_pool.py -x -v --timeout 200 --timeout-method thread \
    > $O/pool_first_r03i.log 2>&1 || { echo "pool tests failed"; tail -40 $O/pool_first_r03i.log; exit 1; }
tail -4 $O/pool_first_r03i.log
bash tools/gpu_session.sh r03i tests stepmode selfplay

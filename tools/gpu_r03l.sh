#!/bin/bash
# split row encode in k_step_ws: step-path tests, step-mode bench + profile, self-play benches + profile
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_env_api.py tests/test_gpu_opponent_pool.py \
    -x -v --timeout 200 --timeout-method thread > $O/tests_r03l.log 2>&1 || { echo "tests failed"; tail -40 $O/tests_r03l.log; exit 1; }
tail -3 $O/tests_r03l.log
bash tools/gpu_session.sh r03l stepmode selfplay || exit 1
bash tools/gpu_sp_prof.sh

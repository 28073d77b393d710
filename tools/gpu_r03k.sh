#!/bin/bash
# grouped actor (narrow tails, 16 waves): opponent-pool tests, self-play benches, self-play profile
set -o pipefail
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_opponent_pool.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread \
    > $O/pool_r03k.log 2>&1 || { echo "tests failed"; tail -40 $O/pool_r03k.log; exit 1; }
tail -3 $O/pool_r03k.log
bash tools/gpu_session.sh r03k selfplay || exit 1
bash tools/gpu_sp_prof.sh

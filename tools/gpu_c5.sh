#!/bin/bash
# GPU session: full parity suite, then the config-5 self-play bench (fused actor) + kernel stats.
set -o pipefail
TAG=${1:-c5}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $O/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest_gpu_$TAG.log; exit 1; }
tail -1 $O/pytest_gpu_$TAG.log
timeout -k 10 300 python tools/bench_selfplay.py > $O/sp_$TAG.json 2> $O/sp_$TAG.err || { tail -20 $O/sp_$TAG.err; exit 1; }
cat $O/sp_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_sp_$TAG -o run -- python3 tools/bench_selfplay.py --iters 32 > $O/sp_prof_$TAG.json 2> $O/sp_prof_$TAG.err
echo rc $?

#!/bin/bash
# One GPU session: bench (JSON line) + rocprofv3 kernel-trace stats of the same command.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --steps 200 --warmup 50 > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err
echo "exit $?"

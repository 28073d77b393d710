#!/bin/bash
# One GPU session: [parity tests] bench (JSON line), rocprofv3 kernel-trace stats of the bench,
# PMC passes.  Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
TAG=${1:-r01}
TESTS=${2:-1}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -x -q -m gpu --durations=8 > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
fi
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --steps 256 --warmup 64 > $OUT/bench_prof_$TAG.json 2> $OUT/bench_prof_$TAG.err && \
bash tools/pmc.sh $TAG
echo "exit $?"

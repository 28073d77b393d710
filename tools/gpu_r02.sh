#!/bin/bash
# Round-2 GPU session: parity suite, smoke, the driver's bench command, the default bench line, and
# rocprofv3 kernel-trace stats of the headline variant.  Every GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
TAG=${1:-r02a}
TESTS=${2:-1}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
if [ "$TESTS" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 \
      > $O/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest_gpu_$TAG.log; exit 1; }
  tail -3 $O/pytest_gpu_$TAG.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_$TAG.log; exit 1; }
  tail -1 $O/smoke_$TAG.log
fi
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$TAG.json 2> $O/bench_driver_$TAG.err || { tail -20 $O/bench_driver_$TAG.err; exit 1; }
cat $O/bench_driver_$TAG.json
timeout -k 10 600 python3 bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --steps 1024 --warmup 128 > $O/bench_prof_$TAG.json 2> $O/bench_prof_$TAG.err || { tail -20 $O/bench_prof_$TAG.err; exit 1; }
echo "done"

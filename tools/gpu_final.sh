#!/bin/bash
# Round-end verification on one GPU: full parity suite, smoke(), headline bench (JSON line),
# rocprofv3 kernel-trace stats of the bench, config-5 self-play bench.  Each GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
TAG=${1:-fin}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest_gpu_$TAG.log; exit 1; }
tail -1 $O/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_$TAG.log; exit 1; }
tail -1 $O/smoke_$TAG.log
timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --steps 256 --warmup 64 > $O/bench_prof_$TAG.json 2> $O/bench_prof_$TAG.err || { echo "rocprof failed"; exit 1; }
head -5 $O/prof_$TAG/run_kernel_stats.csv
timeout -k 10 300 python tools/bench_selfplay.py > $O/sp_$TAG.json 2> $O/sp_$TAG.err || { tail -20 $O/sp_$TAG.err; exit 1; }
cat $O/sp_$TAG.json

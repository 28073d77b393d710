#!/bin/bash
# Round-2 re-entry: tools/gpu_final.sh, the driver's bench command, then the rollout with the pool
# refill as a separate k_refill launch (what the fused deal costs the rollout kernel).
set -o pipefail
TAG=${1:-r02o}
O=gpurun_out
bash tools/gpu_final.sh $TAG || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$TAG.json 2> $O/bench_driver_$TAG.err || { tail -20 $O/bench_driver_$TAG.err; exit 1; }
cat $O/bench_driver_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_sep_$TAG -o run -- \
    python3 bench.py --no-cpu-baseline --only --refill separate --steps 256 --warmup 64 > $O/bench_sep_$TAG.json 2> $O/bench_sep_$TAG.err || { tail -20 $O/bench_sep_$TAG.err; exit 1; }
head -6 $O/prof_sep_$TAG/run_kernel_stats.csv

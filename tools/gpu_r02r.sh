#!/bin/bash
# Round-2 closing check: tools/gpu_final.sh, the driver's bench command, and a 2-rank rehearsal of
# the driver's torch.distributed.run bench on one card (gloo; both ranks share the GPU).
set -o pipefail
TAG=${1:-r02r}
O=gpurun_out
bash tools/gpu_final.sh $TAG || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$TAG.json 2> $O/bench_driver_$TAG.err || { tail -20 $O/bench_driver_$TAG.err; exit 1; }
cut -c1-300 $O/bench_driver_$TAG.json
SPLENDOR_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_2rank_$TAG.json 2> $O/bench_2rank_$TAG.err || { tail -30 $O/bench_2rank_$TAG.err; exit 1; }
cut -c1-300 $O/bench_2rank_$TAG.json

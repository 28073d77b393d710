# Round-2: 3/4-player store headline lines (C4's per-GPU share is 4p x 32768) and a 2-rank
# rehearsal of the driver's multi-GPU bench on one card (gloo; both ranks share the GPU)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/mp_r02.jsonl
for cfg in "3 65536" "4 65536" "4 32768"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --players $1 --tables $2 --steps 256 --warmup 128 >> gpurun_out/mp_r02.jsonl 2> gpurun_out/mp_err.txt || { tail -20 gpurun_out/mp_err.txt; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/mp_r02.jsonl"):
    d = json.loads(l); c = d["config"]
    print(c["players"], c["tables_per_gpu"], d["value"], d["roofline"]["kernel_avg_us"], d["roofline"]["frac"],
          "| inplace", d["in_place_l3"]["value"], "| step", d["other_mode"]["value"], d["other_mode"]["roofline"]["kernel_avg_us"])
PY
SPLENDOR_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_2rank_r02.json 2> gpurun_out/bench_2rank_r02.err || { tail -30 gpurun_out/bench_2rank_r02.err; exit 1; }
cut -c1-400 gpurun_out/bench_2rank_r02.json

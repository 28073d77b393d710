set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for p in always half; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --sp-tables 0 --c4-tables 0 --pipeline $p > gpurun_out/pipe_${p}_$r.json 2>gpurun_out/pipe_${p}_$r.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/pipe_${p}_$r.json').read().strip().splitlines()[-1]); print('$p', $r, d['value'], d['roofline']['kernel_avg_us'], d['roofline']['kernel'])"
done; done

#!/bin/bash
# Timed-region diagnostics of the driver's short bench command (host enqueue, GPU span, wall).
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/diag_a.json 2> $O/diag_a.err || { tail -20 $O/diag_a.err; exit 1; }
grep "timed region" $O/diag_a.err
python3 -c "import json;d=json.load(open('$O/diag_a.json'));print(d['value'],d['roofline']['kernel_avg_us'])"

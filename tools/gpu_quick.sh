#!/bin/bash
# GPU session: parity tests, stamps timeline, bench (both modes).  Stops at the first failure.
set -o pipefail
TAG=${1:-q}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -2 $OUT/pytest_gpu_$TAG.log
if [ -z "$NO_STAMPS" ]; then
  timeout -k 10 500 python tools/stamps.py --run > $OUT/stamps_$TAG.txt 2>&1 || { echo "stamps failed"; exit 1; }
  cat $OUT/stamps_$TAG.txt
fi
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -20 $OUT/bench_$TAG.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_$TAG.json'))
print('MAIN', d['config']['mode'], 'VALUE', d['value'], 'ms/step', d['ms_per_step'], 'kernel us', d['roofline']['kernel_avg_us'], 'frac', d['roofline']['frac'])
o=d.get('other_mode')
if o: print('OTHER', o['mode'], 'VALUE', o['value'], 'ms/step', o['ms_per_step'], 'kernel us', o['roofline']['kernel_avg_us'], 'frac', o['roofline']['frac'])
"

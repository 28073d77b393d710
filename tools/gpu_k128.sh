#!/bin/bash
# 128-step rollout launches: the headline and delegation GPU tests, the bench, and the PMC passes of
# the store and in-place variants at K = 128.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -x -q -m gpu --timeout 400 --timeout-method thread > $O/k128_tests.log 2>&1 || { tail -30 $O/k128_tests.log; exit 1; }
tail -1 $O/k128_tests.log
timeout -k 10 400 python3 bench.py > $O/bench_k128.json 2> $O/bench_k128.err || { tail -20 $O/bench_k128.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_k128.json'));print(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac'], d['steps'])"
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" VARIANT=store bash tools/pmc.sh k128s || exit 1
PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" VARIANT=inplace bash tools/pmc.sh k128i || exit 1

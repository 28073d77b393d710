set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -x -v -k "dealer" --timeout 120 --timeout-method thread > gpurun_out/dealer_first.log 2>&1 || { echo "dealer tests failed rc=$?"; tail -40 gpurun_out/dealer_first.log; exit 1; }
tail -8 gpurun_out/dealer_first.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r03d.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_gpu_r03d.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r03d.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --players 4 --tables 32768 > gpurun_out/bench_4p_32768_r03d.json 2> gpurun_out/bench_4p_32768_r03d.err || { tail -20 gpurun_out/bench_4p_32768_r03d.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_4p_32768_r03d.json').read().splitlines()[-1]); r=d['roofline']
print(d['value'], r['kernel'], r['kernel_avg_us'], r['frac'])"

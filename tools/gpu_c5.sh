# config 5 with the reference's trained checkpoint: tests + self-play bench (frozen and pool opponents)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_headline.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 || { tail -30 gpurun_out/c5_tests.log; exit 1; }
tail -1 gpurun_out/c5_tests.log
for opp in frozen pool; do
  timeout -k 10 300 python tools/bench_selfplay.py --opponent $opp > gpurun_out/sp_trained_$opp.json 2> gpurun_out/sp_err.txt || { tail -20 gpurun_out/sp_err.txt; exit 1; }
  cut -c1-300 gpurun_out/sp_trained_$opp.json
done
timeout -k 10 300 python tools/bench_selfplay.py --opponent frozen --weights random > gpurun_out/sp_random_frozen.json 2> gpurun_out/sp_err.txt || { tail -20 gpurun_out/sp_err.txt; exit 1; }
cut -c1-300 gpurun_out/sp_random_frozen.json

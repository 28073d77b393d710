# A/B of library builds on the config-5 self-play bench (pool and frozen opponents) + the pool tests
set -o pipefail
mkdir -p gpurun_out
for v in $VARIANTS; do
  for opp in pool frozen; do
    SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python tools/bench_selfplay.py --opponent $opp > gpurun_out/sp_$v_$opp.json 2> gpurun_out/sp_err.txt || { tail -20 gpurun_out/sp_err.txt; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/sp_$v_$opp.json').read().strip().splitlines()[-1]); print('$v', '$opp', d['value'], d['ms_per_dual_step'], d['env_only']['ms_per_dual_step'])"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_opponent_pool.py tests/test_gpu_headline.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/sp_tests.log 2>&1 || { tail -30 gpurun_out/sp_tests.log; exit 1; }
tail -1 gpurun_out/sp_tests.log

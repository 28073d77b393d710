# A/B of the fp32 actor builds (bench_policy) + the policy and config-5 GPU tests on the default library
set -o pipefail
mkdir -p gpurun_out
for v in $VARIANTS; do
  SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python tools/bench_policy.py --iters 20 --fused-only > gpurun_out/pol_$v.json 2> gpurun_out/pol_$v.err || { tail -20 gpurun_out/pol_$v.err; exit 1; }
  echo $v $(cat gpurun_out/pol_$v.json)
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_headline.py tests/test_gpu_opponent_pool.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pol_tests.log 2>&1 || { tail -30 gpurun_out/pol_tests.log; exit 1; }
tail -1 gpurun_out/pol_tests.log

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_opponent_pool.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_pol_r03r.out 2>&1 || { tail -60 gpurun_out/pytest_pol_r03r.out; exit 1; }
tail -5 gpurun_out/pytest_pol_r03r.out
bash tools/gpu_session.sh r03r policy selfplay

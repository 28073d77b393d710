# round-3 fp32-actor session: policy / pool / self-play GPU tests, then the policy benches, the
# k_act32 ablations and the self-play kernel profile.  TAG = $1
set -o pipefail
T=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_opponent_pool.py tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_pol_$T.out 2>&1 || { tail -60 gpurun_out/pytest_pol_$T.out; exit 1; }
tail -3 gpurun_out/pytest_pol_$T.out
bash tools/gpu_session.sh $T policy selfplay || exit 1
bash tools/ablate_policy32.sh || exit 1
bash tools/gpu_sp_prof.sh

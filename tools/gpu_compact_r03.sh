# round-3 compact-observation session: its GPU tests + the dual-step / policy tests, then the
# self-play benches and kernel profile.  TAG = $1
set -o pipefail
T=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact_obs.py tests/test_gpu_policy.py tests/test_gpu_opponent_pool.py tests/test_gpu_headline.py tests/test_wrappers.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_compact_$T.out 2>&1 || { tail -60 gpurun_out/pytest_compact_$T.out; exit 1; }
tail -3 gpurun_out/pytest_compact_$T.out
bash tools/gpu_session.sh $T selfplay || exit 1
bash tools/gpu_sp_prof.sh

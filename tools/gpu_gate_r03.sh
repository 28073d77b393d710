# round-3 fused-gate session: dual-step / self-play GPU tests, then the self-play benches and profile.
set -o pipefail
T=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_opponent_pool.py tests/test_gpu_headline.py tests/test_wrappers.py tests/test_gpu_compact_obs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gate_$T.out 2>&1 || { tail -60 gpurun_out/pytest_gate_$T.out; exit 1; }
tail -3 gpurun_out/pytest_gate_$T.out
bash tools/gpu_session.sh $T selfplay || exit 1
bash tools/gpu_sp_prof.sh

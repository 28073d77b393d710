#!/bin/bash
# Round-2 GPU session: parity suite, smoke, the driver's bench command, the default bench line, and
# rocprofv3 kernel-trace stats of the headline variant.  Every GPU step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
TAG=${1:-r02a}
TESTS=${2:-1}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
if [ "$TESTS" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=10 \
      > $O/pytest_gpu_$TAG.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest_gpu_$TAG.log; exit 1; }
  tail -3 $O/pytest_gpu_$TAG.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke_$TAG.log; exit 1; }
  tail -1 $O/smoke_$TAG.log
fi
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$TAG.json 2> $O/bench_driver_$TAG.err || { tail -20 $O/bench_driver_$TAG.err; exit 1; }
cat $O/bench_driver_$TAG.json
timeout -k 10 600 python3 bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -20 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
# the default bench command itself; full kernel names keep k_rollout_ws<2, 64, true> (per-step store,
# the headline) apart from <2, 64, false> (in place)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- \
    python3 bench.py > $O/bench_prof_$TAG.json 2> $O/bench_prof_$TAG.err || { tail -20 $O/bench_prof_$TAG.err; exit 1; }
echo "done"
timeout -k 10 300 python tools/bench_selfplay.py > $O/sp_pool_$TAG.json 2> $O/sp_pool_$TAG.err || { tail -20 $O/sp_pool_$TAG.err; exit 1; }
cat $O/sp_pool_$TAG.json
timeout -k 10 300 python tools/bench_selfplay.py --opponent frozen > $O/sp_frozen_$TAG.json 2> $O/sp_frozen_$TAG.err || { tail -20 $O/sp_frozen_$TAG.err; exit 1; }
cat $O/sp_frozen_$TAG.json
timeout -k 10 300 python tools/bench_policy.py --iters 20 > $O/policy_$TAG.json 2> $O/policy_$TAG.err || { tail -20 $O/policy_$TAG.err; exit 1; }
cat $O/policy_$TAG.json
if [ "${PMC:-0}" = "1" ]; then
  VARIANT=store bash tools/pmc.sh ${TAG}_store || exit 1
  python tools/pmc_summary.py $O/pmc_${TAG}_store $O/pmc_summary_${TAG}.json --rollout-steps 64 --rollout-key k_rollout_store || exit 1
  VARIANT=inplace bash tools/pmc.sh ${TAG}_inplace || exit 1
  python tools/pmc_summary.py $O/pmc_${TAG}_inplace $O/pmc_summary_${TAG}.json --merge --rollout-steps 64 --rollout-key k_rollout || exit 1
  VARIANT=step bash tools/pmc.sh ${TAG}_step || exit 1
  python tools/pmc_summary.py $O/pmc_${TAG}_step $O/pmc_summary_${TAG}.json --merge || exit 1
fi
echo "all done"

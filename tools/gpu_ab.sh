# A/B of experiment builds on the headline (rollout store) and step mode, then the GPU suite on the
# default library.  VARIANTS = names built by tools/variants.py.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/variants.py bench $VARIANTS -- --only --mode rollout --outputs store --steps 512 --warmup 128 > gpurun_out/ab_roll.txt 2>&1 || { tail -20 gpurun_out/ab_roll.txt; exit 1; }
cut -c1-200 gpurun_out/ab_roll.txt
timeout -k 10 600 python tools/variants.py bench $VARIANTS -- --only --mode step --steps 1024 --warmup 128 > gpurun_out/ab_step.txt 2>&1 || { tail -20 gpurun_out/ab_step.txt; exit 1; }
cut -c1-200 gpurun_out/ab_step.txt
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi

# A/B of experiment builds in step mode (spl_step per env step), then the GPU suite and smoke() on
# the default library.  VARIANTS = names built by tools/variants.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/variants.py bench $VARIANTS -- --only --mode step --steps 1024 --warmup 128 > gpurun_out/ab_step.txt 2>&1 || { tail -20 gpurun_out/ab_step.txt; exit 1; }
cut -c1-300 gpurun_out/ab_step.txt
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab_smoke.log 2>&1 || { tail -20 gpurun_out/ab_smoke.log; exit 1; }
  tail -1 gpurun_out/ab_smoke.log
fi

# A/B of spl_step kernels (variants built by tools/variants.py) + the GPU parity suite on the default library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/variants.py bench ${VARIANTS:-ws0 ws1} -- --only --mode step --steps 1024 --warmup 128 > gpurun_out/sw_bench.txt 2>&1 || { tail -20 gpurun_out/sw_bench.txt; exit 1; }
cut -c1-300 gpurun_out/sw_bench.txt
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/sw_parity.log 2>&1 || { tail -30 gpurun_out/sw_parity.log; exit 1; }
tail -2 gpurun_out/sw_parity.log

# bench A/B of experiment builds (tools/variants.py) on the headline rollout_store variant
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python tools/variants.py bench $VARIANTS -- --only --mode rollout --outputs ${OUTPUTS:-store} --steps 512 --warmup 128 > gpurun_out/var_bench.txt 2>&1 || { tail -20 gpurun_out/var_bench.txt; exit 1; }
cut -c1-300 gpurun_out/var_bench.txt

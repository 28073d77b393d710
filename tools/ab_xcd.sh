#!/bin/bash
# XCD-contiguous workgroup map (SPL_XCD_MAP) A/B on one box: the parity tests on the product build,
# then lib_xmap0 / lib_xmap1 (tools/variants.py build xmap0=-DSPL_XCD_MAP=0 xmap1=-DSPL_XCD_MAP=1)
# alternating on the headline store rollout, the step kernel and C4's 4p x 32768 share.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=${1:?tag}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_env_api.py \
    -x -q --timeout 200 --timeout-method thread > $O/pytest_xmap_$TAG.txt 2>&1 || { tail -30 $O/pytest_xmap_$TAG.txt; exit 1; }
tail -2 $O/pytest_xmap_$TAG.txt
for r in 1 2 3; do
  timeout -k 10 300 python3 tools/variants.py bench xmap0 xmap1 -- --sp-tables 0 --c4-tables 0 >> $O/ab_xcd_store_$TAG.txt || exit 1
  timeout -k 10 300 python3 tools/variants.py bench xmap0 xmap1 -- --mode step --only --sp-tables 0 >> $O/ab_xcd_step_$TAG.txt || exit 1
  timeout -k 10 300 python3 tools/variants.py bench xmap0 xmap1 -- --players 4 --tables 32768 --sp-tables 0 --c4-tables 0 >> $O/ab_xcd_c4_$TAG.txt || exit 1
done
cat $O/ab_xcd_*_$TAG.txt

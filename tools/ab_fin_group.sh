# k_step_ws terminal rows four at a time (lib_fin4) vs one at a time (lib_fin1): the step parity tests on the
# in-tree library, stamps at 65 536 / 16 384 tables, then one-chain step timings alternating.  The variants:
#   python tools/variants.py build fin1=-DSPL_FIN_GROUP=1 fin4=-DSPL_FIN_GROUP=4   (at the commit that had
#   SPL_FIN_GROUP; the grouping was not kept, profiles/r05/fin_group_ab_r05zz4.txt)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_env_api.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fin_r05zz4.txt 2>&1 || exit 1
STAMP_T=65536 timeout -k 10 200 python3 tools/stamps.py --run > gpurun_out/stamps_step_65536_r05zz4.txt 2>&1 || exit 1
STAMP_T=16384 timeout -k 10 200 python3 tools/stamps.py --run > gpurun_out/stamps_step_16384_r05zz4.txt 2>&1 || exit 1
for i in 1 2; do for v in fin1 fin4; do for t in 65536 16384; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 150 python3 tools/bench_step_chains.py --tables $t --chains 1 --rounds 1 | sed "s/^/{\"variant\": \"$v\", \"r\": $i, \"d\": /; s/\$/}/" >> gpurun_out/fin_ab_r05zz4.jsonl || exit 1
done; done; done

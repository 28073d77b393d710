# k_step_ws terminal rows shared by the two waves (SPL_FIN_SPLIT=1, split1) vs all by the rules wave
# (split0): the step parity tests on the in-tree library, then one-chain step timings alternating.
# Variants: python tools/variants.py build split0=-DSPL_FIN_SPLIT=0 split1=-DSPL_FIN_SPLIT=1 (at the commit
# that had SPL_FIN_SPLIT; not kept, profiles/r05/fin_split_ab_r05zz7.txt)
set -o pipefail
T=${1:-r05zz7}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_env_api.py tests/test_gpu_compact_obs.py \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_split_$T.txt 2>&1 || exit 1
for i in 1 2 3; do for v in split0 split1; do for t in 65536 16384; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 150 python3 tools/bench_step_chains.py --tables $t \
      --chains 1 --rounds 1 | sed "s/^/{\"variant\": \"$v\", \"r\": $i, \"d\": /; s/\$/}/" >> gpurun_out/split_ab_$T.jsonl || exit 1
done; done; done

set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_env_api.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_fin_r05zz4.txt 2>&1 || exit 1
STAMP_T=65536 timeout -k 10 200 python3 tools/stamps.py --run > gpurun_out/stamps_step_65536_r05zz4.txt 2>&1 || exit 1
STAMP_T=16384 timeout -k 10 200 python3 tools/stamps.py --run > gpurun_out/stamps_step_16384_r05zz4.txt 2>&1 || exit 1
for i in 1 2; do for v in fin1 fin4; do for t in 65536 16384; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 150 python3 tools/bench_step_chains.py --tables $t --chains 1 --rounds 1 | sed "s/^/{\"variant\": \"$v\", \"r\": $i, \"d\": /; s/\$/}/" >> gpurun_out/fin_ab_r05zz4.jsonl || exit 1
done; done; done

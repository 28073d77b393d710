# round 6: the rollout store's terminal rows and small outputs (reward, terminated, flags, winner) through the
# sc0 nt sc1 stream too (smallnt, -DSPL_ROLL_SMALL_NT=1) against plain (base0 = the product), headline and C4's
# share, arms alternating on one box; then smallnt's rollout-equals-step-chain and headline parity tests
set -o pipefail
O=gpurun_out
T=${TAG:-r06ai}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], '%.4g' % d['value'])" $1; }
for i in 1 2 3; do for v in base0 smallnt; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 > $O/sn_head_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for i in 1 2; do for v in base0 smallnt; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 --players 4 --tables 32768 > $O/sn_c4_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/sn_*_$T.json; do pj $f; done
SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_smallnt.so timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_parity.py -x -q -k "headline_rollout or rollout_equals_step_chain" --timeout 300 --timeout-method thread > $O/pytest_smallnt_$T.out 2>&1; rc=$?; tail -2 $O/pytest_smallnt_$T.out; exit $rc

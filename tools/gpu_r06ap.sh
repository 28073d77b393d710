# round 6: the three-wave step's rows as sc1 buffer stores (tsc1, -DSPL_STEP_TAIL_CPOL=16) against its sc0 nt sc1
# rows (tref = the product), graph-replay HIP events per step at 16 384 / 32 768 / 49 152 tables and forced at
# 65 536 (where the product picks the two-wave shape with sc1 rows: also timed), arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06ap}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $1; }
for tb in 16384 32768 49152; do for i in 1 2; do for v in tref tsc1; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables $tb > $O/tp_${v}_${tb}_${i}_$T.json 2>/dev/null || exit 1
done; done; done
for i in 1 2; do for v in tref tsc1; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --step-tail 1 > $O/tp_${v}_65536w_${i}_$T.json 2>/dev/null || exit 1
done; done
SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_tref.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 > $O/tp_tref_65536auto_1_$T.json 2>/dev/null || exit 1
for f in $O/tp_*_$T.json; do pj $f; done

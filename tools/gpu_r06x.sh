# round 6: the drop-in step kernel's row stores (SPL_STEP_OBS_NT, plain by default) as non-temporal buffer stores
# (stepnt2: nt) and as sc0 nt sc1 (stepnt19), against the default (stepdef), graph-replay HIP events per step at
# 65 536 and 16 384 tables, arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06x}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $1; }
for tb in 65536 16384; do for i in 1 2 3; do for v in stepdef stepnt2 stepnt19; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables $tb > $O/step_${v}_${tb}_${i}_$T.json 2>/dev/null || exit 1
done; done; done
for f in $O/step_*_$T.json; do pj $f; done

# round 6: spl_step's mask block as sc1 buffer stores (msc1, -DSPL_STEP_MASK_CPOL=16) against plain (mref),
# graph-replay HIP events per step at 65 536 and 32 768 tables, arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06ar}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $1; }
for tb in 65536 32768; do for i in 1 2 3; do for v in mref msc1; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables $tb > $O/mk_${v}_${tb}_${i}_$T.json 2>/dev/null || exit 1
done; done; done
for f in $O/mk_*_$T.json; do pj $f; done

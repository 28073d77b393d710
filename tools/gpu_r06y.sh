# round 6: the three-wave step shape's int32 rows as sc0 nt sc1 stores (tailnt1, the new default) against plain
# stores (tailnt0), graph-replay HIP events per step at 32 768 / 16 384 / 4 096 tables and the one-table
# SplendorEnv.step call, arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06y}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $1; }
for tb in 32768 16384 4096; do for i in 1 2 3; do for v in tailnt1 tailnt0; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables $tb > $O/tail_${v}_${tb}_${i}_$T.json 2>/dev/null || exit 1
done; done; done
for f in $O/tail_*_$T.json; do pj $f; done
for i in 1 2; do for v in tailnt1 tailnt0; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 120 python tools/prof_env_step.py 3000 > $O/env_${v}_${i}_$T.json 2>/dev/null || exit 1
  echo "env $v $i $(cat $O/env_${v}_${i}_$T.json | cut -c1-120)"
done; done

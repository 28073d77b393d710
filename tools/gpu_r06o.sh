# round 6: how much of the headline launch the rules waves' dependent gathers (deck top, token table) cost:
# lib_gath0 (-DSPL_ABL=49152: both gathers replaced by constants; wrong results by design) against lib_nt1
# (the shipped build), arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06o}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['value'])" $1; }
for i in 1 2 3; do for v in nt1 gath0; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 > $O/head_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/head_*_$T.json; do pj $f; done

# round 6: confirmation of the headline's store policy, shipped non-temporal (cpn) against sc0 nt sc1 (cp19),
# four alternations on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06v}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], '%.4g' % d['value'])" $1; }
for i in 1 2 3 4; do for v in cpn cp19; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 > $O/head_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/head_*_$T.json; do pj $f; done

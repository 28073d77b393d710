# round 6: per-step rollout-store rows and masks non-temporal (lib_nt1, as shipped) vs plain (lib_nt0,
# -DSPL_ROLL_NT=0), alternating on one box: the headline (2p x 65 536, quad kernel) and C4's share (4p x 32 768)
set -o pipefail
O=gpurun_out
T=${TAG:-r06m}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['value'])" $1; }
for i in 1 2 3; do for v in nt1 nt0; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 > $O/head_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for i in 1 2; do for v in nt1 nt0; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 --players 4 --tables 32768 > $O/c4_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/head_*_$T.json $O/c4_*_$T.json; do pj $f; done

# round 6: timing ablation — the rollout store's small outputs (reward, terminated, flags, winner) not stored
# (nosmall, -DSPL_ABL=256; wrong outputs by design) against the product build (base1), headline and C4's share,
# arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06aj}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], '%.4g' % d['value'])" $1; }
for i in 1 2 3; do for v in base1 nosmall; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 > $O/ns_head_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for i in 1 2; do for v in base1 nosmall; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 --players 4 --tables 32768 > $O/ns_c4_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/ns_*_$T.json; do pj $f; done

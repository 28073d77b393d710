# round 6: the rollout store's NT output stream under other cache policies (SPL_ROLL_CPOL: buffer stores with
# sc0 = 1, nt = 2, sc1 = 16), arms alternating on one box: the headline (2p x 65 536, quad kernel) and C4's share
# (4p x 32 768); cpn = the shipped compiler non-temporal store, cp2 the same policy as a buffer store
set -o pipefail
O=gpurun_out
T=${TAG:-r06u}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], '%.4g' % d['value'])" $1; }
for i in 1 2; do for v in cpn cp2 cp18 cp19 cp16 cp17 cp3; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 > $O/head_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for v in cpn cp18 cp19; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 --players 4 --tables 32768 > $O/c4_${v}_1_$T.json 2>/dev/null || exit 1
done
for f in $O/head_*_$T.json $O/c4_*_$T.json; do pj $f; done

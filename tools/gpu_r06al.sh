# round 6: at 65 536 tables, the three-wave step shape with its sc0 nt sc1 row stores (--step-tail 1) against the
# auto choice there (two waves, plain rows), graph-replay HIP events per step, arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06al}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $1; }
for i in 1 2 3; do for m in auto 1; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --step-tail $m > $O/s65_${m}_${i}_$T.json 2>/dev/null || exit 1
done; done
for tb in 49152; do for i in 1 2; do for m in auto 1; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables $tb --step-tail $m > $O/s49_${m}_${i}_$T.json 2>/dev/null || exit 1
done; done; done
for f in $O/s65_*_$T.json $O/s49_*_$T.json; do pj $f; done

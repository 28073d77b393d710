# round 6: the two-wave step's rows (65 536 tables) under the temporal cache policies (buffer stores sc0 = wsc1,
# sc1 = wsc16, sc0 sc1 = wsc17; without nt) against plain stores (wsref = the product), graph-replay HIP events per
# step, arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06an}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $1; }
for i in 1 2 3; do for v in wsref wsc1 wsc16 wsc17; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 > $O/wsc_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/wsc_*_$T.json; do pj $f; done

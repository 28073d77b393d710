# round 6: k_step_ws (65 536 tables) with half of each row block stored through the NT output stream (sc0 nt sc1)
# and half plain (split1: first half NT, split2: second half NT) against all plain (wsdef), graph-replay HIP
# events per step, arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06z}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $1; }
for i in 1 2 3; do for v in wsdef split1 split2; do
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 > $O/split_${v}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/split_*_$T.json; do pj $f; done

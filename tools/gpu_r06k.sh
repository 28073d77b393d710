# round 6: spl_step's third shape (k_step_wso: the output wave evaluates the mask between its row stores) against
# the two-wave and three-wave shapes, alternating on one box, after the GPU suite
set -o pipefail
O=gpurun_out
T=${TAG:-r06k}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.out 2>&1; rc=$?; tail -3 $O/pytest_gpu_$T.out; [ $rc -eq 0 ] || exit 1
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], r.get('eager_launch_us'))" $1; }
for i in 1 2 3; do for m in 0 2; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --step-tail $m > $O/shape65k_${m}_${i}_$T.json 2>/dev/null || exit 1
done; done
for tb in 32768 16384; do for i in 1 2; do for m in 1 2 0; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables $tb --step-tail $m > $O/shape${tb}_${m}_${i}_$T.json 2>/dev/null || exit 1
done; done; done
for f in $O/shape*_$T.json; do pj $f; done

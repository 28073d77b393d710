# round 6: sc1 row stores in both step shapes — GPU suite, smoke(), then the driver's command
set -o pipefail
O=gpurun_out
T=${TAG:-r06as}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.out 2>&1; rc=$?; tail -2 $O/pytest_gpu_$T.out; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1 || exit 1
tail -1 $O/smoke_$T.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$T.json 2> $O/bench_driver_$T.err || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); o=d['other_mode']; print('%.4g' % d['value'], d['roofline']['frac'], o['ms_per_step'], o['roofline']['kernel'], o['roofline']['kernel_us']['median'], o['roofline']['frac'], '%.4g' % d['config4_share']['value'], '%.4g' % d['config5_selfplay']['value'])" $O/bench_driver_$T.json
for tb in 32768 49152; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables $tb > $O/sq_${tb}_$T.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['config']['tables_per_gpu'], r['kernel'], r['kernel_us']['median'], d['ms_per_step'])" $O/sq_${tb}_$T.json
done

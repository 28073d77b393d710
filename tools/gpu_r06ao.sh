# round 6: the two-wave step's sc1 row stores in the product — GPU suite, smoke(), then the driver's command
set -o pipefail
O=gpurun_out
T=${TAG:-r06ao}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.out 2>&1; rc=$?; tail -2 $O/pytest_gpu_$T.out; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1 || exit 1
tail -1 $O/smoke_$T.txt
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$T.json 2> $O/bench_driver_$T.err || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); o=d['other_mode']; print('%.4g' % d['value'], d['roofline']['frac'], o['ms_per_step'], o['roofline']['kernel'], o['roofline']['kernel_us']['median'], o['roofline']['frac'], '%.4g' % d['config4_share']['value'], '%.4g' % d['config5_selfplay']['value'])" $O/bench_driver_$T.json

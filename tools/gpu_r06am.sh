# round 6: GPU suite, smoke() and a 49 152-table step check (auto must pick the three-wave shape) on the last tree
set -o pipefail
O=gpurun_out
T=${TAG:-r06am}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.out 2>&1; rc=$?; tail -2 $O/pytest_gpu_$T.out; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1 || exit 1
tail -1 $O/smoke_$T.txt
timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables 49152 > $O/s49_auto_$T.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['roofline']['kernel'], d['roofline']['kernel_us']['median'])" $O/s49_auto_$T.json

# round 6: the final-tree session after the store policies and the quad kernel's lead-0 default — GPU suite,
# smoke(), the driver's command, the same under rocprofv3 (kernel stats + timed-region trace), then the quad
# lead confirmed on this box (default = 0 against --partner-lead 4, three alternations)
set -o pipefail
O=gpurun_out
T=${TAG:-r06ae}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.out 2>&1; rc=$?; tail -3 $O/pytest_gpu_$T.out; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$T.json 2> $O/bench_driver_$T.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver_$T -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver_$T.out 2> $O/prof_driver_$T.err || exit 1
cp $O/prof_driver_$T/run_kernel_stats.csv $O/kernel_stats_driver_$T.csv 2>/dev/null || find $O/prof_driver_$T -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_driver_$T.csv \;
python3 tools/trace_timed.py $(find $O/prof_driver_$T -name '*kernel_trace.csv' | head -1) $O/prof_driver_$T.err \
    --source "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ($T)" --out $O/kernel_trace_timed_$T.json > /dev/null || exit 1
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], r['kernel'], r['kernel_us']['median'], '%.4g' % d['value'], d.get('partner_handoffs'))" $1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 > $O/leadc_dflt_${i}_$T.json 2>/dev/null || exit 1
  timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 --partner-lead 4 > $O/leadc_4_${i}_$T.json 2>/dev/null || exit 1
done
for f in $O/leadc_*_$T.json; do pj $f; done

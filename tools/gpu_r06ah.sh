# round 6: the final-tree session (store policies, partner lead 0 in both kernels) — GPU suite, smoke(), the
# driver's command, the same under rocprofv3 (kernel stats + timed-region trace)
set -o pipefail
O=gpurun_out
T=${TAG:-r06ah}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.out 2>&1; rc=$?; tail -3 $O/pytest_gpu_$T.out; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.txt 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$T.json 2> $O/bench_driver_$T.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver_$T -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver_$T.out 2> $O/prof_driver_$T.err || exit 1
cp $O/prof_driver_$T/run_kernel_stats.csv $O/kernel_stats_driver_$T.csv 2>/dev/null || find $O/prof_driver_$T -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_driver_$T.csv \;
python3 tools/trace_timed.py $(find $O/prof_driver_$T -name '*kernel_trace.csv' | head -1) $O/prof_driver_$T.err \
    --source "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ($T)" --out $O/kernel_trace_timed_$T.json > /dev/null || exit 1

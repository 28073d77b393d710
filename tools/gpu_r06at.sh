# round 6: rocprofv3 kernel stats + timed-region trace of the driver's command on the last tree
set -o pipefail
O=gpurun_out
T=${TAG:-r06at}
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver_$T -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver_$T.out 2> $O/prof_driver_$T.err || exit 1
cp $O/prof_driver_$T/run_kernel_stats.csv $O/kernel_stats_driver_$T.csv 2>/dev/null || find $O/prof_driver_$T -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_driver_$T.csv \;
python3 tools/trace_timed.py $(find $O/prof_driver_$T -name '*kernel_trace.csv' | head -1) $O/prof_driver_$T.err \
    --source "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ($T)" --out $O/kernel_trace_timed_$T.json > /dev/null || exit 1
python3 -c "import json; t=json.load(open('$O/kernel_trace_timed_$T.json')); [print(k, v['kernel'], v['timed_median_us']) for k, v in t['regions'].items()]"

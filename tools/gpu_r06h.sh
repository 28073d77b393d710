# round 6: the step kernel's shape by grid size, the XCD-aware narrow tails (tools/gpu_r06g.sh's follow-up)
set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_r06h.out 2>&1; rc=$?; tail -3 $O/pytest_gpu_r06h.out; [ $rc -eq 0 ] || exit 1
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r['kernel'], r['kernel_us']['median'], r.get('eager_launch_us'))" $1; }
for i in 1 2; do for m in 0 1; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables 32768 --step-tail $m > $O/stepab32k_tail${m}_${i}_r06h.json 2>/dev/null || exit 1
done; done
for f in $O/stepab32k_*_r06h.json; do pj $f; done
timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 > $O/step65k_auto_r06h.json 2>/dev/null && pj $O/step65k_auto_r06h.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_sptrace_r06h -o run -- python3 tools/bench_selfplay.py --opponent pool > $O/sptrace_r06h.log 2>&1 || exit 1
python3 tools/dual_step_timeline.py $(find $O/prof_sptrace_r06h -name '*kernel_trace.csv' | head -1) > $O/selfplay_trace_r06h.txt && tail -12 $O/selfplay_trace_r06h.txt

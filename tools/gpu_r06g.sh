set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_r06g.out 2>&1; rc=$?; tail -3 $O/pytest_gpu_r06g.out; [ $rc -eq 0 ] || exit 1
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['ms_per_step'], r['kernel_us']['median'], r.get('eager_launch_us'))" $1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 > $O/stepab_tail_${i}_r06g.json 2>/dev/null || exit 1
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_tail0.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 > $O/stepab_tail0_${i}_r06g.json 2>/dev/null || exit 1
done
for f in $O/stepab_*_r06g.json; do pj $f; done
for i in 1 2; do
  timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables 16384 > $O/stepab16k_tail_${i}_r06g.json 2>/dev/null || exit 1
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_tail0.so timeout -k 10 300 python bench.py --mode step --only --no-cpu-baseline --sp-tables 0 --tables 16384 > $O/stepab16k_tail0_${i}_r06g.json 2>/dev/null || exit 1
done
for f in $O/stepab16k_*_r06g.json; do pj $f; done
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_selfplay.py --opponent pool > $O/spab_new_${i}_r06g.json 2>/dev/null || exit 1
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_narrow_old.so timeout -k 10 300 python tools/bench_selfplay.py --opponent pool > $O/spab_old_${i}_r06g.json 2>/dev/null || exit 1
done
for f in $O/spab_*_r06g.json; do echo "$f $(tail -1 $f | cut -c1-220)"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_sptrace_r06g -o run -- python3 tools/bench_selfplay.py --opponent pool > $O/sptrace_r06g.log 2>&1 || exit 1
python3 tools/dual_step_timeline.py $(find $O/prof_sptrace_r06g -name '*kernel_trace.csv' | head -1) > $O/selfplay_trace_r06g.txt && tail -12 $O/selfplay_trace_r06g.txt

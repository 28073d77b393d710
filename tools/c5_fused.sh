set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_policy.py -x -q > $O/pytest_policy_p2.log 2>&1 || { tail -30 $O/pytest_policy_p2.log; exit 1; }
tail -1 $O/pytest_policy_p2.log
timeout -k 10 300 python tools/bench_selfplay.py > $O/sp_fused.json 2> $O/sp_fused.err && cat $O/sp_fused.json && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_spf -o run -- python3 tools/bench_selfplay.py --iters 32 > $O/spf_prof.json 2> $O/spf_prof.err
echo rc $?

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python tools/bench_selfplay.py > $O/sp_fp32.json 2> $O/sp_fp32.err && \
timeout -k 10 300 python tools/bench_selfplay.py --bf16 > $O/sp_bf16.json 2> $O/sp_bf16.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_sp -o run -- python3 tools/bench_selfplay.py --iters 32 > $O/sp_prof.json 2> $O/sp_prof.err
echo rc $?

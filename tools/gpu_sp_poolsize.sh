set -o pipefail
for ps in 0 1 3 6 12; do
  timeout -k 10 200 python3 tools/bench_selfplay.py --opponent pool --pool-size $ps > gpurun_out/sps_$ps.json 2> gpurun_out/sps_$ps.err || { tail -5 gpurun_out/sps_$ps.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sps_$ps.json'));print('pool_size $ps', d['value'], d['ms_per_dual_step'])"
done

# round 6: the six-wave dealer's partner hand-off lead under the sc0 nt sc1 row stores (C4's per-GPU share, 4p x
# 32 768): 4 (default), 0 (off), 8; arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06ag}
pj() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1].split('/')[-1], r['kernel'], r['kernel_us']['median'], '%.4g' % d['value'], d.get('partner_handoffs'))" $1; }
for i in 1 2 3; do for l in 4 0 8; do
  timeout -k 10 300 python bench.py --only --no-cpu-baseline --sp-tables 0 --players 4 --tables 32768 --partner-lead $l > $O/c4lead_${l}_${i}_$T.json 2>/dev/null || exit 1
done; done
for f in $O/c4lead_*_$T.json; do pj $f; done

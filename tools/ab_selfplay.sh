#!/bin/bash
# A/B of library variants (splendor-gym_amd/ablate/libp32v_<name>.so, tools/ab_policy32.sh BUILD=1) on
# the config-5 self-play loop: tools/bench_selfplay.py under rocprofv3 kernel-trace stats, alternating,
# `rounds` passes; prints ms per dual step and the k_act32 / narrow-tail kernel averages.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_sp
mkdir -p $O
for r in $(seq 1 ${1:-2}); do
  for name in ${NAMES:?names}; do
    SPLENDOR_AMD_LIB=$PWD/splendor-gym_amd/ablate/libp32v_$name.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d $O/${name}_$r -o run -- python3 tools/bench_selfplay.py > $O/${name}_$r.json 2> $O/${name}_$r.err \
      || { echo "fail $name"; tail -5 $O/${name}_$r.err; exit 1; }
    python3 - $O/${name}_$r $name $r <<'PY'
import csv, json, sys
d, name, r = sys.argv[1:]
rows = {x["Name"].split("(")[0].replace("void ", ""): float(x["AverageNs"]) / 1e3 for x in csv.DictReader(open(d + "/run_kernel_stats.csv"))}
sp = json.loads([l for l in open(d + ".json") if l.startswith("{")][-1])
print(name, "pass", r, "dual_ms", sp["ms_per_dual_step"], {k: round(v, 1) for k, v in rows.items() if "act32" in k})
PY
  done
done

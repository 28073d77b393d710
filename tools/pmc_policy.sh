#!/bin/bash
# PMC passes over the fused fp32 actor (k_act32<true,true> sample + critic, k_act32<false,false> greedy;
# tools/bench_policy.py --fused-only at 65 536 tables), one rocprofv3 --pmc pass per counter group
# (--kernel-trace only), then a per-kernel summary: MFMA busy fraction, wave-cycle split, LDS
# instructions and bank conflicts, L2 (TCC) requests / hits and HBM bytes.
#   tools/pmc_policy.sh TAG     (POL_ARGS=--config5-only: config 5's agent call alone)
set -o pipefail
TAG=${1:-pol}
export TMPDIR=/tmp
O=gpurun_out/pmc_pol_$TAG; mkdir -p $O
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SALU" \
           "FETCH_SIZE" \
           "TCC_HIT_sum TCC_MISS_sum TCC_READ_sum" \
           "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "k_act32" --output-format csv \
      -d $O/p$i -o run -- python3 tools/bench_policy.py --fused-only --iters 5 $POL_ARGS > $O/p$i.log 2>&1 \
      || { echo "pass $i ($grp) failed"; tail -5 $O/p$i.log; }
done
python3 - "$O" <<'PY'
import csv, glob, collections, json, sys
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{O}/p*/run_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        acc[k][c].append(v)
out = {}
for k, cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    rec = {c: round(v) for c, v in m.items()}
    g = m.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in m:  # GRBM_GUI_ACTIVE sums the 8 XCDs; 256 CUs x 4 SIMDs
        rec["mfma_busy_frac_of_simd_cycles"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), 4)
    if m.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in m:
                rec[c + "_frac"] = round(m[c] / m["SQ_WAVE_CYCLES"], 4)
    if m.get("SQ_INSTS_LDS"):
        rec["lds_bank_conflict_per_lds_inst"] = round(m.get("SQ_LDS_BANK_CONFLICT", 0) / m["SQ_INSTS_LDS"], 3)
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
        rec["tcc_hit_rate"] = round(m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
    out[k] = rec
print(json.dumps(out, indent=1))
json.dump(out, open(f"{O}/summary.json", "w"), indent=1)
PY

#!/bin/bash
# PMC passes over one bench workload (one rocprofv3 --pmc pass per counter group, each with
# --kernel-trace only, as gpurun requires), then the summary into profiles/pmc_summary.json.
#   tools/pmc.sh TAG PLAYERS TABLES VARIANT [GROUPS]
# VARIANT: store (rollout, per-step blocks of a [128, T, ...] store; the headline), inplace, step.
# GROUPS: "traffic" (FETCH_SIZE; WRITE_SIZE only) or "all" (default: traffic + SQ/TCC groups).
set -o pipefail
TAG=${1:?tag}
P=${2:-2}
T=${3:-65536}
VARIANT=${4:-store}
WHICH=${5:-all}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="--no-cpu-baseline --only --players $P --tables $T"
if [ "$VARIANT" = "step" ]; then
  ARGS="$COMMON --mode step --graph-steps 0 --steps 64 --warmup 64"
else
  ARGS="$COMMON --mode rollout --outputs $VARIANT --steps 128 --warmup 128"
fi
TRAFFIC="FETCH_SIZE;WRITE_SIZE"
MORE="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;\
SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS;\
GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM;\
TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM"
if [ "$WHICH" = "traffic" ]; then G="$TRAFFIC"; else G="$TRAFFIC;$MORE"; fi
IFS=';' read -ra GROUPS_LIST <<< "$G"
i=0
for grp in "${GROUPS_LIST[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc ${grp} --kernel-include-regex "k_step|k_rollout|k_refill" \
      --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
# the summary accumulates workloads: start from the committed one (copy it back into profiles/)
[ -f gpurun_out/pmc_summary.json ] || cp profiles/pmc_summary.json gpurun_out/pmc_summary.json
python3 tools/pmc_summary.py $OUT gpurun_out/pmc_summary.json --players $P --tables $T --rollout-steps 128 \
    > $OUT/summary.txt || { echo "pmc summary failed"; exit 1; }
cat $OUT/summary.txt

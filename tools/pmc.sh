#!/bin/bash
# PMC passes for the step, rollout and refill kernels (one rocprofv3 --pmc pass per counter group, each
# with --kernel-trace only as gpurun requires).  The bench runs one variant (--only): VARIANT=store
# (headline: rollout with per-step blocks of a [64, T, ...] store), inplace, or step.
set -o pipefail
TAG=${1:-r02}
VARIANT=${VARIANT:-store}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$VARIANT" = "step" ]; then
  BENCH="python3 bench.py --no-cpu-baseline --only --mode step --graph-steps 0 --steps 64 --warmup 64"
else
  BENCH="python3 bench.py --no-cpu-baseline --only --mode rollout --outputs $VARIANT --steps 128 --warmup 128"
fi
GROUPS_DEFAULT="FETCH_SIZE;WRITE_SIZE;\
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU;\
SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS;\
GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_VMEM;\
TCC_EA0_RDREQ TCC_EA0_WRREQ TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM"
IFS=';' read -ra GROUPS_LIST <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
i=0
for grp in "${GROUPS_LIST[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${grp} --kernel-include-regex "k_step|k_rollout|k_refill" \
      --output-format csv -d $OUT/p$i -o run -- $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "pmc done"

#!/bin/bash
# Ablation timing of k_act (spl_policy.hip, -DSPL_ACT_ABL=<bits>): build variants here
# (BUILD=1), or time each under rocprofv3 kernel-trace stats on the GPU box.
set -o pipefail
D=splendor-gym_amd/ablate
C=splendor-gym_amd/csrc
VARIANTS="full:0 no_mfma:1 no_epi:2 no_xload:4 no_ring:8 only_ring:7 only_mfma:14"
if [ "${BUILD:-0}" = "1" ]; then
  mkdir -p $D
  for v in $VARIANTS; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSPL_ACT_ABL=${v#*:} -shared \
      -o $D/libpol_${v%%:*}.so $C/spl_engine.hip $C/spl_policy.hip $C/spl_dual.hip || exit 1
  done
  exit 0
fi
O=gpurun_out/abl_pol
mkdir -p $O
export TMPDIR=/tmp
for v in $VARIANTS; do
  n=${v%%:*}
  SPLENDOR_AMD_LIB=$PWD/$D/libpol_$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/$n -o run -- python3 tools/bench_policy.py --fused-only --iters 20 > $O/$n.json 2> $O/$n.err || { echo "fail $n"; exit 1; }
  echo "$n $(grep -h 'k_act' $O/$n/run_kernel_stats.csv | tr '\n' ' ')"
done

#!/bin/bash
# Ablation timing of k_act32 (spl_policy32.hip, -DSPL_POL_ABL=<bits>; wrong results by design except
# "full"): build the variants here (BUILD=1; the other sources compiled once), or time each under
# rocprofv3 kernel-trace stats on the GPU box.  Bits: 1 tanh = identity, 2 one weight chunk (no ring
# streaming, no per-chunk barrier), 4 A planes read once per tile, 8 no MFMA (a VALU stand-in).
set -o pipefail
D=splendor-gym_amd/ablate
C=splendor-gym_amd/csrc
VARIANTS=${VARIANTS:-"full:0 notanh:1 noring:2 noafrd:4 noring_notanh:3 mfma_only:7"}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950"
if [ "${BUILD:-0}" = "1" ]; then
  mkdir -p $D/obj
  for s in spl_engine spl_policy spl_dual; do
    if [ $C/obj/$s.o -nt $C/$s.hip ]; then cp $C/obj/$s.o $D/obj/$s.o; fi  # the product build's objects (csrc/Makefile)
    [ $D/obj/$s.o -nt $C/$s.hip ] || /opt/rocm/bin/hipcc $F -c -o $D/obj/$s.o $C/$s.hip || exit 1
  done
  for v in $VARIANTS; do
    /opt/rocm/bin/hipcc $F -DSPL_POL_ABL=${v#*:} -c -o $D/obj/p32_${v%%:*}.o $C/spl_policy32.hip || exit 1
    /opt/rocm/bin/hipcc $F -shared -o $D/libp32_${v%%:*}.so $D/obj/spl_engine.o $D/obj/spl_policy.o \
      $D/obj/spl_dual.o $D/obj/p32_${v%%:*}.o || exit 1
  done
  exit 0
fi
O=gpurun_out/abl_p32
mkdir -p $O
export TMPDIR=/tmp
for v in $VARIANTS; do
  n=${v%%:*}
  SPLENDOR_AMD_LIB=$PWD/$D/libp32_$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/$n -o run -- python3 tools/bench_policy.py --fused-only --iters 20 > $O/$n.json 2> $O/$n.err || { echo "fail $n"; exit 1; }
  echo "$n $(grep -h 'k_act32' $O/$n/run_kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done

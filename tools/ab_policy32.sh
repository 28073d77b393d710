#!/bin/bash
# A/B of k_act32 build variants (spl_policy32.hip), alternating on one box:
#   BUILD=1 tools/ab_policy32.sh            # here: the variants below into splendor-gym_amd/ablate/
#   tools/ab_policy32.sh [rounds]           # GPU box: tools/bench_policy.py per variant, `rounds` passes
# Variants: name:REV:FLAGS (REV = a git revision of the sources, or "wt" for the working tree).
set -o pipefail
D=splendor-gym_amd/ablate
VARIANTS=${VARIANTS:-"head:HEAD: wt:wt:"}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950"
if [ "${BUILD:-0}" = "1" ]; then
  mkdir -p $D/obj
  for s in spl_engine spl_policy spl_dual; do
    [ $D/obj/$s.o -nt splendor-gym_amd/csrc/$s.hip ] || /opt/rocm/bin/hipcc $F -c -o $D/obj/$s.o splendor-gym_amd/csrc/$s.hip || exit 1
  done
  for v in $VARIANTS; do
    IFS=: read -r name rev flags <<< "$v"
    src=splendor-gym_amd/csrc/spl_policy32.hip
    if [ "$rev" != "wt" ]; then
      t=$(mktemp -d); git archive "$rev" splendor-gym_amd/csrc include | tar -x -C $t; src=$t/splendor-gym_amd/csrc/spl_policy32.hip
    fi
    /opt/rocm/bin/hipcc $F ${flags//,/ } -c -o $D/obj/p32v_$name.o $src || exit 1
    /opt/rocm/bin/hipcc $F -shared -o $D/libp32v_$name.so $D/obj/spl_engine.o $D/obj/spl_policy.o $D/obj/spl_dual.o \
      $D/obj/p32v_$name.o || exit 1
  done
  exit 0
fi
O=gpurun_out/ab_p32
mkdir -p $O
for r in $(seq 1 ${1:-2}); do
  for v in $VARIANTS; do
    name=${v%%:*}
    SPLENDOR_AMD_LIB=$PWD/$D/libp32v_$name.so timeout -k 10 120 python3 tools/bench_policy.py --fused-only --iters 30 \
      > $O/${name}_$r.json 2> $O/${name}_$r.err || { echo "fail $name"; tail -5 $O/${name}_$r.err; exit 1; }
    echo "$name pass $r $(python3 -c "import json,sys; d=json.load(open('$O/${name}_$r.json')); print(d['fused_fp32_sample_us'], d['fused_fp32_greedy_us'])")"
  done
done

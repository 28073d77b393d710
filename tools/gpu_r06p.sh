# round 6: config 5's agent call (k_act32<true,true>: trained weights, compact rows, sample + critic, 65 536
# tables) with its non-MFMA work compiled out (mfma_only: -DSPL_POL_ABL=103 = tanh identity | one weight chunk |
# A planes once per tile | no per-table epilogue | no observation loads) and with its MFMAs replaced by one VALU
# op each (no_mfma: 8), against the shipped kernel (full), arms alternating, rocprofv3 kernel-trace stats
set -o pipefail
D=splendor-gym_amd/ablate
O=gpurun_out/abl_p32_r06p
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do for n in full mfma_only no_mfma; do
  SPLENDOR_AMD_LIB=$PWD/$D/libp32_$n.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/${n}_$i -o run -- python3 tools/bench_policy.py --config5-only --fused-only --iters 20 > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "fail $n"; exit 1; }
  echo "$n $i $(grep -h 'k_act32' $O/${n}_$i/run_kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
done; done

# round 6: what config 5's agent call (k_act32<true,true>, trained weights, compact rows, sample + critic, 65 536
# tables) spends outside its MFMAs: the kernel with every MFMA removed (nomfma: -DSPL_POL_ABL=512, an empty asm
# keeps the operands live) and that with one more part removed (notanh 1, noring 2, aonce 4, noepi 32), the
# skeleton without any of them (skel 615), the MFMA-only build (103) and the shipped kernel (full); arms
# alternating, rocprofv3 kernel-trace stats (25 calls each)
set -o pipefail
D=splendor-gym_amd/ablate
O=gpurun_out/abl_p32_r06q
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do for n in full mfma_only nomfma nomfma_notanh nomfma_noring nomfma_aonce nomfma_noepi skel; do
  SPLENDOR_AMD_LIB=$PWD/$D/libp32_$n.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/${n}_$i -o run -- python3 tools/bench_policy.py --config5-only --fused-only --iters 20 > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "fail $n"; exit 1; }
done; done
python3 - <<'PY'
import csv, glob
for f in sorted(glob.glob('gpurun_out/abl_p32_r06q/*/run_kernel_stats.csv')):
    for r in csv.DictReader(open(f)):
        if 'k_act32' in r['Name']:
            print(f.split('/')[-2], r['Calls'], 'avg %.1f min %.1f max %.1f us' % (float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3, float(r['MaxNs']) / 1e3))
PY

# round 6: the dual step's opponent step (both int32 and compact rows, two-wave shape at 65 536 tables) with its
# int32 rows as sc0 nt sc1 stores (bothnt) against plain (the product build), config 5 per GPU
# (tools/bench_selfplay.py --opponent pool), arms alternating on one box
set -o pipefail
O=gpurun_out
T=${TAG:-r06aa}
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_selfplay.py --opponent pool > $O/sp_base_${i}_$T.json 2>/dev/null || exit 1
  SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_bothnt.so timeout -k 10 300 python tools/bench_selfplay.py --opponent pool > $O/sp_bothnt_${i}_$T.json 2>/dev/null || exit 1
done
for f in $O/sp_*_$T.json; do echo "$f $(tail -1 $f | cut -c1-220)"; done

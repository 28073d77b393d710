# Per-kernel register / LDS / scratch usage of the gfx950 build (hipcc -Rpass-analysis=kernel-resource-usage)
set -o pipefail
D=$(cd "$(dirname "$0")/.." && pwd)/splendor-gym_amd/csrc
for f in spl_engine.hip spl_policy.hip spl_policy32.hip spl_dual.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -c -Rpass-analysis=kernel-resource-usage \
      -o /dev/null "$D/$f" 2>&1
done | python3 -c '
import re, sys, subprocess
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark:\s+(.*?):\s+(.*?) \[-Rpass", line)
    if not m: continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}; rows.append(cur)
    elif cur is not None:
        cur[k] = v
cols = ["VGPRs", "AGPRs", "TotalSGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
print("kernel | " + " | ".join(c.split(" [")[0] for c in cols))
for r in rows:
    if "(" in r["name"] and "k_" in r["name"]:
        print(r["name"].split("(")[0] + " | " + " | ".join(r.get(c, "-") for c in cols))
'

# k_seg small-packet grid cut (kSegSmallMean = 400 B) re-check (measurement only):
# U{40..600} (mean 320), U{40..1000} (mean 520), U{64..1500} (mean 782) with the
# small grid forced off (YU_SEG_SMALL_BLOCKS=0) or on at every mean (=3 via a
# tiny batch mean is not possible from the host, so 0 vs default only).
set -o pipefail
mkdir -p gpurun_out
args=()
for rep in 1 2 3; do for cfg in 9 10; do args+=("$cfg" "$cfg YU_SEG_SMALL_BLOCKS=0" "$cfg YU_BLOCKS_PER_CU=3"); done; done
bash tools/ab.sh "${args[@]}" > gpurun_out/small_mean.log 2>&1 || { tail gpurun_out/small_mean.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/small_mean.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round (\d):\s+([\d.]+) us',l)
    if m and cur and m.group(1) != '0': d[cur].append(float(m.group(2)))
for k,v in sorted(d.items()): print(f"{k:50s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

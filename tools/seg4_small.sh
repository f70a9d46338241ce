# 4 KiB vs 8 KiB k_seg tiles on small ragged batches (measurement only).
set -o pipefail
mkdir -p gpurun_out
args=()
for rep in 1 2 3; do for cfg in 6 8 16; do args+=("$cfg" "$cfg YU_RAGGED=seg4"); done; done
bash tools/ab.sh "${args[@]}" > gpurun_out/seg4_small.log 2>&1 || { tail gpurun_out/seg4_small.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/seg4_small.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round (\d):\s+([\d.]+) us.*\s(\S+)$',l)
    if m and cur and m.group(1) != '0': d[cur+' '+m.group(3)].append(float(m.group(2)))
for k,v in sorted(d.items()): print(f"{k:50s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

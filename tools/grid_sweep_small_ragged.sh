# Small ragged k_seg launches (measurement only): does the size of the launched
# grid matter when only YU_SEG_SMALL_BLOCKS (3) blocks per CU work?
set -o pipefail
mkdir -p gpurun_out
args=()
for rep in 1 2 3; do
  for cfg in 6 8 16; do
    for b in 0 3 6 12; do
      if [ "$b" = 0 ]; then args+=("$cfg"); else args+=("$cfg YU_BLOCKS_PER_CU=$b"); fi
    done
  done
done
bash tools/ab.sh "${args[@]}" > gpurun_out/grid_smallrag.log 2>&1 || { tail gpurun_out/grid_smallrag.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/grid_smallrag.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round (\d):\s+([\d.]+) us',l)
    if m and cur and m.group(1) != '0': d[cur].append(float(m.group(2)))
for k,v in sorted(d.items()): print(f"{k:40s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

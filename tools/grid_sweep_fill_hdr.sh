# Grid sweeps (measurement only): in-place writers and the IPv4 header kernel.
set -o pipefail
mkdir -p gpurun_out
args=()
for rep in 1 2; do
  for b in 0 8 16 32; do
    e=""; [ "$b" = 0 ] || e="YU_BLOCKS_PER_CU=$b"
    args+=("3 KB_FILL=1 $e" "12 $e" "13 $e")
  done
  for b in 0 4 8 12; do
    e=""; [ "$b" = 0 ] || e="YU_BLOCKS_PER_CU=$b"
    args+=("14 KB_FILL=1 $e")
  done
  for b in 0 2 4 6; do
    e=""; [ "$b" = 0 ] || e="YU_SEG_SMALL_BLOCKS=$b"
    args+=("8 KB_FILL=1 KB_ALIGN4=1 $e")
  done
done
bash tools/ab.sh "${args[@]}" > gpurun_out/grid_fill.log 2>&1 || { tail gpurun_out/grid_fill.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/grid_fill.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round \d:\s+([\d.]+) us',l)
    if m and cur: d[cur].append(float(m.group(1)))
for k,v in sorted(d.items()): print(f"{k:50s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

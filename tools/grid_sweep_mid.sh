# Grid sweep for dense mid-size uniform packets on k_seg (measurement only):
# kbench 14 (1M UDP datagrams of KB_LEN bytes) at several blocks per CU.
set -o pipefail
mkdir -p gpurun_out
args=()
for rep in 1 2; do
for len in 136 160 200 256 320 384 420; do
  for b in 0 6 8 10; do
    if [ "$b" = 0 ]; then args+=("14 KB_LEN=$len"); else args+=("14 KB_LEN=$len YU_BLOCKS_PER_CU=$b"); fi
  done
done
done
bash tools/ab.sh "${args[@]}" > gpurun_out/grid_mid.log 2>&1 || { tail gpurun_out/grid_mid.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/grid_mid.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round \d:\s+([\d.]+) us',l)
    if m and cur: d[cur].append(float(m.group(1)))
for k,v in d.items(): print(f"{k:45s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

# k_seg grid: exactly the resident blocks (YU_BLOCKS_PER_CU=3/4, no idle blocks that exit) vs the default over-sized grid
set -o pipefail
mkdir -p gpurun_out
B3=YU_BLOCKS_PER_CU=3
bash tools/ab.sh "16" "16 $B3" "16 YU_BLOCKS_PER_CU=4" "6" "6 $B3" "8" "8 $B3" "5" "5 $B3" "5 KB_MODE=8" "5 KB_MODE=8 $B3" \
  "4" "4 $B3" "7" "7 $B3" "15" "15 $B3" "16" "16 $B3" "6" "6 $B3" > gpurun_out/kbench_ab_seg_grid.log 2>&1 || { tail gpurun_out/kbench_ab_seg_grid.log; exit 1; }
python3 - <<'PY'
import re,statistics,collections
d=collections.defaultdict(list);cur=None
for l in open('gpurun_out/kbench_ab_seg_grid.log'):
    if l.startswith('=='): cur=l[3:].strip(); continue
    m=re.search(r'round \d+:\s+([\d.]+) us',l)
    if m and cur: d[cur].append(float(m.group(1)))
for k,v in d.items(): print(f"{k:45s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  n={len(v)}")
PY

# k_seg load policy on small vs large ragged batches: YU_NT=0 (plain) vs the default (nt)
set -o pipefail
mkdir -p gpurun_out
bash tools/ab.sh "16" "16 YU_NT=0" "6" "6 YU_NT=0" "8" "8 YU_NT=0" "5" "5 YU_NT=0" "5 KB_MODE=8" "5 KB_MODE=8 YU_NT=0" "4" "4 YU_NT=0" \
  "16" "16 YU_NT=0" "6" "6 YU_NT=0" > gpurun_out/kbench_ab_seg_nt.log 2>&1 || { tail gpurun_out/kbench_ab_seg_nt.log; exit 1; }
python3 - <<'PY'
import re,statistics,collections
d=collections.defaultdict(list);cur=None
for l in open('gpurun_out/kbench_ab_seg_nt.log'):
    if l.startswith('=='): cur=l[3:].strip(); continue
    m=re.search(r'round \d+:\s+([\d.]+) us',l)
    if m and cur: d[cur].append(float(m.group(1)))
for k,v in d.items(): print(f"{k:45s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  n={len(v)}")
PY

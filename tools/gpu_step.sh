# code object target: gfx950:xnack- (tools/varA) vs the default gfx950 (xnack any)
set -o pipefail
mkdir -p gpurun_out
A=LD_LIBRARY_PATH=tools/varA
bash tools/ab.sh "3" "3 $A" "16" "16 $A" "4" "4 $A" "5 KB_MODE=8" "5 KB_MODE=8 $A" "2" "2 $A" "15" "15 $A" \
  "3" "3 $A" "16" "16 $A" > gpurun_out/kbench_ab_xnack.log 2>&1 || { tail gpurun_out/kbench_ab_xnack.log; exit 1; }
python3 - <<'PY'
import re,statistics,collections
d=collections.defaultdict(list);cur=None;kern={}
for l in open('gpurun_out/kbench_ab_xnack.log'):
    if l.startswith('=='): cur=l[3:].strip(); continue
    m=re.search(r'round \d+:\s+([\d.]+) us.*\)\s+(\S+)$',l.strip())
    if m and cur: d[cur].append(float(m.group(1))); kern[cur]=m.group(2)
for k,v in d.items(): print(f"{k:45s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  n={len(v)} {kern[k]}")
PY

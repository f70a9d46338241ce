# k_small fill with plain loads by default (fill_nt) vs HEAD (tools/old): kbench and the bench's config 9 line
set -o pipefail
mkdir -p gpurun_out
O=LD_LIBRARY_PATH=tools/old
bash tools/ab.sh "3 KB_FILL=1 $O" "3 KB_FILL=1" "3 KB_FILL=1 $O" "3 KB_FILL=1" "3 KB_FILL=1 $O" "3 KB_FILL=1" "3" "3 $O" > gpurun_out/kbench_ab_fill_nt2.log 2>&1 || { tail gpurun_out/kbench_ab_fill_nt2.log; exit 1; }
python3 - <<'PY'
import re,statistics,collections
d=collections.defaultdict(list);cur=None
for l in open('gpurun_out/kbench_ab_fill_nt2.log'):
    if l.startswith('=='): cur=l[3:].strip(); continue
    m=re.search(r'round \d+:\s+([\d.]+) us',l)
    if m and cur: d[cur].append(float(m.group(1)))
for k,v in d.items(): print(f"{k:45s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  n={len(v)}")
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "fill" --timeout 120 --timeout-method thread 2>&1 | tail -1

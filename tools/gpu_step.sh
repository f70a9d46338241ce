# k_seg TX/RX/DG: one scan per tile over lane-contiguous sums (TS) vs HEAD (tools/old): parity, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ts.log 2>&1 || { tail -30 gpurun_out/gpu_tests_ts.log; exit 1; }
tail -1 gpurun_out/gpu_tests_ts.log
O=LD_LIBRARY_PATH=tools/old
bash tools/ab.sh "16 $O" "16" "15 $O" "15" "8 $O" "8" "5 KB_MODE=8 $O" "5 KB_MODE=8" "14 KB_LEN=160 $O" "14 KB_LEN=160" "7 $O" "7" "6 $O" "6" \
  "16 $O" "16" "15 $O" "15" "8 $O" "8" "5 KB_MODE=8 $O" "5 KB_MODE=8" "7 $O" "7" > gpurun_out/kbench_ab_ts.log 2>&1 || { tail gpurun_out/kbench_ab_ts.log; exit 1; }
python3 - <<'PY'
import re,statistics,collections
d=collections.defaultdict(list);cur=None
for l in open('gpurun_out/kbench_ab_ts.log'):
    if l.startswith('=='): cur=l[3:].strip(); continue
    m=re.search(r'round \d+:\s+([\d.]+) us',l)
    if m and cur: d[cur].append(float(m.group(1)))
for k,v in d.items(): print(f"{k:45s} median {statistics.median(v):8.1f}  min {min(v):8.1f}  n={len(v)}")
PY

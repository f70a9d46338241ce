# Uniform k_seg<4> grid change: parity + timing; ragged k_seg grid sweep (measurement only).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "uniform or seg or fuzz or size" > gpurun_out/grid_tests.log 2>&1 || { tail -30 gpurun_out/grid_tests.log; exit 1; }
tail -1 gpurun_out/grid_tests.log
args=()
for rep in 1 2; do
  for len in 136 256 384; do args+=("14 KB_LEN=$len"); done
  for cfg in 4 5 15; do
    for b in 0 3 6 12; do
      if [ "$b" = 0 ]; then args+=("$cfg"); else args+=("$cfg YU_BLOCKS_PER_CU=$b"); fi
    done
  done
done
bash tools/ab.sh "${args[@]}" > gpurun_out/grid_rag.log 2>&1 || { tail gpurun_out/grid_rag.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/grid_rag.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round \d:\s+([\d.]+) us',l)
    if m and cur: d[cur].append(float(m.group(1)))
for k,v in d.items(): print(f"{k:45s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

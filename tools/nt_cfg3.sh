# Config 3 load policy re-check with the runs kernel (measurement only).
set -o pipefail
mkdir -p gpurun_out
args=()
for rep in 1 2 3; do for nt in 2 1 0; do args+=("3 YU_NT=$nt"); done; done
bash tools/ab.sh "${args[@]}" > gpurun_out/nt_cfg3.log 2>&1 || { tail gpurun_out/nt_cfg3.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/nt_cfg3.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round (\d):\s+([\d.]+) us',l)
    if m and cur and m.group(1) != '0': d[cur].append(float(m.group(2)))
for k,v in sorted(d.items()): print(f"{k:50s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

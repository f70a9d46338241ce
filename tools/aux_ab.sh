# nt-load cache-policy bits A/B (measurement only): libraries built with -DYU_NT_AUX=<aux>.
set -o pipefail
mkdir -p gpurun_out
args=()
for rep in 1 2 3; do
  for cfg in 3 4 2; do
    args+=("$cfg" "$cfg LD_LIBRARY_PATH=tools/aux3" "$cfg LD_LIBRARY_PATH=tools/aux16" "$cfg LD_LIBRARY_PATH=tools/aux18" "$cfg LD_LIBRARY_PATH=tools/aux19")
  done
done
bash tools/ab.sh "${args[@]}" > gpurun_out/aux_ab.log 2>&1 || { tail gpurun_out/aux_ab.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/aux_ab.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round (\d):\s+([\d.]+) us',l)
    if m and cur and m.group(1) != '0': d[cur].append(float(m.group(2)))
for k,v in sorted(d.items()): print(f"{k:50s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

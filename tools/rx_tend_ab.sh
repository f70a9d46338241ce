# VERIFY_RX / TX_DATAGRAM transport end from the next packet's start: parity, then A/B
# against the previous library in tools/old (measurement only).
set -o pipefail
mkdir -p gpurun_out
YU_RX_FUZZ_ITERS=60 YU_TX_FUZZ_ITERS=60 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "rx or datagram or dg or ragged or fuzz or tun" > gpurun_out/tend_tests.log 2>&1 || { tail -30 gpurun_out/tend_tests.log; exit 1; }
tail -1 gpurun_out/tend_tests.log
args=()
for rep in 1 2 3; do
  args+=("16" "16 LD_LIBRARY_PATH=tools/old" "15 KB_MODE=8" "15 KB_MODE=8 LD_LIBRARY_PATH=tools/old" "15" "15 LD_LIBRARY_PATH=tools/old")
done
bash tools/ab.sh "${args[@]}" > gpurun_out/tend_ab.log 2>&1 || { tail gpurun_out/tend_ab.log; exit 1; }
python3 - <<'PY'
import re,collections
cur=None; d=collections.defaultdict(list)
for l in open('gpurun_out/tend_ab.log'):
    if l.startswith('=='): cur=l.strip()[3:]
    m=re.search(r'round (\d):\s+([\d.]+) us',l)
    if m and cur and m.group(1) != '0': d[cur].append(float(m.group(2)))
for k,v in sorted(d.items()): print(f"{k:50s} min {min(v):6.1f} med {sorted(v)[len(v)//2]:6.1f}")
PY

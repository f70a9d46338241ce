# round 4, call X: TX_DATAGRAM in-place chunk size below 40 (measurement setting
# YU_DG_FILL_CH=40/32/24): parity of the DG fill tests, kbench 15 in place
set -o pipefail
mkdir -p gpurun_out
for ch in 32 24; do
  YU_DG_FILL_CH=$ch timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "tx_datagram" > gpurun_out/gpu_tests_r04x_dg$ch.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r04x_dg$ch.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_r04x_dg$ch.log
done
hipcc -O2 -std=c++17 -Iinclude tools/kbench.cpp -Lyustack_amd -lyucsum -ldl -Wl,-rpath,$PWD/yustack_amd -o /tmp/kbench || exit 1
for i in 1 2 3; do
  for ch in 40 32 24; do
    echo "== YU_DG_FILL_CH=$ch"
    YU_DG_FILL_CH=$ch KB_FILL=1 KB_ALIGN4=1 timeout -k 10 100 /tmp/kbench 15 || exit 1
  done
done > gpurun_out/kbench_ab_r04x_dg_fill_chunk.log 2>&1
python3 - <<'PY'
import re, collections, statistics
d = collections.defaultdict(list); ch = None
for l in open("gpurun_out/kbench_ab_r04x_dg_fill_chunk.log"):
    m = re.match(r"== YU_DG_FILL_CH=(\d+)", l)
    if m: ch = m.group(1); continue
    m = re.match(r"config(\d+) round \d+:\s+([\d.]+) us.*\s(k_\S+)$", l.strip())
    if m: d[(m.group(3), ch)].append(float(m.group(2)))
for k in sorted(d): print(k, "median", statistics.median(d[k]), sorted(d[k]))
PY
echo ok

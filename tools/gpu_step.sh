# round 4, call U: TXW chunk size sweep (measurement settings YU_FILL_WB=1..4:
# 64, 40, 48, 32 packets per chunk) on small UDP (8) and mid-size TCP (7) fills,
# plus parity of the fill tests at 48 and 60
set -o pipefail
mkdir -p gpurun_out
for wb in 2 4; do
  YU_FILL_WB=$wb timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fill_ragged or fuzz" > gpurun_out/gpu_tests_r04u_wb$wb.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r04u_wb$wb.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_r04u_wb$wb.log
done
hipcc -O2 -std=c++17 -Iinclude tools/kbench.cpp -Lyustack_amd -lyucsum -ldl -Wl,-rpath,$PWD/yustack_amd -o /tmp/kbench || exit 1
for i in 1 2 3; do
  for wb in 1 2 3 4; do
    echo "== YU_FILL_WB=$wb"
    YU_FILL_WB=$wb KB_FILL=1 KB_ALIGN4=1 timeout -k 10 120 /tmp/kbench 8 7 || exit 1
  done
done > gpurun_out/kbench_ab_r04u_txw_chunk_sweep.log 2>&1
python3 - <<'PY'
import re, collections
d = collections.defaultdict(list); wb = None
for l in open("gpurun_out/kbench_ab_r04u_txw_chunk_sweep.log"):
    m = re.match(r"== YU_FILL_WB=(\d)", l)
    if m: wb = m.group(1); continue
    m = re.match(r"config(\d+) round \d+:\s+([\d.]+) us", l)
    if m: d[(m.group(1), wb)].append(float(m.group(2)))
for k in sorted(d): print(k, sorted(d[k]))
PY
echo ok

# round 4, call V: k_seg with 40- / 48-packet chunks for the 1M-packet picks
# (YU_SEG_CH, measurement): the GPU suite with 40, then kbench over the ragged
# shapes (4: U{64..9000}, 5: U{64..1500}, 15: TX_DATAGRAM, 16: small RX, 8/7 fills)
set -o pipefail
mkdir -p gpurun_out
YU_SEG_CH=40 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r04v_ch40.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r04v_ch40.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r04v_ch40.log
hipcc -O2 -std=c++17 -Iinclude tools/kbench.cpp -Lyustack_amd -lyucsum -ldl -Wl,-rpath,$PWD/yustack_amd -o /tmp/kbench || exit 1
for i in 1 2 3; do
  for ch in 0 40 48; do
    echo "== YU_SEG_CH=$ch"
    YU_SEG_CH=$ch timeout -k 10 200 /tmp/kbench 4 5 15 16 || exit 1
    YU_SEG_CH=$ch KB_MODE=8 timeout -k 10 100 /tmp/kbench 15 || exit 1
    YU_SEG_CH=$ch KB_FILL=1 KB_ALIGN4=1 timeout -k 10 100 /tmp/kbench 8 7 15 || exit 1
  done
done > gpurun_out/kbench_ab_r04v_seg_chunk.log 2>&1
python3 - <<'PY'
import re, collections
d = collections.defaultdict(list); ch = None
for l in open("gpurun_out/kbench_ab_r04v_seg_chunk.log"):
    m = re.match(r"== YU_SEG_CH=(\d+)", l)
    if m: ch = m.group(1); continue
    m = re.match(r"config(\d+) round \d+:\s+([\d.]+) us.*\s(k_\S+)$", l.strip())
    if m: d[(int(m.group(1)), m.group(3).split(',c')[0].rstrip('>'), ch)].append(float(m.group(2)))
import statistics
for k in sorted(d): print(k, "median", statistics.median(d[k]), sorted(d[k]))
PY
echo ok

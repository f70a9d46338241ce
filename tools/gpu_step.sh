# round 4, call H: the write-back per tile (wb_tile) for TXW and the new DGW kind
# (TX_DATAGRAM in place): GPU suite, fill tests with the write-back off, kbench A/B
# against the round-start library (tools/old), bench line, trace + PMC of 12 / 13
set -o pipefail
mkdir -p gpurun_out
T=r04h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$T.log
YU_FILL_WB=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fill or fuzz or kernel_verified" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_${T}_wb0.log 2>&1 || { tail -40 gpurun_out/gpu_tests_${T}_wb0.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${T}_wb0.log
O=LD_LIBRARY_PATH=tools/old
F="KB_FILL=1 KB_ALIGN4=1"
timeout -k 10 900 bash tools/ab.sh "8 $F $O" "8 $F" "8 $F $O" "8 $F" "7 $F $O" "7 $F" "7 $F $O" "7 $F" "15 $F $O" "15 $F" "15 $F $O" "15 $F" \
  "16 $O" "16" "8 $O" "8" "15 $O" "15" > gpurun_out/kbench_ab_$T.log 2>&1 || { tail gpurun_out/kbench_ab_$T.log; exit 1; }
grep -E "^==|round 2" gpurun_out/kbench_ab_$T.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail gpurun_out/bench_$T.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['roofline']['frac']);[print(k,v['kernel_avg_us'],v['roofline_frac'],v['kernel']) for k,v in d['other_configs'].items()]"
CFGS="12 13" timeout -k 10 600 bash tools/profile.sh $T || exit 1
echo ok

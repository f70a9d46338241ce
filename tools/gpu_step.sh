# round 4, call B: GPU suite on the tree with the 4-wave RX kind (SegChunk32, fused
# park) and the TX kind's whole-line in-place write-back; the fill tests under each
# YU_FILL_WB (tools/wbplain: the write-back with plain stores); kbench A/B against the round-start library (tools/old); fill A/B with
# WRITE_SIZE; SQ counters for config 7 both ways; the driver-style bench line; trace +
# PMC passes of configs 7, 12, 13
set -o pipefail
mkdir -p gpurun_out/pmc_fillwb
T=r04b
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
for wb in 0; do
  YU_FILL_WB=$wb timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fill or fuzz or kernel_verified" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_${T}_wb$wb.log 2>&1 || { tail -40 gpurun_out/gpu_tests_${T}_wb$wb.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_${T}_wb$wb.log
done
O=LD_LIBRARY_PATH=tools/old
F="KB_FILL=1 KB_ALIGN4=1"
P=LD_LIBRARY_PATH=tools/wbplain
timeout -k 10 900 bash tools/ab.sh "16 $O" "16" "16 $O" "16" "16 $O" "16" "6 $O" "6" "5 $O" "5" "4 $O" "4" "15 $O" "15" "8 $O" "8" "3 $O" "3" \
  "8 $F $O" "8 $F YU_FILL_WB=0" "8 $F" "8 $F $P" "8 $F $O" "8 $F YU_FILL_WB=0" "8 $F" "8 $F $P" \
  "7 $F YU_FILL_WB=0" "7 $F" "7 $F $P" "15 $F $O" "15 $F" > gpurun_out/kbench_ab_$T.log 2>&1 || { tail gpurun_out/kbench_ab_$T.log; exit 1; }
grep -E "^==|round 2" gpurun_out/kbench_ab_$T.log
cd /tmp && export TMPDIR=/tmp
for wb in 0 1; do
  for c in WRITE_SIZE FETCH_SIZE; do
    YU_FILL_WB=$wb KB_FILL=1 KB_ALIGN4=1 timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmc_fillwb/wb${wb}_$c -o run -- $R/tools/kbench 8 > $R/gpurun_out/pmc_fillwb/wb${wb}_$c.txt 2>&1 || { echo "pmc wb$wb $c failed"; exit 1; }
  done
done
cd $R
TAG=_new bash tools/pmc_sq.sh 16 || exit 1
TAG=_old bash tools/pmc_sq.sh 16 LD_LIBRARY_PATH=$R/tools/old || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail gpurun_out/bench_$T.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['roofline']['frac']);[print(k,v['kernel_avg_us'],v['roofline_frac']) for k,v in d['other_configs'].items()]"
CFGS="7 12 13" timeout -k 10 600 bash tools/profile.sh $T || exit 1
echo ok

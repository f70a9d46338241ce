# round 4, call B: GPU suite on the tree with the 4-wave RX kind (SegChunk32, fused
# park), kbench A/B against HEAD's library (tools/old), SQ counters for config 7
# both ways, the driver-style bench line, trace + PMC passes of configs 7, 12, 13
set -o pipefail
mkdir -p gpurun_out
T=r04b
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$T.log
O=LD_LIBRARY_PATH=tools/old
timeout -k 10 900 bash tools/ab.sh "16 $O" "16" "16 $O" "16" "16 $O" "16" "6 $O" "6" "5 $O" "5" "4 $O" "4" "15 $O" "15" "8 $O" "8" "3 $O" "3" "8 KB_FILL=1 KB_ALIGN4=1 $O" "8 KB_FILL=1 KB_ALIGN4=1" "15 KB_FILL=1 KB_ALIGN4=1 $O" "15 KB_FILL=1 KB_ALIGN4=1" > gpurun_out/kbench_ab_$T.log 2>&1 || { tail gpurun_out/kbench_ab_$T.log; exit 1; }
grep -E "^==|round 2" gpurun_out/kbench_ab_$T.log
TAG=_new bash tools/pmc_sq.sh 16 || exit 1
TAG=_old bash tools/pmc_sq.sh 16 LD_LIBRARY_PATH=$R/tools/old || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail gpurun_out/bench_$T.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));print(d['value'],d['roofline']['frac']);[print(k,v['kernel_avg_us'],v['roofline_frac']) for k,v in d['other_configs'].items()]"
CFGS="7 12 13" timeout -k 10 600 bash tools/profile.sh $T || exit 1
echo ok

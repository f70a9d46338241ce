# round 4, call M: TX_DATAGRAM in place storing each field as soon as its value is
# known (while the header line is probably still in L2): GPU suite, the fill tests
# with the write-back off, kbench A/B against the previous commit (tools/prev)
set -o pipefail
mkdir -p gpurun_out
T=r04m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1 || { tail -60 gpurun_out/gpu_tests_$T.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$T.log
P=LD_LIBRARY_PATH=tools/prev
F="KB_FILL=1 KB_ALIGN4=1"
timeout -k 10 900 bash tools/ab.sh "15 $F $P" "15 $F" "15 $F $P" "15 $F" "15 $F $P" "15 $F" "15 $P" "15" > gpurun_out/kbench_ab_$T.log 2>&1 || { tail gpurun_out/kbench_ab_$T.log; exit 1; }
grep -E "^==|round 2" gpurun_out/kbench_ab_$T.log
echo ok

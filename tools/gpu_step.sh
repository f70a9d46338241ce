# round 4, call S: TXW with 56-packet chunks (YU_FILL_WB=2, measurement setting):
# parity of the fill / fuzz / kernel-verified tests with it, then kbench A/B against
# the 64-packet TXW kind on small UDP (8) and mid-size TCP (7) fills
set -o pipefail
mkdir -p gpurun_out
YU_FILL_WB=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "fill or fuzz or kernel_verified" > gpurun_out/gpu_tests_r04s_c56.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r04s_c56.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r04s_c56.log
hipcc -O2 -std=c++17 -Iinclude tools/kbench.cpp -Lyustack_amd -lyucsum -ldl -Wl,-rpath,$PWD/yustack_amd -o /tmp/kbench || exit 1
for i in 1 2 3; do
  for wb in 1 2; do
    echo "== YU_FILL_WB=$wb"
    YU_FILL_WB=$wb KB_FILL=1 KB_ALIGN4=1 timeout -k 10 120 /tmp/kbench 8 7 || exit 1
  done
done > gpurun_out/kbench_ab_r04s_txw_c56.log 2>&1
grep -E "==|config" gpurun_out/kbench_ab_r04s_txw_c56.log | tail -30
echo ok

# k_rl (one lane per packet, ragged small packets) prototype: parity with YU_RAGGED=lane forced, then A/B against k_seg
set -o pipefail
mkdir -p gpurun_out
YU_RAGGED=lane timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_krl.log 2>&1 || { tail -30 gpurun_out/gpu_tests_krl.log; exit 1; }
tail -2 gpurun_out/gpu_tests_krl.log
bash tools/ab.sh "6" "6 YU_RAGGED=lane" "6 YU_RAGGED=lane4" "6 YU_RAGGED=lane YU_NT=1" \
  "8" "8 YU_RAGGED=lane" "8 YU_RAGGED=lane4" "5" "5 YU_RAGGED=lane" "7" "7 YU_RAGGED=lane" \
  "6" "6 YU_RAGGED=lane" "6 YU_RAGGED=lane4" > gpurun_out/kbench_ab_krl.log 2>&1 || { tail gpurun_out/kbench_ab_krl.log; exit 1; }
grep -E "^==|round 1" gpurun_out/kbench_ab_krl.log

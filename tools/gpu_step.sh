# round 4, call J: the rest of the closing profiles (trace + PMC of configs 6, 7, 9,
# 10, 11, 12, 13), and the fill / fuzz tests with the ragged kernels forced to 4 KiB
# tiles (YU_RAGGED=seg4: the TXW kind's k_seg<4,txw> form)
set -o pipefail
mkdir -p gpurun_out
T=r04i
YU_RAGGED=seg4 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fill or fuzz or kernel_verified" --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_${T}_seg4.log 2>&1 || { tail -40 gpurun_out/gpu_tests_${T}_seg4.log; exit 1; }
tail -1 gpurun_out/gpu_tests_${T}_seg4.log
CFGS="6 7 9 10 11 12 13" timeout -k 10 1000 bash tools/profile.sh $T || exit 1
echo ok

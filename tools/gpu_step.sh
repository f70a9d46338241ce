set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "multi_device" > gpurun_out/t_multi.log 2>&1 || { tail -30 gpurun_out/t_multi.log; exit 1; }
tail -1 gpurun_out/t_multi.log

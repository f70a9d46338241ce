set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/t_cpp.log 2>&1 || { tail -30 gpurun_out/t_cpp.log; exit 1; }
tail -1 gpurun_out/t_cpp.log

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "tx_datagram or refexec" > gpurun_out/t_dg.log 2>&1 || { tail -40 gpurun_out/t_dg.log; exit 1; }
tail -2 gpurun_out/t_dg.log

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "rx or tx_datagram or fuzz or ragged" > gpurun_out/t_rx.log 2>&1 || { tail -30 gpurun_out/t_rx.log; exit 1; }
tail -1 gpurun_out/t_rx.log
args=()
for r in 1 2; do
  args+=("15" "15 LD_LIBRARY_PATH=tools/old" "15 KB_MODE=8" "15 KB_MODE=8 LD_LIBRARY_PATH=tools/old" "16" "16 LD_LIBRARY_PATH=tools/old")
done
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_rx.log 2>&1 || { tail gpurun_out/ab_rx.log; exit 1; }

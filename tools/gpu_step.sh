set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "tx_datagram" > gpurun_out/t_dg.log 2>&1 || { tail -30 gpurun_out/t_dg.log; exit 1; }
tail -2 gpurun_out/t_dg.log
args=()
for r in 1 2; do
  args+=("15" "15 LD_LIBRARY_PATH=tools/old" "15 KB_FILL=1" "15 KB_FILL=1 LD_LIBRARY_PATH=tools/old" "15 KB_MODE=8")
done
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_dg.log 2>&1 || { tail gpurun_out/ab_dg.log; exit 1; }
grep -E "==|round 2" gpurun_out/ab_dg.log | paste - - | awk '{print $3,$4,$5,$6,$10,$11,$NF}'

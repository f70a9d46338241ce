set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "tx or fill or fuzz or ragged" > gpurun_out/t_tx.log 2>&1 || { tail -30 gpurun_out/t_tx.log; exit 1; }
tail -2 gpurun_out/t_tx.log
args=()
for r in 1 2; do
  args+=("7" "7 LD_LIBRARY_PATH=tools/old" "8" "8 LD_LIBRARY_PATH=tools/old" "7 KB_FILL=1 KB_ALIGN4=1" "7 KB_FILL=1 KB_ALIGN4=1 LD_LIBRARY_PATH=tools/old" "8 KB_FILL=1 KB_ALIGN4=1" "8 KB_FILL=1 KB_ALIGN4=1 LD_LIBRARY_PATH=tools/old")
done
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_tx.log 2>&1 || { tail gpurun_out/ab_tx.log; exit 1; }

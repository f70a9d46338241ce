set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "small or uniform or fill or fuzz or config" > gpurun_out/t_ks.log 2>&1 || { tail -30 gpurun_out/t_ks.log; exit 1; }
tail -1 gpurun_out/t_ks.log
args=()
for r in 1 2 3; do
  args+=("3" "3 LD_LIBRARY_PATH=tools/old")
done
args+=("3 KB_FILL=1" "3 KB_FILL=1 LD_LIBRARY_PATH=tools/old" "14 KB_LEN=768" "14 KB_LEN=768 LD_LIBRARY_PATH=tools/old" "14 KB_LEN=2000" "14 KB_LEN=2000 LD_LIBRARY_PATH=tools/old" "3 KB_N=131072" "3 KB_N=131072 LD_LIBRARY_PATH=tools/old")
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_ks.log 2>&1 || { tail gpurun_out/ab_ks.log; exit 1; }

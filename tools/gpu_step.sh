set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "k_small or full_size or transport_uniform or fuzz or 1500 or refexec" > gpurun_out/t_dpp.log 2>&1 || { tail -30 gpurun_out/t_dpp.log; exit 1; }
tail -1 gpurun_out/t_dpp.log
args=()
for r in 1 2 3; do args+=("3 LD_LIBRARY_PATH=tools/old" "3"); done
args+=("14 KB_LEN=768 LD_LIBRARY_PATH=tools/old" "14 KB_LEN=768" "14 KB_LEN=2000 LD_LIBRARY_PATH=tools/old" "14 KB_LEN=2000")
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_dpp.log 2>&1 || { tail gpurun_out/ab_dpp.log; exit 1; }
grep -E "==|round 2" gpurun_out/ab_dpp.log

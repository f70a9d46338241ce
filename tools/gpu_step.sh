set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "lane or tiny or fill or fuzz or full_size or uniform" > gpurun_out/t_grid6.log 2>&1 || { tail -30 gpurun_out/t_grid6.log; exit 1; }
tail -1 gpurun_out/t_grid6.log
args=()
for r in 1 2; do
 for c in "2" "14 KB_LEN=72" "14 KB_LEN=32" "14 KB_LEN=124" "14 KB_LEN=72 KB_FILL=1" "14 KB_LEN=64 KB_FILL=1"; do args+=("$c LD_LIBRARY_PATH=tools/old" "$c"); done
done
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_grid6.log 2>&1 || { tail gpurun_out/ab_grid6.log; exit 1; }
grep -E "==|round 2" gpurun_out/ab_grid6.log | paste - - | awk '{print $3,$4,$5,$6, $10, $11}'

set -o pipefail
mkdir -p gpurun_out
args=()
for n in 16384 32768 65536 131072; do
  args+=("3 KB_N=$n YU_RUNS=0" "3 KB_N=$n YU_RUNS=2" "14 KB_LEN=768 KB_N=$n YU_RUNS=0" "14 KB_LEN=768 KB_N=$n YU_RUNS=2")
done
for r in 1 2 3; do args+=("3 LD_LIBRARY_PATH=tools/old" "3"); done
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_run6.log 2>&1 || { tail gpurun_out/ab_run6.log; exit 1; }
grep -E "==|round 2" gpurun_out/ab_run6.log

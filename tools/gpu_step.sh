set -o pipefail
mkdir -p gpurun_out
args=()
for r in 1 2; do
  args+=("3")
  for b in 2 3 4 6 8; do args+=("3 YU_RUNS=0 YU_BLOCKS_PER_CU=$b" "3 YU_RUNS=0 YU_BLOCKS_PER_CU=$b YU_NT=1"); done
done
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_inter_lowgrid.log 2>&1 || { tail gpurun_out/ab_inter_lowgrid.log; exit 1; }
grep -E "==|round 2" gpurun_out/ab_inter_lowgrid.log | paste - - | awk '{print $3,$4,$5,$6,$10,$11}'

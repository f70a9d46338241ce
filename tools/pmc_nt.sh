#!/bin/bash
# FETCH_SIZE of kbench config 3 under both load policies (measurement only).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_nt
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
for nt in 2 1 0; do
  YU_NT=$nt YU_BLOCKS_PER_CU=64 timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/nt$nt" -o run -- "$ROOT/tools/kbench" 3 > "$OUT/kbench_nt$nt.txt"
  YU_NT=$nt YU_BLOCKS_PER_CU=64 timeout -k 10 200 "$ROOT/tools/kbench" 3 > "$OUT/kbench_nt${nt}_plain.txt"
done

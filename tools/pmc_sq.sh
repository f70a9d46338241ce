#!/bin/bash
# SQ stall breakdown of one kbench config (measurement only; run on the GPU box):
# tools/pmc_sq.sh <cfg> [ENV=val ...]  ->  gpurun_out/sq_<cfg>/...
# WAIT_ANY (waitcnt/barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY ~ WAVE_CYCLES.
set -eu
cfg=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sq_${cfg}${TAG:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
env "$@" timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$OUT" -o run -- "$ROOT/tools/kbench" "$cfg" > "$OUT/kbench.txt"

#!/bin/bash
# SQ stall breakdown of one kbench config (measurement only; run on the GPU box):
# tools/pmc_sq.sh <cfg> [ENV=val ...]  ->  gpurun_out/sq_<cfg>/...
# WAIT_ANY (waitcnt/barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY ~ WAVE_CYCLES.
# SQ_COUNTERS="..." replaces the set (at most 8 SQ_ counters per pass).
set -eu
cfg=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/sq_${cfg}${TAG:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CTRS=${SQ_COUNTERS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"}
# shellcheck disable=SC2086
env "$@" timeout -s KILL 90 rocprofv3 --pmc $CTRS --output-format csv -d "$OUT" -o run -- "$ROOT/tools/kbench" "$cfg" > "$OUT/kbench.txt"

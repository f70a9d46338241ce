#!/bin/bash
# kbench sweep over the persistent-grid size and the load policy (measurement only).
# usage: tools/sweep.sh "<nt values>" "<blocks/CU values>" [configs...]
NTS=${1:-"1 0"}; BS=${2:-"2 4 8 16"}; shift 2
for nt in $NTS; do for b in $BS; do
  echo "== YU_NT=$nt YU_BLOCKS_PER_CU=$b"
  YU_NT=$nt YU_BLOCKS_PER_CU=$b timeout -k 5 120 tools/kbench "$@" || exit 1
done; done

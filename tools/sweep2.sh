#!/bin/bash
# Grid-size x variant sweep for one config (measurement only).
cfg=$1
for v in "" "k_small<32,6>" "k_small<64,4>"; do for b in 4 6 8 12 16 24 32; do
  echo "== VARIANT=${v:-auto} YU_BLOCKS_PER_CU=$b"
  YU_VARIANT=$v YU_BLOCKS_PER_CU=$b timeout -k 5 120 tools/kbench $cfg || exit 1
done; done

#!/bin/bash
# Variant / grid A/B on the GPU box (measurement only): tools/ab.sh "<cfg> <VAR=val ...>" ...
# Each argument is one kbench run: a config number followed by env assignments.
# The library reads its measurement knobs only under YU_TUNING=1, which every run sets.
set -u
for spec in "$@"; do
  read -r cfg envs <<< "$spec"
  echo "== config $cfg ${envs:-default}"
  env YU_TUNING=1 $envs timeout -k 5 120 tools/kbench "$cfg" || exit 1
done

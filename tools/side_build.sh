#!/bin/bash
# Side build of libyucsum.so for A/B runs and tracing (measurement only; never the shipped
# library, which is always yustack_amd/libyucsum.so built from the working tree).
#   tools/side_build.sh <dir> [rev|WORK] [patch.py]
#   <dir>     output directory, e.g. tools/old; load it with LD_LIBRARY_PATH=<dir> (tools/ab.sh)
#   rev       sources at that git revision (default HEAD); WORK = the working tree
#   patch.py  run on the copied kernel file, e.g. tools/seg_trace_patch.py for tools/seg_trace
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/${1:?usage: side_build.sh <dir> [rev|WORK] [patch.py]}
REV=${2:-HEAD}
PATCH=${3:-}
rm -rf "$D/yustack_amd" "$D/include"
mkdir -p "$D/yustack_amd/csrc" "$D/include"
get() {  # get <repo path> <dest>
  if [ "$REV" = WORK ]; then cp "$ROOT/$1" "$2"; else git -C "$ROOT" show "$REV:$1" > "$2"; fi
}
for f in Makefile yucsum_kernels.hip yucsum_host.cpp yucsum_scalar.cpp yucsum_internal.h; do
  get "yustack_amd/csrc/$f" "$D/yustack_amd/csrc/$f"
done
get include/yucsum.h "$D/include/yucsum.h"
if [ -n "$PATCH" ]; then python3 "$PATCH" "$D/yustack_amd/csrc/yucsum_kernels.hip"; fi
make -s -C "$D/yustack_amd/csrc" -j8
# one copy of the library, no objects: every gpurun call ships the tree
mv "$D/yustack_amd/libyucsum.so" "$D/libyucsum.so"
rm -rf "$D/yustack_amd/csrc/build"
echo "built $D/libyucsum.so from ${REV}${PATCH:+ + $PATCH}"

set -o pipefail
mkdir -p gpurun_out
args=()
for r in 1 2; do for c in "8 KB_FILL=1 KB_ALIGN4=1" "7 KB_FILL=1 KB_ALIGN4=1" "8 KB_ALIGN4=1"; do args+=("$c LD_LIBRARY_PATH=tools/old" "$c"); done; done
bash tools/ab.sh "${args[@]}" > gpurun_out/ab_tilewb2.log 2>&1 || { tail gpurun_out/ab_tilewb2.log; exit 1; }
grep -E "==|round 2" gpurun_out/ab_tilewb2.log

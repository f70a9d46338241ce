# ablation (timing only, values wrong): k_seg DG kind without the transport field's byte reads (tools/varA)
set -o pipefail
mkdir -p gpurun_out
A=LD_LIBRARY_PATH=tools/varA
bash tools/ab.sh "15" "15 $A" "5 KB_MODE=8" "15" "15 $A" "5 KB_MODE=8" > gpurun_out/kbench_abl_dg_fb.log 2>&1 || { tail gpurun_out/kbench_abl_dg_fb.log; exit 1; }
grep -E "^==|round" gpurun_out/kbench_abl_dg_fb.log

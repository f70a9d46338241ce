# round 4, call K: load policy of the ragged in-place writers -- plain loads
# (YU_NT=0: the field's line more often still cached when its store arrives) against
# the default non-temporal k_seg loads, for TX_DATAGRAM in place (kbench 15), TCP
# segments U{64..1500} (7) and small UDP datagrams (8, the TXW kind)
set -o pipefail
mkdir -p gpurun_out
F="KB_FILL=1 KB_ALIGN4=1"
timeout -k 10 900 bash tools/ab.sh "15 $F" "15 $F YU_NT=0" "15 $F" "15 $F YU_NT=0" "7 $F" "7 $F YU_NT=0" "7 $F" "7 $F YU_NT=0" \
  "8 $F" "8 $F YU_NT=0" "8 $F" "8 $F YU_NT=0" "15" "15 YU_NT=0" > gpurun_out/kbench_ab_r04k_fill_nt.log 2>&1 || { tail gpurun_out/kbench_ab_r04k_fill_nt.log; exit 1; }
grep -E "^==|round" gpurun_out/kbench_ab_r04k_fill_nt.log
echo ok

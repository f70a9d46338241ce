# round 4, call F: SQ instruction / stall counters of config 7's kernel (kbench 16):
# the round-start RX kind (tools/old) against the one-tile straight-line path
# (tools/rxfast, side build of 3e46d4c) -- did that path cut instructions?
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
C2="SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_BRANCH"
for lib in old rxfast; do
  TAG=_${lib}_a SQ_COUNTERS="$C1" bash tools/pmc_sq.sh 16 LD_LIBRARY_PATH=$R/tools/$lib || exit 1
  TAG=_${lib}_b SQ_COUNTERS="$C2" bash tools/pmc_sq.sh 16 LD_LIBRARY_PATH=$R/tools/$lib || exit 1
done
python3 tools/sq_summary.py gpurun_out/sq_16_old_a gpurun_out/sq_16_rxfast_a gpurun_out/sq_16_old_b gpurun_out/sq_16_rxfast_b
echo ok

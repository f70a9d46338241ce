# round-3 tree after the k_seg instruction cuts: bench line at the driver's settings, trace + PMC of
# configs 6, 7, 11, and SQ stall counters of the small-datagram shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03d.json 2> gpurun_out/bench_r03d.err || { tail gpurun_out/bench_r03d.err; exit 1; }
CFGS="7 6 11" timeout -k 10 600 bash tools/profile.sh r03b > gpurun_out/profile_r03b.log 2>&1 || { tail -20 gpurun_out/profile_r03b.log; exit 1; }
LDSC="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
for c in 16 6 3; do bash tools/pmc_sq.sh $c || exit 1; done
python tools/sq_summary.py gpurun_out/sq_* > gpurun_out/sq_summary_r03.txt
for c in 16 6 3; do TAG=_lds SQ_COUNTERS="$LDSC" bash tools/pmc_sq.sh $c || exit 1; done
python tools/sq_summary.py gpurun_out/sq_* > gpurun_out/sq_summary_r03.txt
echo ok

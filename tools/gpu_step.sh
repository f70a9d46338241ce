# the GPU parity suite with each ragged measurement override forced (k_rag, 4 KiB k_seg, 16-packet
# chunks, a wave per packet): every ragged kernel the selection can be forced onto, bit-exact
set -o pipefail
mkdir -p gpurun_out
for r in rag seg4 seg16 loop; do
  YU_RAGGED=$r timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_forced_$r.log 2>&1 || { tail -30 gpurun_out/gpu_tests_forced_$r.log; exit 1; }
  echo "$r: $(tail -1 gpurun_out/gpu_tests_forced_$r.log)"
done

#!/bin/bash
# The GPU parity and out-of-contract suites with each ragged measurement override forced (run on the GPU
# box). The library reads the override only under YU_TUNING=1, and the tests then
# assert parity only, not the default kernel choice (tests/test_gpu_parity.py FORCED).
# Logs under gpurun_out/forced/; the first failure or time limit ends the script.
#   gpurun --timeout 1500 -- 'bash tools/forced_suite.sh r05c'
set -o pipefail
TAG=${1:-forced}
mkdir -p gpurun_out/forced
for v in ${FORCED_VARIANTS:-rag seg4 seg16 loop}; do
  # the override took effect: the kernel the library picks for a 1M-packet RAW batch
  echo "$v: picks $(YU_TUNING=1 YU_RAGGED=$v python -c 'from yustack_amd import batch; print(batch.ragged_variant("raw", 1 << 20))' 2>/dev/null)"
  YU_TUNING=1 YU_RAGGED=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contract.py \
    -m gpu -q -x \
    --timeout 240 --timeout-method thread > gpurun_out/forced/gpu_tests_${TAG}_$v.log 2>&1 \
    || { tail -30 gpurun_out/forced/gpu_tests_${TAG}_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/forced/gpu_tests_${TAG}_$v.log)"
done

#!/bin/bash
# Round-end verification on the GPU box, the same three steps the driver runs:
# GPU parity tests, smoke(), and the default bench line. Each step has its own
# time limit; the first failure ends the script. Logs under gpurun_out/.
#   gpurun --timeout 1100 -- 'bash tools/verify_round.sh final5'
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -1 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
echo ok

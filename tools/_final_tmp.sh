set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_final5.log 2>&1 || { tail -40 gpurun_out/gpu_tests_final5.log; exit 1; }
tail -1 gpurun_out/gpu_tests_final5.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke5.log 2>&1 || { tail gpurun_out/smoke5.log; exit 1; }
tail -1 gpurun_out/smoke5.log
timeout -k 10 400 python bench.py > gpurun_out/bench_final5.json 2> gpurun_out/bench_final5.err || { tail gpurun_out/bench_final5.err; exit 1; }
echo ok

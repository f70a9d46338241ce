set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_r03a.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r03a.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r03a.log
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench_r03a_2ranks.json 2> gpurun_out/bench_r03a_2ranks.err || { tail gpurun_out/bench_r03a_2ranks.err; exit 1; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err || { tail gpurun_out/bench_r03a.err; exit 1; }
echo ok

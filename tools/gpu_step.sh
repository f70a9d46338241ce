# round 4, last calls: the final tree verified as the driver runs it (GPU suite,
# smoke, default bench line: tools/verify_round.sh) plus the driver-settings line.
#   gpurun --timeout 1200 -- 'bash tools/gpu_step.sh r04f'
set -o pipefail
TAG=${1:-final}
mkdir -p gpurun_out
bash tools/verify_round.sh $TAG || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_driver.json 2> gpurun_out/bench_${TAG}_driver.err || { tail gpurun_out/bench_${TAG}_driver.err; exit 1; }
echo bench-ok

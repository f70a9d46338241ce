# scratch: the GPU step of the current session's latest gpurun call (round 5).
# The suite runs to the end unless it dies (test failures are read from the log;
# a fault, abort, signal or time limit ends the call), then smoke() and the default
# bench line, each under its own time limit.
#   gpurun --timeout 1200 -- 'bash tools/gpu_step.sh r05a'
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 -rf --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests_$TAG.log
[ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
[ $rc -eq 0 ] || { echo "pytest rc $rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_driver.json 2> gpurun_out/bench_${TAG}_driver.err || { tail gpurun_out/bench_${TAG}_driver.err; exit 1; }
echo bench-ok
if [ -n "${ASAN:-}" ]; then
  ASAN_OPTIONS=detect_leaks=0 timeout -k 10 300 tests/cpp/build/test_checksum_asan --gpu > gpurun_out/cpp_asan_$TAG.log 2>&1 || { tail -30 gpurun_out/cpp_asan_$TAG.log; exit 1; }
  tail -1 gpurun_out/cpp_asan_$TAG.log
fi
if [ -n "${FUZZ_SEED_BASE:-}" ]; then
  bash tools/fuzz_long.sh || exit 1
fi
[ -n "${PROF_CFGS:-}" ] || exit 0
CFGS="$PROF_CFGS" timeout -k 10 900 bash tools/profile.sh $TAG || exit 1
echo prof-ok

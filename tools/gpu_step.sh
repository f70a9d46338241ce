# round 4, call R: the C++ tests with the pipelined host batches added, plain and
# with the host code under ASan + UBSan (tools/build_asan.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_cpp.py -m gpu > gpurun_out/cpp_gpu_r04r.log 2>&1 || { tail -30 gpurun_out/cpp_gpu_r04r.log; exit 1; }
tail -1 gpurun_out/cpp_gpu_r04r.log
ASAN_OPTIONS=detect_leaks=0 timeout -k 10 300 tests/cpp/build/test_checksum_asan --gpu > gpurun_out/cpp_asan_r04r.log 2>&1 || { tail -40 gpurun_out/cpp_asan_r04r.log; exit 1; }
tail -2 gpurun_out/cpp_asan_r04r.log
echo ok

# round 4, call Q: the C++ reference-style tests, batched device and host paths
# included, with the host code under ASan + UBSan (device code as shipped; built
# here by tools/build_asan.sh, -fsanitize only after -Xarch_host)
set -o pipefail
mkdir -p gpurun_out
ASAN_OPTIONS=detect_leaks=0 timeout -k 10 300 tests/cpp/build/test_checksum_asan --gpu > gpurun_out/cpp_asan_r04q.log 2>&1 || { tail -40 gpurun_out/cpp_asan_r04q.log; exit 1; }
tail -2 gpurun_out/cpp_asan_r04q.log
echo ok

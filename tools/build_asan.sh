#!/bin/bash
# Builds tests/cpp/build/test_checksum_asan: the C++ reference-style tests
# (tests/cpp/test_checksum.cpp) linked with the product sources compiled in, the
# HOST code under AddressSanitizer + UBSan (each -fsanitize after -Xarch_host; the
# gfx950 device code is compiled as shipped — GPU sanitizers are not available).
# Run on the GPU box:  ASAN_OPTIONS=detect_leaks=0 tests/cpp/build/test_checksum_asan --gpu
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p tests/cpp/build
/opt/rocm/bin/hipcc -O1 -g -std=c++17 --offload-arch=gfx950 \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer \
  -DYU_TEST_QUICK_EXIT -Iinclude -Iyustack_amd/csrc \
  tests/cpp/test_checksum.cpp yustack_amd/csrc/yucsum_host.cpp yustack_amd/csrc/yucsum_scalar.cpp \
  yustack_amd/csrc/yucsum_kernels.hip \
  -Loracle/build -lcsum_oracle -Wl,-rpath,'$ORIGIN/../../../oracle/build' \
  -o tests/cpp/build/test_checksum_asan

"""Builds and runs tests/cpp/test_checksum.cpp (C++ mirror of the reference API,
reference-style packet tests). CPU part here; the batched part under -m gpu."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "test_checksum.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_checksum")


@pytest.fixture(scope="module")
def binary():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(
            os.path.getmtime(SRC), os.path.getmtime(os.path.join(ROOT, "include", "yustack", "checksum.hpp"))):
        cmd = ["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", f"-I{ROOT}/include", SRC, "-o", BIN,
               f"-L{ROOT}/yustack_amd", "-lyucsum", f"-L{ROOT}/oracle/build", "-lcsum_oracle",
               f"-Wl,-rpath,{ROOT}/yustack_amd", f"-Wl,-rpath,{ROOT}/oracle/build",
               "-Wl,-rpath,$ORIGIN/../../../yustack_amd", "-Wl,-rpath,$ORIGIN/../../../oracle/build"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
    return BIN


def test_cpp_reference_style_cpu(binary):
    r = subprocess.run([binary], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "ok" in r.stdout


@pytest.mark.gpu
def test_cpp_reference_style_gpu(binary):
    r = subprocess.run([binary, "--gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "cpu+gpu" in r.stdout

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


SAN = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
       "-fno-omit-frame-pointer", f"-I{ROOT}/include"]


def test_scalar_and_mirror_under_sanitizers(tmp_path):
    """Host code under AddressSanitizer + UBSan (host only: GPU sanitizers are not
    available): the scalar drop-in against the oracle on exact-size buffers at every
    alignment (tests/cpp/sanitize_scalar.cpp), and the C++ mirror's reference-style
    packet tests (the CPU part of tests/cpp/test_checksum.cpp)."""
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")
    scalar = str(tmp_path / "sanitize_scalar")
    r = subprocess.run(["g++", *SAN, os.path.join(ROOT, "tests", "cpp", "sanitize_scalar.cpp"),
                        os.path.join(ROOT, "yustack_amd", "csrc", "yucsum_scalar.cpp"),
                        "-x", "c", os.path.join(ROOT, "oracle", "csum_oracle.c"), "-lpthread", "-o", scalar],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([scalar], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]
    mirror = str(tmp_path / "test_checksum_san")
    r = subprocess.run(["g++", *SAN, "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", SRC,
                        f"-L{ROOT}/yustack_amd", "-lyucsum", f"-L{ROOT}/oracle/build", "-lcsum_oracle",
                        "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{ROOT}/yustack_amd",
                        f"-Wl,-rpath,{ROOT}/oracle/build", "-o", mirror],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([mirror], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]

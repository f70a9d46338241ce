"""Static checks of the cgo shim (bindings/go/checksum), which this image cannot
compile (no Go toolchain): every C function it calls is declared in include/yucsum.h
and exported by libyucsum.so, every C constant it names is defined there, each cgo
preamble compiles as C against the header, and each file keeps to its Go toolchain
floor."""
import glob
import os
import re
import subprocess

import pytest

from yustack_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GODIR = os.path.join(ROOT, "bindings", "go", "checksum")
HDR = os.path.join(ROOT, "include", "yucsum.h")
# file -> the newest Go release it may need. The scalar drop-in and the packed-batch
# calls must build with the Go the reference's unchanged callers need (1.10:
# sleep/sleep_unsafe.go:66-67 declares runtime.gopark with its Go 1.10 signature);
# the per-packet burst calls need runtime.Pinner (Go 1.21) and say so in a build
# constraint.
FLOORS = {"checksum.go": (1, 10), "batch.go": (1, 10), "checksum_test.go": (1, 10),
          "packets_go121.go": (1, 21), "packets_go121_test.go": (1, 21)}
# APIs and syntax newer than Go 1.10, with the release that introduced them
POST_110 = {
    r"\bunsafe\.Slice\b": (1, 17), r"\bunsafe\.(Add|String|StringData|SliceData)\b": (1, 17),
    r"\bruntime\.Pinner\b": (1, 21), r"\bany\b": (1, 18), r"\[\w+ (any|comparable)\]": (1, 18),
    r"\b(min|max|clear)\(": (1, 21), r"\berrors\.(Is|As|Unwrap|Join)\b": (1, 13), r"%w": (1, 13),
    r"\bstrings\.(Cut|Builder)\b": (1, 10), r"\b(os\.ReadFile|os\.WriteFile|io\.ReadAll)\b": (1, 16),
    r"^//go:build": (1, 17), r"\bt\.(Cleanup|TempDir|Setenv)\(": (1, 14),
}


def _files(tests=False):
    return sorted(f for f in glob.glob(os.path.join(GODIR, "*.go")) if tests or not f.endswith("_test.go"))


def _go():
    """The package's non-test source, all files."""
    return "\n".join(open(f).read() for f in _files())


def test_every_go_file_has_a_floor():
    assert {os.path.basename(f) for f in _files(tests=True)} == set(FLOORS)


@pytest.mark.parametrize("name", sorted(FLOORS))
def test_go_file_keeps_to_its_toolchain_floor(name):
    src = open(os.path.join(GODIR, name)).read()
    code = "\n".join(ln for ln in src.splitlines() if not ln.lstrip().startswith("//") or ln.startswith("//go:build"))
    floor = FLOORS[name]
    for pat, since in POST_110.items():
        if since > floor:
            assert not re.search(pat, code, re.M), f"{name} uses {pat} (Go {since[0]}.{since[1]}), floor {floor}"
    if floor > (1, 10):  # newer than the callers' toolchain: excluded from it by a constraint
        tag = f"go{floor[0]}.{floor[1]}"
        assert src.startswith(f"//go:build {tag}\n// +build {tag}\n\npackage checksum"), name
    else:
        assert "+build" not in src and "//go:build" not in src, name


def test_scalar_drop_in_stands_alone():
    """checksum.go alone holds the reference's three functions and the #cgo flags;
    packets_go121.go is the only user of runtime.Pinner."""
    src = open(os.path.join(GODIR, "checksum.go")).read()
    for sig in ("func Checksum(buf []byte, initial uint16) uint16",
                "func PseudoHeaderChecksum(protocol uint32, srcAddr string, dstAddr string) uint16",
                "func ChecksumCombine(a, b uint16) uint16"):
        assert sig in src
    assert "#cgo LDFLAGS" in src and "\"runtime\"" not in src
    for f in _files(tests=True):
        code = [ln for ln in open(f).read().splitlines() if not ln.lstrip().startswith("//")]
        if any("runtime.Pinner" in ln for ln in code):
            assert os.path.basename(f) == "packets_go121.go", f


def test_go_calls_are_declared_and_exported():
    go, hdr = _go(), open(HDR).read()
    calls = set(re.findall(r"\bC\.(yu_\w+)\(", go))
    assert {"yu_checksum", "yu_csum_batch_host_uniform", "yu_csum_batch_host_ragged_multi",
            "yu_csum_batch_host_iov_multi"} <= calls
    for f in calls:
        assert re.search(rf"\b{f}\s*\(", hdr), f"{f} not declared in include/yucsum.h"
        assert f in _lib.EXPORTS, f"{f} not in the library's export list"
        assert hasattr(_lib.lib(), f), f"{f} not exported by libyucsum.so"


def test_go_constants_are_defined():
    go, hdr = _go(), open(HDR).read()
    for c in set(re.findall(r"\bC\.(YU_\w+)\b", go)):
        assert re.search(rf"#define\s+{c}\b", hdr), f"{c} not defined in include/yucsum.h"
    for t in set(re.findall(r"\bC\.(yu_iovec)\b", go)):
        assert f"}} {t};" in hdr


@pytest.mark.parametrize("name", ["checksum.go", "batch.go", "packets_go121.go"])
def test_cgo_preamble_compiles_as_c(tmp_path, name):
    go = open(os.path.join(GODIR, name)).read()
    m = re.search(r"/\*\n(.*?)\*/\nimport \"C\"", go, re.S)
    assert m, "cgo preamble not found"
    pre = "\n".join(line for line in m.group(1).splitlines() if not line.startswith("#cgo"))
    src = tmp_path / "pre.c"
    src.write_text(pre + "\nint main(void) { return yu_abi_version() == YUCSUM_ABI_VERSION ? 0 : 1; }\n")
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-fsyntax-only",
                        f"-I{ROOT}/include", str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _func_body(go, name):
    m = re.search(rf"\nfunc {name}\(.*?\n}}\n", go, re.S)
    assert m, name
    return m.group(0)


def test_go_batch_calls_check_side_arrays_and_sizes():
    """Every Go batch entry point rejects initial / addrs slices shorter than the
    batch before the C call reads 2n / 8n bytes of them, passes side arrays only
    through sideArgs (no &initial[0] on an empty slice), and BatchHostUniform's data
    size check cannot wrap."""
    go = _go()
    side = _func_body(go, "checkSide")
    assert "uint64(len(initial)) < n" in side and "uint64(len(addrs))/8" in side
    for f in ("BatchHostUniform", "BatchHostRagged", "BatchHostPackets", "FillHostPackets"):
        body = _func_body(go, f)
        assert "checkSide(" in body, f
        assert "sideArgs(initial, addrs)" in body, f
        assert body.index("checkSide(") < body.index("C.yu_") if "C.yu_" in body else True, f
        assert "&initial[0]" not in body and "&addrs[0]" not in body, f
    uni = _func_body(go, "BatchHostUniform")
    assert "(n-1)*stride" not in uni.replace("// overflow-safe form of (n-1)*stride", "")
    assert "/(n-1)" in uni


def test_go_literal_constants_match_the_header(tmp_path):
    """HostContextPinnedMax is a plain integer literal in batch.go (no macro expression
    for cgo to evaluate): it must equal the header's
    YU_HOST_CONTEXT_PINNED_MAX + YU_HOST_BURST_CONTEXT_PINNED_MAX, as the C compiler
    evaluates them."""
    go = open(os.path.join(GODIR, "batch.go")).read()
    m = re.search(r"const HostContextPinnedMax uint64 = (\d+)\b", go)
    assert m, "HostContextPinnedMax is not a literal"
    src = tmp_path / "c.c"
    src.write_text('#include <stdio.h>\n#include "yucsum.h"\nint main(void) { printf("%llu", '
                   "(unsigned long long)(YU_HOST_CONTEXT_PINNED_MAX + YU_HOST_BURST_CONTEXT_PINNED_MAX)); }\n")
    exe = tmp_path / "c"
    subprocess.run(["gcc", f"-I{ROOT}/include", str(src), "-o", str(exe)], check=True)
    assert int(m.group(1)) == int(subprocess.run([str(exe)], capture_output=True, text=True).stdout)

"""Static checks of the cgo shim (bindings/go/checksum), which this image cannot
compile (no Go toolchain): every C function it calls is declared in include/yucsum.h
and exported by libyucsum.so, every C constant it names is defined there, and its cgo
preamble compiles as C against the header."""
import os
import re
import subprocess

from yustack_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "bindings", "go", "checksum", "checksum.go")
HDR = os.path.join(ROOT, "include", "yucsum.h")


def _go():
    return open(GO).read()


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


def test_cgo_preamble_compiles_as_c(tmp_path):
    go = _go()
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

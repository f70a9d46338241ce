"""The Go shim's own Go code, executed. bindings/go/checksum/checksum.go keeps the
reference's three signatures (checksum/checksum.go:4-35) and sums buffers under
256 bytes in Go (goSum), calling the C ABI only above that. There is no Go toolchain
here, so the file runs in tests/golden/goexec.py (the Go-subset interpreter the
fixture generator runs the reference's source with): every call below stays on the
pure-Go path and is compared with the oracle (oracle/oracle.py, checksum.go:4-35
restated). Parity unpinned by a real Go build; this pins the shim's Go-side logic
(odd tails, the uint32 accumulation, the combine, the pseudo header) against the
same oracle the GPU path is held to."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import goexec as G  # noqa: E402

from oracle import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def shim():
    it = G.Interp(os.path.join(ROOT, "bindings", "go"))
    it.load("checksum", files=["checksum.go"])
    return it


def test_checksum_short_buffers(shim):
    """Every length 0..255 (the Go side of the cgo cut), random bytes and initial
    values, plus all-0x00 / all-0xFF buffers (the one's-complement edge cases)."""
    rng = np.random.default_rng(2026)
    for n in range(256):
        for b in (bytes(rng.integers(0, 256, size=n, dtype=np.uint8)), b"\x00" * n, b"\xff" * n):
            init = int(rng.integers(0, 65536))
            for i in (0, init, 0xFFFF):
                got = shim.call("checksum", "Checksum", G.from_bytes(b), G.Int(i, "uint16")).v
                assert got == O.checksum(b, i), (n, b[:8], i)


def test_checksum_combine(shim):
    rng = np.random.default_rng(7)
    pairs = [(0, 0), (0xFFFF, 0xFFFF), (0xFFFF, 1), (1, 0xFFFF), (0x8000, 0x8000)]
    pairs += [tuple(int(x) for x in rng.integers(0, 65536, size=2)) for _ in range(500)]
    for a, b in pairs:
        got = shim.call("checksum", "ChecksumCombine", G.Int(a, "uint16"), G.Int(b, "uint16")).v
        assert got == O.checksum_combine(a, b), (a, b)


def test_pseudo_header_checksum(shim):
    """IPv4 addresses as Go strings (types/route.go:90-92 passes tcpip.Address values),
    protocols 6 / 17 and others; also odd-length strings, which Checksum's odd tail
    handles."""
    rng = np.random.default_rng(11)
    for k in range(300):
        n = 4 if k < 250 else int(rng.integers(0, 17))
        src = bytes(rng.integers(0, 256, size=n, dtype=np.uint8))
        dst = bytes(rng.integers(0, 256, size=n, dtype=np.uint8))
        proto = (6, 17, 1, 0, 255)[k % 5]
        got = shim.call("checksum", "PseudoHeaderChecksum", G.Int(proto, "uint32"), G.Str(src), G.Str(dst)).v
        assert got == O.pseudo_header_checksum(proto, src, dst), (proto, src, dst)

"""The Go shim's own Go code, executed. bindings/go/checksum keeps the reference's
three signatures (checksum/checksum.go:4-35), sums buffers under 256 bytes in Go
(goSum) and calls the C ABI for longer ones and for batches (batch.go). There is no Go
toolchain here, so the files run in tests/golden/goexec.py (the Go-subset interpreter
the fixture generator runs the reference's source with), with every `C.*` name bound
to libyucsum through ctypes: the shim's conversions, argument checks and status
mapping run as written, and its C calls reach the product library. Results are compared
with the oracle (oracle/oracle.py, checksum.go:4-35 and the senders restated).
Parity unpinned by a real Go build; this pins the shim's Go-side logic against the
same oracle the GPU path is held to. The batched calls need a GPU (`-m gpu` below);
without one the shim must map the library's YU_ENODEV to its ErrNoDevice."""
import ctypes
import os
import re
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import goexec as G  # noqa: E402

from oracle import oracle as O  # noqa: E402


class GoError:
    """An `error` value made by the errors.New / fmt.Errorf stubs."""

    def __init__(self, msg):
        self.msg = msg

    def __repr__(self):
        return f"error({self.msg!r})"


_CTYPES = {"uint8": np.uint8, "uint16": np.uint16, "uint32": np.uint32, "uint64": np.uint64,
           "int": np.int64, "int32": np.int32, "C.int": np.int32, "C.uint16_t": np.uint16,
           "C.uint64_t": np.uint64}


def _marshal(ref, keep, post):
    """A `&s[i]` handed to C: bytes in place (the slice's bytearray), other element
    types copied into a numpy array and, after the call, back into the Go slice."""
    s = ref.s
    if isinstance(s, G.Slice):
        cbuf = (ctypes.c_char * len(s.buf)).from_buffer(s.buf)
        keep.append(cbuf)
        return ctypes.addressof(cbuf) + s.off + ref.i
    et = s.t[2:]
    arr = np.array([x.v for x in s.items], dtype=_CTYPES[et])
    keep.append(arr)

    def back():
        for k in range(len(s.items)):
            s.items[k] = G.Int(int(arr[k]), s.items[k].t)
    post.append(back)
    return arr.ctypes.data + ref.i * arr.itemsize


def cgo_stubs():
    """The `C.*`, `unsafe`, `errors` and `fmt` names the shim uses: C types as integer
    conversions, C functions as ctypes calls into libyucsum, C constants from yucsum.h."""
    from yustack_amd import _lib
    L = _lib.lib()

    def cfunc(name):
        f = getattr(L, name)

        def call(*args):
            keep, post, cargs = [], [], []
            for a in args:
                if isinstance(a, G.Ref):
                    cargs.append(_marshal(a, keep, post))
                elif isinstance(a, G.Int):
                    cargs.append(a.v)
                else:
                    cargs.append(a)
            r = f(*cargs)
            for fn in post:
                fn()
            return G.Int(r, "int32") if isinstance(r, int) else r
        return call

    stubs = {"errors.New": lambda m: GoError(m.b.decode()),
             "fmt.Errorf": lambda f, *a: GoError(f.b.decode()),
             "unsafe.Pointer": lambda x: x,
             "C.GoString": lambda b: G.Str(b or b"")}
    for t, w in (("C.int", "int32"), ("C.uint64_t", "uint64"), ("C.uint32_t", "uint32"),
                 ("C.uint16_t", "uint16"), ("C.size_t", "uint64")):
        stubs[t] = (lambda w: lambda x: G.Int(x.v, w))(w)
    for name in _lib.EXPORTS:
        stubs["C." + name] = cfunc(name)
    hdr = open(os.path.join(ROOT, "include", "yucsum.h")).read()
    for nm, v in re.findall(r"#define (YU_\w+) \(?(-?(?:0x[0-9A-Fa-f]+|\d+))u?\)?\s", hdr):
        stubs["C." + nm] = G.Int(int(v, 0))
    return stubs


class FakeT:
    """A *testing.T for the shim's own Go tests: Fatal / Fatalf end the test."""

    def Fatal(self, *a):
        raise G.GoFatal(repr(a))

    def Fatalf(self, *a):
        raise G.GoFatal(repr(a))


def load_shim():
    it = G.Interp(os.path.join(ROOT, "bindings", "go"))
    it.stubs.update(cgo_stubs())
    it.load("checksum", files=["checksum.go", "batch.go", "checksum_test.go"])
    return it


@pytest.fixture(scope="module")
def shim():
    return load_shim()


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


def test_checksum_long_buffers_through_the_c_abi(shim):
    """Buffers of 256 bytes and more go through `C.yu_checksum` (the product's scalar
    drop-in) with the shim's pointer and size conversions; every result equals the
    oracle's, including the uint32 wrap past 131072 bytes."""
    rng = np.random.default_rng(5)
    for n in list(range(256, 300)) + [1499, 1500, 4096, 65535, 131072, 131073, 200001]:
        b = bytes(rng.integers(0, 256, size=n, dtype=np.uint8))
        i = int(rng.integers(0, 65536))
        assert shim.call("checksum", "Checksum", G.from_bytes(b), G.Int(i, "uint16")).v == O.checksum(b, i), n
    ff = b"\xff" * 131074
    assert shim.call("checksum", "Checksum", G.from_bytes(ff), G.Int(0xFFFF, "uint16")).v == 65534


def test_shim_go_tests(shim):
    """The shim's own Go tests that need no GPU and no goroutines: TestRFC1071 and
    TestShortArgumentsRejected (too-short side arrays, a wrapping size product and a
    length past the data are errors before any C call)."""
    for name in ("TestRFC1071", "TestShortArgumentsRejected"):
        shim.call("checksum", name, FakeT())


def test_batch_without_a_device_is_err_no_device(shim):
    """Valid batched calls reach the C ABI; with no HIP device it returns YU_ENODEV and
    the shim's status() maps it to the package's ErrNoDevice."""
    from yustack_amd import _lib
    if _lib.lib().yu_device_count() > 0:
        pytest.skip("a HIP device is visible (the GPU test below covers this path)")
    data = G.from_bytes(bytes(4 * 100))
    out = G.GoList([G.Int(0, "uint16")] * 4, "[]uint16")
    err = shim.call("checksum", "BatchHostUniform", data, G.Int(100, "uint64"), G.Int(100, "uint32"),
                    G.Int(4, "uint64"), G.Int(0, "Mode"), None, None, out, G.Int(0, "int"))
    assert err is shim.pkgs["checksum"].vars["ErrNoDevice"][3]
    assert shim.call("checksum", "HostContexts").v >= 1


@pytest.mark.gpu
def test_batch_calls_on_the_gpu(dev, oracle_c):
    """BatchHostUniform (sendTCP field values, address records) and BatchHostRagged
    (RAW with initial values, one shard and two) run through the interpreted shim into
    libyucsum on the GPU; the results it hands back in `out` equal the oracle's."""
    it = load_shim()
    rng = np.random.default_rng(21)
    n, L = 300, 1500
    data = rng.integers(0, 256, size=n * L, dtype=np.uint8)
    data.reshape(n, L)[:, 12] = 0x50
    addrs = rng.integers(0, 256, size=8 * n, dtype=np.uint8)
    want = oracle_c.batch(data, O.MODE_TCP, stride=L, length=L, n=n, addrs=addrs)
    out = G.GoList([G.Int(0, "uint16") for _ in range(n)], "[]uint16")
    err = it.call("checksum", "BatchHostUniform", G.from_bytes(data.tobytes()), G.Int(L, "uint64"),
                  G.Int(L, "uint32"), G.Int(n, "uint64"), G.Int(2, "Mode"), None,
                  G.from_bytes(addrs.tobytes()), out, G.Int(0, "int"))
    assert err is None, err
    assert [x.v for x in out.items] == [int(v) for v in want]

    lens = rng.integers(40, 1501, size=n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    rag = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    init = rng.integers(0, 65536, size=n, dtype=np.uint16)
    want = oracle_c.batch(rag, O.MODE_RAW, offsets=offs, initial_arr=init)
    for devices in ([], [G.Int(0, "int"), G.Int(0, "int")]):
        out = G.GoList([G.Int(0, "uint16") for _ in range(n)], "[]uint16")
        err = it.call("checksum", "BatchHostRagged", G.from_bytes(rag.tobytes()),
                      G.GoList([G.Int(int(o), "uint64") for o in offs], "[]uint64"), G.Int(0, "Mode"),
                      G.GoList([G.Int(int(v), "uint16") for v in init], "[]uint16"), None, out, *devices)
        assert err is None, err
        assert [x.v for x in out.items] == [int(v) for v in want], len(devices)


REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "checksum")), reason="the reference is not here")
def test_reference_callers_unchanged_on_shim():
    """north_star: header/ipv4.go, header/tcp.go and header/udp.go call the engine
    unchanged. The reference's own callers — sendUDP (transport/udp/endpoint.go:164-187),
    sendTCP / sendTCPWithOptions (transport/tcp/connect.go:556-586, :288-322),
    sendICMPv4 (network/ipv4/icmp.go:36-45) through types.Route and the ipv4 endpoint's
    WritePacket (network/ipv4/ipv4.go:80-97), the header methods (header/ipv4.go:177-179,
    header/tcp.go:165-173, header/udp.go:67-75) and checker.IPv4 / checker.TCP
    (checker/checker.go:25-40,71-99) — run from /root/reference as they are, with
    package checksum resolved to bindings/go/checksum (checksum.go, batch.go) and its
    `C.*` names bound to libyucsum. The fixture generator (tests/golden/make_refexec.py)
    runs on that interpreter with its seeded inputs: every stored field, every checker
    xsum and every Checksum / PseudoHeaderChecksum / ChecksumCombine vector must equal
    the committed refexec.json, which the same generator made with the reference's own
    checksum.go. Payloads of 256 bytes and more cross into C.yu_checksum (counted).
    Test infrastructure only (the interpreter reads the reference at run time): parity
    stays unpinned by a Go build."""
    import json
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import make_refexec as M
    it = G.load_path(REF, checksum=(os.path.join(ROOT, "bindings", "go", "checksum"), ["checksum.go", "batch.go"]))
    stubs = cgo_stubs()
    calls = {"yu_checksum": 0, "bytes": 0}
    inner = stubs["C.yu_checksum"]

    def counted(p, n, init):
        calls["yu_checksum"] += 1
        calls["bytes"] += n.v
        return inner(p, n, init)
    stubs["C.yu_checksum"] = counted
    it.stubs.update(stubs)
    # the package the callers resolve is the shim: its own helper exists, the reference's file is not loaded
    assert "goSum" in it.pkgs["checksum"].funcs and "BatchHostUniform" in it.pkgs["checksum"].funcs
    got = json.loads(json.dumps(M.build(M.Ref(it))))
    with open(os.path.join(ROOT, "tests", "golden", "refexec.json")) as f:
        want = json.load(f)
    assert got.keys() == want.keys()
    for key in want:
        if key == "modes":
            for mode, vecs in want["modes"].items():
                assert len(got["modes"][mode]) == len(vecs), mode
                bad = [i for i, (a, b) in enumerate(zip(got["modes"][mode], vecs)) if a != b]
                assert not bad, (mode, bad[:5], [got["modes"][mode][i] for i in bad[:2]], [vecs[i] for i in bad[:2]])
        else:
            assert got[key] == want[key], key
    n_exec = sum(1 for vecs in want["modes"].values() for v in vecs if v["src"] == "exec")
    print(f"{n_exec} executed-caller vectors on the shim; C.yu_checksum: {calls['yu_checksum']} calls, "
          f"{calls['bytes']} bytes")
    assert calls["yu_checksum"] > 100 and calls["bytes"] > 100_000, calls

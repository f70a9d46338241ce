"""The C-ABI boundary: the library loads, exports exactly what include/yucsum.h
declares, keeps the oracle out of the product, and fails loudly (a status, never a
CPU fallback) when no GPU is present. CPU only — no compute calls on a device."""
import ctypes
import os
import re
import subprocess

import pytest
import torch

from yustack_amd import _lib, batch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "yucsum.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(yu_[a-z0-9_]+)\s*\(", src)))


def exported_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_library_loads_and_exports_header():
    L = _lib.lib()
    decl = declared_functions()
    assert len(decl) >= 12
    exported = exported_symbols()
    for name in decl:
        assert name in exported, name
        assert hasattr(L, name)
    assert set(_lib.EXPORTS) == set(decl)
    assert L.yu_abi_version() == 1


def test_product_does_not_link_oracle():
    exported = exported_symbols()
    assert not any(s.startswith("or_") for s in exported)
    needed = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "oracle" not in needed
    assert "libamdhip64" in needed


def test_strerror():
    assert _lib.strerror(0) == "ok"
    assert _lib.strerror(-22) == "invalid argument"
    assert _lib.strerror(-19) == "no HIP device"


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_batched_entry_points_fail_without_gpu():
    L = _lib.lib()
    assert L.yu_device_count() == 0
    buf = (ctypes.c_uint8 * 64)()
    out = (ctypes.c_uint16 * 4)()
    rc = L.yu_csum_batch_uniform(ctypes.addressof(buf), 16, 16, 4, 0, None, 0, None, ctypes.addressof(out), None)
    assert rc == _lib.YU_ENODEV
    offs = (ctypes.c_uint64 * 5)(0, 16, 32, 48, 64)
    rc = L.yu_csum_batch_ragged(ctypes.addressof(buf), ctypes.addressof(offs), 4, 0, None, 0, None,
                                ctypes.addressof(out), None)
    assert rc == _lib.YU_ENODEV
    rc = L.yu_csum_batch_host_uniform(ctypes.addressof(buf), 16, 16, 4, 0, None, 0, None, ctypes.addressof(out), 0)
    assert rc == _lib.YU_ENODEV
    rc = L.yu_csum_batch_host_ragged(ctypes.addressof(buf), ctypes.addressof(offs), 4, 0, None, 0, None,
                                     ctypes.addressof(out), 0)
    assert rc == _lib.YU_ENODEV
    iov = (_lib.YuIovec * 4)(*[_lib.YuIovec(ctypes.addressof(buf) + 16 * i, 16) for i in range(4)])
    first = (ctypes.c_uint64 * 5)(0, 1, 2, 3, 4)
    rc = L.yu_csum_batch_host_iov(ctypes.addressof(iov), ctypes.addressof(first), 4, 8, None, 0, None,
                                  ctypes.addressof(out), 0)
    assert rc == _lib.YU_ENODEV
    devs = (ctypes.c_int * 2)(0, 0)
    pd = ctypes.addressof(devs)
    rc = L.yu_csum_batch_host_uniform_multi(ctypes.addressof(buf), 16, 16, 4, 0, None, 0, None,
                                            ctypes.addressof(out), pd, 2)
    assert rc == _lib.YU_ENODEV
    rc = L.yu_csum_batch_host_ragged_multi(ctypes.addressof(buf), ctypes.addressof(offs), 4, 0, None, 0,
                                           None, ctypes.addressof(out), pd, 2)
    assert rc == _lib.YU_ENODEV
    rc = L.yu_csum_batch_host_iov_multi(ctypes.addressof(iov), ctypes.addressof(first), 4, 8, None, 0, None,
                                        ctypes.addressof(out), pd, 2)
    assert rc == _lib.YU_ENODEV


def test_argument_validation_precedes_device():
    L = _lib.lib()
    buf = (ctypes.c_uint8 * 64)()
    out = (ctypes.c_uint16 * 4)()
    p, o = ctypes.addressof(buf), ctypes.addressof(out)
    assert L.yu_csum_batch_uniform(p, 16, 16, 4, 99, None, 0, None, o, None) == _lib.YU_EINVAL  # mode
    assert L.yu_csum_batch_uniform(p, 16, 16, 4, 0, None, 0, None, None, None) == _lib.YU_EINVAL  # out
    assert L.yu_csum_batch_uniform(p, 16, 70000, 4, 2, None, 0, None, o, None) == _lib.YU_EINVAL  # > 65535
    assert L.yu_csum_batch_uniform(p, 16, 4, 4, 1, None, 0, None, o, None) == _lib.YU_EINVAL  # < UDP header
    assert L.yu_csum_batch_uniform(p, 16, 0xFFFF0001, 1, 0, None, 0, None, o, None) == _lib.YU_EINVAL  # > YU_MAX_RAW_LEN
    assert L.yu_csum_batch_uniform(p, 16, 16, 0, 0, None, 0, None, o, None) == 0  # empty batch: no-op
    # (n-1)*stride + len past the end of the address space: rejected, not wrapped
    huge = 1 << 62
    assert L.yu_csum_batch_uniform(p, huge, 16, 5, 0, None, 0, None, o, None) == _lib.YU_EINVAL
    assert L.yu_csum_fill_uniform(p, huge, 16, 5, 1, None, 0, None, o, None) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_uniform(p, huge, 16, 5, 0, None, 0, None, o, 0) == _lib.YU_EINVAL
    assert L.yu_csum_fill_host_uniform(p, huge, 16, 5, 1, None, 0, None, o, 0) == _lib.YU_EINVAL
    devs1 = (ctypes.c_int * 1)(0)
    assert L.yu_csum_batch_host_uniform_multi(p, huge, 16, 5, 0, None, 0, None, o, ctypes.addressof(devs1),
                                              1) == _lib.YU_EINVAL
    assert L.yu_csum_fill_uniform(p, 16, 16, 4, 0, None, 0, None, o, None) == _lib.YU_EINVAL  # RAW not TX
    assert L.yu_csum_fill_uniform(p + 1, 16, 16, 4, 1, None, 0, None, o, None) == _lib.YU_EINVAL  # unaligned
    assert L.yu_csum_batch_ragged(p, None, 4, 0, None, 0, None, o, None) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_uniform(p, 16, 16, 4, 99, None, 0, None, o, 0) == _lib.YU_EINVAL
    for f in (L.yu_csum_fill_host_ragged, L.yu_csum_fill_host_iov):  # RAW / verify: not TX
        assert f(p, p, 4, 0, None, 0, None, o, 0) == _lib.YU_EINVAL
        assert f(p, p, 4, 6, None, 0, None, o, 0) == _lib.YU_EINVAL
    assert L.yu_csum_fill_host_uniform(p, 16, 16, 4, 0, None, 0, None, o, 0) == _lib.YU_EINVAL
    # host ragged / iov: offsets and views are host memory, checked before any device work
    bad = (ctypes.c_uint64 * 5)(0, 16, 8, 48, 64)  # decreasing
    assert L.yu_csum_batch_host_ragged(p, ctypes.addressof(bad), 4, 0, None, 0, None, o, 0) == _lib.YU_EINVAL
    big = (ctypes.c_uint64 * 2)(0, 70000)  # > 65535 in a transport mode
    assert L.yu_csum_batch_host_ragged(p, ctypes.addressof(big), 1, 2, None, 0, None, o, 0) == _lib.YU_EINVAL
    iov = (_lib.YuIovec * 2)(_lib.YuIovec(None, 5), _lib.YuIovec(p, 4))  # NULL view with bytes
    first = (ctypes.c_uint64 * 2)(0, 2)
    assert L.yu_csum_batch_host_iov(ctypes.addressof(iov), ctypes.addressof(first), 1, 0, None, 0, None,
                                    o, 0) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_iov(ctypes.addressof(iov), ctypes.addressof(first), 1, 10, None, 0, None,
                                    o, 0) == _lib.YU_EINVAL  # mode
    # view lengths whose sum wraps 64 bits to a small packet are refused, not summed
    huge = (_lib.YuIovec * 2)(_lib.YuIovec(p, 1 << 63), _lib.YuIovec(p, (1 << 63) + 4))
    assert L.yu_csum_batch_host_iov(ctypes.addressof(huge), ctypes.addressof(first), 1, 0, None, 0, None,
                                    o, 0) == _lib.YU_EINVAL
    # multi-GPU host calls: device list and batch checked before any device work
    devs = (ctypes.c_int * 2)(0, 0)
    pd = ctypes.addressof(devs)
    assert L.yu_csum_batch_host_uniform_multi(p, 16, 16, 4, 0, None, 0, None, o, None, 2) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_uniform_multi(p, 16, 16, 4, 0, None, 0, None, o, pd, 0) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_uniform_multi(p, 16, 16, 4, 0, None, 0, None, o, pd, 65) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_uniform_multi(p, 16, 70000, 4, 2, None, 0, None, o, pd, 2) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_uniform_multi(p, 16, 16, 0, 0, None, 0, None, o, pd, 2) == 0  # empty
    assert L.yu_csum_batch_host_ragged_multi(p, ctypes.addressof(bad), 4, 0, None, 0, None, o, pd,
                                             2) == _lib.YU_EINVAL
    assert L.yu_csum_batch_host_iov_multi(ctypes.addressof(iov), ctypes.addressof(first), 1, 0, None, 0,
                                          None, o, pd, 2) == _lib.YU_EINVAL


def test_python_front_end_refuses_cpu_tensors():
    d = torch.zeros(64, dtype=torch.uint8)
    with pytest.raises(TypeError):
        batch.checksum_uniform(d, 16, 16, 4, "raw")
    with pytest.raises(TypeError):
        batch.checksum_ragged(d, torch.zeros(5, dtype=torch.int64), "raw")
    with pytest.raises(ValueError):
        batch._mode(12)


@pytest.mark.parametrize("stride,length,mode,align,want", [
    (64, 64, "raw", 0, "k_lane<4>"),
    (64, 64, "udp", 0, "k_lane<4>"),         # TX field masked by subtraction
    (20, 20, "raw", 0, "k_lane<2>"),
    (8, 8, "udp", 0, "k_lane<2>"),           # strides up to 32 bytes
    (64, 20, "raw", 0, "k_tiny<4>"),         # sparse: k_lane would load 3x the bytes
    (64, 64, "udp", 1, "k_seg<4,tx>"),       # unaligned dense: the segmented stream sum
    (128, 120, "verify_tcp", 0, "k_tiny<8>"),   # > 112 bytes: every k_tiny<8> lane loads
    (128, 100, "raw", 0, "k_lane<8>"),          # 64 whole strides per wave step in LDS
    (100, 100, "tcp", 0, "k_lane<7>"),
    (72, 72, "udp", 0, "k_lane<5>"),            # sendUDP datagram: 8-B header + 64-B payload
    (72, 70, "raw", 2, "k_seg<4>"),             # unaligned: no k_lane
    (256, 70, "raw", 2, "k_small<8,1>"),        # unaligned and sparse
    (136, 128, "raw", 0, "k_tiny<8>"),          # stride > 128: no k_lane
    (1500, 1500, "tcp", 0, "k_small<16,6>"),
    (1500, 1500, "tcp", 2, "k_small<16,6>"),     # 1503 still fits 1536
    (1536, 1536, "raw", 1, "k_small<32,4>"),     # 1539 > 1536
    (9000, 9000, "raw", 0, "k_seg<8>"),          # dense > 3 KiB in a large batch
    (20000, 9000, "raw", 0, "k_loop<4,LE>"),     # sparse: a wave per packet
    (400000, 200000, "raw", 0, "k_loop<4,BE>"),  # sparse, > 131072: exact uint32 wrap path
    (1500, 1500, "ipv4", 0, "k_hdr"),            # only the <= 60-byte header is read
    (20, 20, "udp", 3, "k_seg<4,tx>"),
    (320, 320, "tcp", 0, "k_seg<4,tx>"),        # 129..704 B dense
    (512, 512, "raw", 0, "k_seg<8>"),
    (62, 62, "raw", 1, "k_seg<4>"),
    (200, 62, "raw", 1, "k_small<8,1>"),     # sparse: 65 > 64
])
def test_variant_selection(stride, length, mode, align, want):
    assert batch.variant(stride, length, mode, align, n=1 << 20) == want


@pytest.mark.parametrize("stride,length,n,want", [
    (9000, 9000, 1 << 20, "k_seg<8>"),      # dense > 3 KiB, enough chunks for the GPU
    (9000, 9000, 1000, "k_loop<4,LE>"),     # a few huge packets: a wave per packet
    (320, 320, 1000, "k_small<16,2>"),       # small batches keep per-packet lane groups
    (320, 320, 1 << 20, "k_seg<4>"),
    (66, 66, 1000, "k_small<8,1>"),          # unaligned, small batch
    (200000, 200000, 1 << 17, "k_seg<8>"),  # > 131072: k_seg's exact byte-sum path
    (20000, 9000, 1 << 20, "k_loop<4,LE>"),  # sparse
])
def test_variant_selection_by_batch_size(stride, length, n, want):
    assert batch.variant(stride, length, "raw", 0, n=n) == want


# k_seg's TX / RX / DG kinds keep positions in 32 bits: 63 strides plus a 65535-byte
# packet and its 3 head bytes must stay under 2 GiB (kSeg32Stride in yucsum_kernels.hip)
SEG32_STRIDE = ((1 << 31) - 65535 - 3) // 63


@pytest.mark.parametrize("mode,kern,loop", [("verify_rx", "k_seg<8,rx>", "k_loop<4,rx>"),
                                             ("tx_datagram", "k_seg<8,dg>", "k_loop<4,dg>")])
def test_sparse_datagram_batches_leave_k_seg(mode, kern, loop):
    """Uniform VERIFY_RX / TX_DATAGRAM batches whose 64-packet chunk could span 2 GiB
    take a wave per datagram instead (a GPU run at that size would need > 100 GB)."""
    n = 1 << 20
    assert batch.variant(1500, 1500, mode, 0, n=n) == kern
    assert batch.variant(SEG32_STRIDE, 1500, mode, 0, n=n) == kern
    assert batch.variant(SEG32_STRIDE + 1, 1500, mode, 0, n=n) == loop


_KNOB_PROBE = (
    "import sys; sys.path.insert(0, %r)\n"
    "from yustack_amd import _lib\n"
    "L = _lib.lib()\n"
    "print(L.yu_ragged_variant_n(0, 1 << 20).decode(), L.yu_uniform_variant_n(1500, 1500, 1 << 20, 2, 0).decode(),\n"
    "      L.yu_ragged_fill_variant_n(1, 1 << 20).decode())\n" % ROOT)


def _variants_under(env_extra):
    env = {k: v for k, v in os.environ.items() if not k.startswith("YU_")}
    env.update(env_extra)
    r = subprocess.run([__import__("sys").executable, "-c", _KNOB_PROBE], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return r.stdout.split(), r.stderr


def test_tuning_knobs_need_the_gate():
    """The measurement knobs (YU_RAGGED, YU_VARIANT, YU_FILL_WB, ...) change the
    kernel choice only when YU_TUNING=1 is set too; an inherited knob alone leaves
    the library's own choice (the reference's whole config surface
    is two package variables, link/tundev/tundev.go:20 and link/sniffer/sniffer.go:14)."""
    knobs = {"YU_RAGGED": "loop", "YU_VARIANT": "k_small<32,4>", "YU_FILL_WB": "0", "YU_NT": "1"}
    default, err0 = _variants_under({})
    assert default == ["k_seg<8>", "k_small<16,6>", "k_seg<8,txw,c48>"]
    inherited, err1 = _variants_under(knobs)
    assert inherited == default and "tuning knob" not in err1
    for bad_gate in ("0", "yes", "11", ""):
        assert _variants_under(dict(knobs, YU_TUNING=bad_gate))[0] == default
    tuned, err2 = _variants_under(dict(knobs, YU_TUNING="1"))
    assert tuned == ["k_loop<4,BE>", "k_small<32,4>", "k_loop<4,LE>"]
    # the open gate names each knob it reads
    assert "tuning knob YU_RAGGED=loop" in err2 and "tuning knob YU_VARIANT=k_small<32,4>" in err2
    # YU_FILL_WB alone (no forced ragged kernel): the TX kind instead of TXW
    assert _variants_under({"YU_TUNING": "1", "YU_FILL_WB": "0"})[0][2] == "k_seg<8,tx>"


SOURCES = [os.path.join(ROOT, "yustack_amd", "csrc", f) for f in ("yucsum_kernels.hip", "yucsum_host.cpp",
                                                                  "yucsum_scalar.cpp")]


def _header_einval_tags():
    src = open(HEADER).read()
    block = src[src.index("Preconditions: every YU_EINVAL"):src.index("Where the writers differ")]
    return set(re.findall(r"/\*\s+\[([a-z-]+)\]", block))


def test_every_einval_is_documented():
    """Static check: each `return YU_EINVAL` in the library
    carries an `EINVAL:<tag>` comment, every tag is one include/yucsum.h's
    Preconditions list documents, and every documented tag is used."""
    documented = _header_einval_tags()
    assert len(documented) >= 14, documented
    used = set()
    for path in SOURCES:
        lines = open(path).read().splitlines()
        for k, line in enumerate(lines):
            if "return YU_EINVAL" not in line:
                continue
            m = re.search(r"EINVAL:([a-z-]+(?: / [a-z-]+)*)", line)
            assert m, f"{os.path.basename(path)}:{k + 1}: untagged YU_EINVAL: {line.strip()}"
            for tag in m.group(1).split(" / "):
                assert tag in documented, f"{os.path.basename(path)}:{k + 1}: [{tag}] not in yucsum.h"
                used.add(tag)
    assert used == documented, documented ^ used


def test_each_documented_einval_is_returned():
    """One call per documented precondition, each returning YU_EINVAL before any
    device work (so on this GPU-less host too); plus the cases the header states
    are NOT errors (an unaligned ragged fill, NULL out in a fill call), which get
    past validation and stop at the missing device."""
    L = _lib.lib()
    EINVAL = _lib.YU_EINVAL
    buf = (ctypes.c_uint8 * 256)()
    out = (ctypes.c_uint16 * 8)()
    p, o = ctypes.addressof(buf), ctypes.addressof(out)
    offs = (ctypes.c_uint64 * 5)(0, 16, 32, 48, 64)
    po = ctypes.addressof(offs)
    dec = (ctypes.c_uint64 * 5)(0, 16, 8, 48, 64)
    iov = (_lib.YuIovec * 4)(*[_lib.YuIovec(p + 16 * i, 16) for i in range(4)])
    first = (ctypes.c_uint64 * 5)(0, 1, 2, 3, 4)
    devs = (ctypes.c_int * 2)(0, 0)
    pd = ctypes.addressof(devs)
    cases = {
        "mode": [L.yu_csum_batch_uniform(p, 16, 16, 4, YU_MODE_COUNT, None, 0, None, o, None),
                 L.yu_csum_batch_ragged(p, po, 4, -1, None, 0, None, o, None),
                 L.yu_csum_batch_host_ragged(p, po, 4, 10, None, 0, None, o, 0),
                 L.yu_csum_batch_host_iov_multi(ctypes.addressof(iov), ctypes.addressof(first), 4, 99, None, 0,
                                                None, o, pd, 2)],
        "out": [L.yu_csum_batch_ragged(p, po, 4, 0, None, 0, None, None, None),
                L.yu_csum_batch_host_uniform(p, 16, 16, 4, 0, None, 0, None, None, 0)],
        "fill-mode": [L.yu_csum_fill_uniform(p, 16, 16, 4, 0, None, 0, None, o, None),  # RAW
                      L.yu_csum_fill_ragged(p, po, 4, 8, None, 0, None, o, None),        # VERIFY_RX
                      L.yu_csum_fill_host_ragged(p, po, 4, 5, None, 0, None, o, 0)],     # VERIFY_IPV4
        "side-align": [L.yu_csum_batch_uniform(p, 16, 16, 4, 0, p + 1, 0, None, o, None),
                       L.yu_csum_batch_uniform(p, 16, 16, 4, 1, None, 0, p + 2, o, None),
                       L.yu_csum_batch_ragged(p, po, 4, 0, None, 0, None, o + 1, None)],
        "data": [L.yu_csum_batch_uniform(None, 16, 16, 4, 0, None, 0, None, o, None),
                 L.yu_csum_batch_ragged(None, po, 4, 0, None, 0, None, o, None),
                 L.yu_csum_batch_host_uniform(None, 16, 16, 4, 0, None, 0, None, o, 0),
                 L.yu_csum_batch_host_ragged(None, po, 4, 0, None, 0, None, o, 0)],
        "len-transport": [L.yu_csum_batch_uniform(p, 16, 65536, 1, 2, None, 0, None, o, None),
                          L.yu_csum_batch_host_uniform(p, 16, 65536, 1, 1, None, 0, None, o, 0)],
        "len-raw": [L.yu_csum_batch_uniform(p, 16, 0xFFFF0001, 1, 0, None, 0, None, o, None)],
        "len-min": [L.yu_csum_batch_uniform(p, 16, 7, 4, 1, None, 0, None, o, None),    # UDP < 8
                    L.yu_csum_batch_uniform(p, 32, 19, 4, 2, None, 0, None, o, None),   # TCP < 20
                    L.yu_csum_batch_uniform(p, 16, 3, 4, 4, None, 0, None, o, None),    # ICMP < 4
                    L.yu_csum_batch_uniform(p, 16, 0, 4, 3, None, 0, None, o, None)],   # IPv4: no IHL byte
        "span": [L.yu_csum_batch_uniform(p, 1 << 62, 16, 5, 0, None, 0, None, o, None)],
        "offsets": [L.yu_csum_batch_ragged(p, None, 4, 0, None, 0, None, o, None),
                    L.yu_csum_batch_ragged(p, po + 4, 4, 0, None, 0, None, o, None),
                    L.yu_csum_batch_host_ragged(p, ctypes.addressof(dec), 4, 0, None, 0, None, o, 0),
                    L.yu_csum_batch_host_iov(ctypes.addressof(iov), None, 4, 0, None, 0, None, o, 0)],
        "iov-view": [L.yu_csum_batch_host_iov(None, ctypes.addressof(first), 4, 0, None, 0, None, o, 0)],
        "fill-align": [L.yu_csum_fill_uniform(p + 2, 16, 16, 4, 1, None, 0, None, o, None),
                       L.yu_csum_fill_uniform(p, 18, 16, 4, 1, None, 0, None, o, None)],
        "fill-overlap": [L.yu_csum_fill_uniform(p, 16, 20, 4, 1, None, 0, None, o, None)],
        "devices": [L.yu_csum_batch_host_uniform_multi(p, 16, 16, 4, 0, None, 0, None, o, None, 2),
                    L.yu_csum_batch_host_ragged_multi(p, po, 4, 0, None, 0, None, o, pd, 0),
                    L.yu_csum_batch_host_iov_multi(ctypes.addressof(iov), ctypes.addressof(first), 4, 0, None,
                                                   0, None, o, pd, 65)],
    }
    assert set(cases) == _header_einval_tags()
    # an empty batch is a no-op, NULL results array included (before any device)
    pd1 = ctypes.addressof((ctypes.c_int * 1)(0))
    assert L.yu_csum_batch_uniform(p, 16, 16, 0, 0, None, 0, None, None, None) == 0
    assert L.yu_csum_batch_ragged(p, po, 0, 1, None, 0, None, None, None) == 0
    assert L.yu_csum_batch_host_uniform(p, 16, 16, 0, 0, None, 0, None, None, 0) == 0
    assert L.yu_csum_batch_host_ragged(p, po, 0, 0, None, 0, None, None, 0) == 0
    assert L.yu_csum_batch_host_iov(ctypes.addressof(iov), ctypes.addressof(first), 0, 0, None, 0, None,
                                    None, 0) == 0
    assert L.yu_csum_batch_host_uniform_multi(p, 16, 16, 0, 0, None, 0, None, None, pd1, 1) == 0
    for tag, rcs in cases.items():
        assert all(rc == EINVAL for rc in rcs), (tag, rcs)
    if not torch.cuda.is_available():
        # documented as accepted: they pass validation and stop at the missing device
        nodev = _lib.YU_ENODEV
        uo = (ctypes.c_uint64 * 5)(1, 18, 33, 51, 64)  # odd offsets
        assert L.yu_csum_fill_ragged(p + 1, ctypes.addressof(uo), 4, 1, None, 0, None, None, None) == nodev
        assert L.yu_csum_fill_ragged(p + 3, po, 4, 9, None, 0, None, o, None) == nodev
        assert L.yu_csum_fill_host_ragged(p + 1, ctypes.addressof(uo), 4, 1, None, 0, None, None, 0) == nodev


YU_MODE_COUNT = 10


def test_host_staging_pool_bound_and_setting():
    """The host path's context pool (include/yucsum.h, Host-path staging): K from
    YU_HOST_CONTEXTS (default 4, clamped to 1..64, read without the tuning gate), no
    staging before a first call (or after a trim), the per-context bounds as the header
    states them."""
    L = _lib.lib()
    if L.yu_device_count() > 0:  # (on a GPU box earlier tests of this process may hold staging)
        assert L.yu_host_staging_trim(0) == 0
    assert L.yu_host_staging_bytes(0, None) == 0 and L.yu_host_staging_bytes(-1, None) == 0
    assert L.yu_host_staging_trim(64) == _lib.YU_ENODEV
    src = open(HEADER).read()
    assert "#define YU_HOST_SLICE_BYTES (32ull << 20)" in src and "#define YU_HOST_SLICE_PACKETS (1ull << 18)" in src
    assert _lib.HOST_CONTEXT_PINNED_MAX == 3 * ((32 << 20) + 26 * (1 << 18) + 72)  # ~115.5 MiB
    assert _lib.HOST_BURST_CONTEXT_PINNED_MAX == (4 << 20) + 26 * (1 << 18) + 72  # ~10.5 MiB, one slot
    assert _lib.HOST_BURST_CONTEXT_DEVICE_MAX == (4 << 20) + 22 * (1 << 18) + 8
    probe = f"import sys; sys.path.insert(0, {ROOT!r}); from yustack_amd import _lib; print(_lib.lib().yu_host_contexts())"
    for val, want in ((None, 4), ("2", 2), ("0", 1), ("100", 64), ("junk", 4)):
        env = {k: v for k, v in os.environ.items() if not k.startswith("YU_")}
        if val is not None:
            env["YU_HOST_CONTEXTS"] = val
        r = subprocess.run([__import__("sys").executable, "-c", probe], env=env, capture_output=True, text=True,
                           timeout=60)
        assert r.returncode == 0 and int(r.stdout) == want, (val, r.stdout, r.stderr)


_ORDER = r"""
import sys
sys.path.insert(0, %r)
from yustack_amd import _lib
n = _lib.lib().yu_device_count()
import torch
print(n, torch.cuda.is_available())
"""


@pytest.mark.gpu
def test_library_first_then_torch_share_the_device():
    """PyTorch-ROCm bundles its own HIP runtime; the library binds /opt/rocm's. When the
    library initialised its runtime first, torch's saw no device (and the other way
    round: profiles/r05/load_order_r05.log). The loader now brings torch's in first, so
    a process that calls the library before touching torch still has both."""
    r = subprocess.run([__import__("sys").executable, "-c", _ORDER % ROOT], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    n, ok = r.stdout.split()
    assert int(n) >= 1 and ok == "True", r.stdout


_MISORDERED = r"""
import ctypes, sys
sys.path.insert(0, %r)
ctypes.CDLL(%r)          # a user program loads the library by ctypes first ...
import torch             # ... and torch (with its own HIP runtime) after it
from yustack_amd import _lib
try:
    _lib.lib()
except ImportError as e:
    print("refused:", e)
    sys.exit(0)
print("loaded", _lib.lib().yu_hip_runtime_path())
sys.exit(3)
"""

_ORDERED = r"""
import sys
sys.path.insert(0, %r)
from yustack_amd import _lib
L = _lib.lib()
import os
print(os.path.realpath(L.yu_hip_runtime_path().decode()), os.path.realpath(_lib.torch_hip_runtime() or ""))
"""


def test_runtime_binding_is_checked_at_load():
    """the loader checks which HIP runtime the library's calls are
    bound to (yu_hip_runtime_path, dladdr of its own hipGetDevice reference). Through
    the loader (torch first) it is torch's bundled runtime; a library loaded by ctypes
    before torch is bound to /opt/rocm's, and the loader refuses it with an ImportError
    that names the fix, instead of a later silent "no device". No GPU needed: binding
    happens at load time."""
    import sys
    r = subprocess.run([sys.executable, "-c", _ORDERED % ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    ours, theirs = r.stdout.split()
    if theirs == os.path.realpath(""):  # a torch that uses the system runtime: nothing to check
        pytest.skip("torch bundles no HIP runtime here")
    assert ours == theirs
    r = subprocess.run([sys.executable, "-c", _MISORDERED % (ROOT, _lib.LIB_PATH)], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, (r.stdout, r.stderr[-2000:])
    assert "refused:" in r.stdout and "import torch" in r.stdout and "/opt/rocm" in r.stdout, r.stdout

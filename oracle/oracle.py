"""TEST INFRASTRUCTURE ONLY — parity checker for the yustack_amd checksum engine.

Two independent CPU restatements of yustack's checksum path
(/root/reference/checksum/checksum.go and its call sites):

* ``C`` — ctypes binding of ``oracle/csum_oracle.c`` (built by ``oracle/Makefile``
  into ``oracle/build/libcsum_oracle.so``), used for large batches and as the
  cpu_baseline in bench.py;
* the pure-Python twin below, used for small cases and fixture generation.

Only ``tests/``, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg may
import this module. The product package ``yustack_amd`` never does.

PARITY UNPINNED (by the task's rule): the reference is Go (no
toolchain in this image) and ships no known-answer vectors, so it cannot pin this
oracle. The evidence it rests on instead: known answers produced by executing the
reference's own source (checksum/checksum.go, header/{ipv4,tcp,udp}.go) with the
Go-subset interpreter tests/golden/goexec.py (tests/golden/refexec.json; the
interpreter is this repo's stand-in for the absent toolchain), RFC 1071 §3's published
example, the reference's own test-side property (checker/checker.go:32-35,80-92) on
packets built the way its test harnesses build them, agreement of the two independent
restatements plus the closed form, and datagrams the Linux kernel verified or built
(tests/golden/kernel_verified.npz).
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libcsum_oracle.so")

MODE_RAW, MODE_UDP, MODE_TCP, MODE_IPV4, MODE_ICMP = 0, 1, 2, 3, 4
MODE_VERIFY_IPV4, MODE_VERIFY_TCP, MODE_VERIFY_UDP, MODE_VERIFY_RX = 5, 6, 7, 8
MODE_TX_DATAGRAM = 9
MODE_NAMES = {
    MODE_RAW: "raw", MODE_UDP: "udp", MODE_TCP: "tcp", MODE_IPV4: "ipv4",
    MODE_ICMP: "icmp", MODE_VERIFY_IPV4: "verify_ipv4",
    MODE_VERIFY_TCP: "verify_tcp", MODE_VERIFY_UDP: "verify_udp",
    MODE_VERIFY_RX: "verify_rx", MODE_TX_DATAGRAM: "tx_datagram",
}


def outputs(mode: int) -> int:
    """Results per packet (include/yucsum.h YU_MODE_OUTPUTS)."""
    return 2 if mode == MODE_TX_DATAGRAM else 1
RX_IP_OK, RX_L4, RX_L4_OK, RX_INVALID = 1, 2, 4, 8  # include/yucsum.h YU_RX_*


# --------------------------------------------------------------------------
# Pure-Python twin (literal restatement of the Go code)
# --------------------------------------------------------------------------
def checksum_combine(a: int, b: int) -> int:
    """checksum/checksum.go:32-35"""
    v = (a + b) & 0xFFFFFFFF
    return (v + (v >> 16)) & 0xFFFF


def checksum(buf: bytes, initial: int) -> int:
    """checksum/checksum.go:4-18 (uint32 accumulator, wraps mod 2^32)."""
    v = initial & 0xFFFF
    l = len(buf)
    if l & 1:
        l -= 1
        v = (v + (buf[l] << 8)) & 0xFFFFFFFF
    # the even-length loop, vectorised with numpy but with identical arithmetic
    if l:
        a = np.frombuffer(bytes(buf[:l]), dtype=np.uint8).astype(np.uint64)
        s = int((a[0::2] * 256 + a[1::2]).sum())
        v = (v + s) & 0xFFFFFFFF
    return checksum_combine(v & 0xFFFF, v >> 16)


def checksum_loop(buf: bytes, initial: int) -> int:
    """checksum/checksum.go:4-18 as a literal per-pair loop (small inputs)."""
    v = initial & 0xFFFF
    l = len(buf)
    if l & 1:
        l -= 1
        v = (v + (buf[l] << 8)) & 0xFFFFFFFF
    for i in range(0, l, 2):
        v = (v + (buf[i] << 8) + buf[i + 1]) & 0xFFFFFFFF
    return checksum_combine(v & 0xFFFF, v >> 16)


def checksum_closed_form(buf: bytes, initial: int) -> int:
    """Closed form of A1 for len <= 131072: S = initial + sum of
    big-endian words; result 0 iff S == 0, else ((S-1) mod 65535) + 1."""
    assert len(buf) <= 131072
    b = bytes(buf) + (b"\0" if len(buf) & 1 else b"")
    a = np.frombuffer(b, dtype=np.uint8).astype(np.uint64)
    s = int((a[0::2] * 256 + a[1::2]).sum()) + (initial & 0xFFFF) if len(b) else (initial & 0xFFFF)
    return 0 if s == 0 else ((s - 1) % 65535) + 1


def pseudo_header_checksum(protocol: int, src: bytes, dst: bytes) -> int:
    """checksum/checksum.go:24-28"""
    x = checksum(src, 0)
    x = checksum(dst, x)
    return checksum(bytes([0, protocol & 0xFF]), x)


def udp_calculate_checksum(udp: bytes, partial: int, total_length: int) -> int:
    """header/udp.go:67-75"""
    c = checksum(struct.pack(">H", total_length & 0xFFFF), partial)
    return checksum(bytes(udp[:8]), c)


def tcp_calculate_checksum(tcp: bytes, partial: int, total_len: int) -> int:
    """header/tcp.go:165-173"""
    c = checksum(struct.pack(">H", total_len & 0xFFFF), partial)
    doff = (tcp[12] >> 4) * 4
    return checksum(bytes(tcp[:doff]), c)


def ipv4_calculate_checksum(ip: bytes) -> int:
    """header/ipv4.go:177-179 (HeaderLength header/ipv4.go:91-93)"""
    hl = (ip[0] & 0xF) * 4
    return checksum(bytes(ip[:hl]), 0)


def _pseudo(proto, addrs, initial_arr, initial, p):
    if addrs is not None:
        a = bytes(addrs[8 * p: 8 * p + 8])
        return pseudo_header_checksum(proto, a[:4], a[4:])
    return int(initial_arr[p]) if initial_arr is not None else initial


def packet(mode: int, pkt: bytes, initial_arr=None, initial: int = 0, addrs=None, p: int = 0) -> int:
    """One packet of a batch, composed as the reference call sites do (see
    csum_oracle.c or_packet for the citations)."""
    pkt = bytes(pkt)
    if mode == MODE_RAW:
        init = int(initial_arr[p]) if initial_arr is not None else initial
        return checksum(pkt, init)
    if mode == MODE_UDP:  # transport/udp/endpoint.go:164-187
        hdr = bytearray(pkt[:8]); hdr[6:8] = b"\0\0"
        xsum = _pseudo(17, addrs, initial_arr, initial, p)
        data = pkt[8:]
        length = (8 + len(data)) & 0xFFFF
        xsum = checksum(data, xsum)
        return ~udp_calculate_checksum(bytes(hdr), xsum, length) & 0xFFFF
    if mode == MODE_TCP:  # transport/tcp/connect.go:556-586
        doff = (pkt[12] >> 4) * 4
        hdr = bytearray(pkt[:doff]); hdr[16:18] = b"\0\0"
        xsum = _pseudo(6, addrs, initial_arr, initial, p)
        data = pkt[doff:]
        length = (doff + len(data)) & 0xFFFF
        xsum = checksum(data, xsum)
        return ~tcp_calculate_checksum(bytes(hdr), xsum, length) & 0xFFFF
    if mode == MODE_IPV4:  # network/ipv4/ipv4.go:80-97
        hdr = bytearray(pkt[:64])  # the packet as Encode left it (field 0)
        if len(hdr) >= 12:
            hdr[10:12] = b"\0\0"
        return ~ipv4_calculate_checksum(bytes(hdr)) & 0xFFFF
    if mode == MODE_ICMP:  # network/ipv4/icmp.go:36-45
        hdr = bytearray(pkt[:4]); hdr[2:4] = b"\0\0"
        return ~checksum(bytes(hdr), checksum(pkt[4:], 0)) & 0xFFFF
    if mode == MODE_VERIFY_IPV4:  # checker/checker.go:32
        return ipv4_calculate_checksum(pkt)
    if mode in (MODE_VERIFY_TCP, MODE_VERIFY_UDP):  # checker/checker.go:80-88
        proto = 6 if mode == MODE_VERIFY_TCP else 17
        l = len(pkt) & 0xFFFF
        xsum = _pseudo(proto, addrs, initial_arr, initial, p)
        xsum = checksum(bytes([l >> 8, l & 0xFF]), xsum)
        return checksum(pkt, xsum)
    if mode == MODE_VERIFY_RX:  # checker/checker.go:25-40,71-92 on a received packet
        if len(pkt) < 20:
            return RX_INVALID
        hl = (pkt[0] & 0xF) * 4
        tl = (pkt[2] << 8) | pkt[3]
        if hl > tl or tl > len(pkt):
            return RX_INVALID
        r = 0
        if ipv4_calculate_checksum(pkt) in (0, 0xFFFF):
            r |= RX_IP_OK
        proto = pkt[9]
        if proto in (1, 6, 17):
            r |= RX_L4
            payload = pkt[hl:tl]
            if proto == 1:
                xs = checksum(payload, 0)
            else:
                xs = pseudo_header_checksum(proto, pkt[12:16], pkt[16:20])
                xs = checksum(bytes([(len(payload) >> 8) & 0xFF, len(payload) & 0xFF]), xs)
                xs = checksum(payload, xs)
            if xs in (0, 0xFFFF):
                r |= RX_L4_OK
        return r
    raise ValueError(f"bad mode {mode}")


def _one(mode, pkt, initial_arr, initial, addrs, p):
    if mode == MODE_TX_DATAGRAM:
        return list(tx_datagram(pkt))
    return [packet(mode, pkt, initial_arr, initial, addrs, p)]


def batch_uniform_py(data, stride, length, n, mode, initial_arr=None, initial=0, addrs=None):
    data = bytes(data)
    return np.array([v for p in range(n)
                     for v in _one(mode, data[p * stride: p * stride + length], initial_arr, initial, addrs, p)],
                    dtype=np.uint16)


def batch_ragged_py(data, offsets, mode, initial_arr=None, initial=0, addrs=None):
    data = bytes(data)
    n = len(offsets) - 1
    return np.array([v for p in range(n)
                     for v in _one(mode, data[int(offsets[p]): int(offsets[p + 1])], initial_arr, initial,
                                   addrs, p)], dtype=np.uint16)


# --------------------------------------------------------------------------
# C restatement (ctypes)
# --------------------------------------------------------------------------
def tx_datagram(pkt: bytes) -> tuple[int, int]:
    """YU_MODE_TX_DATAGRAM (include/yucsum.h): the IPv4 header field WritePacket
    stores (network/ipv4/ipv4.go:80-97) and the transport field its sender stores
    (transport/udp/endpoint.go:164-187, transport/tcp/connect.go:556-586,
    network/ipv4/icmp.go:36-45) for a whole outgoing datagram, the pseudo header
    from its own addresses; (0, 0) outside 20 <= HeaderLength <= TotalLength <= len."""
    pkt = bytes(pkt)
    if len(pkt) < 20:
        return 0, 0
    hl = (pkt[0] & 0xF) * 4
    tl = (pkt[2] << 8) | pkt[3]
    if hl < 20 or hl > tl or tl > len(pkt):
        return 0, 0
    ip = packet(MODE_IPV4, pkt)
    seg, rec, proto = pkt[hl:tl], np.frombuffer(pkt[12:20], np.uint8), pkt[9]
    l4 = 0
    if proto == 17 and len(seg) >= 8:
        l4 = packet(MODE_UDP, seg, addrs=rec)
    elif proto == 6 and len(seg) >= 20:
        l4 = packet(MODE_TCP, seg, addrs=rec)
    elif proto == 1 and len(seg) >= 4:
        l4 = packet(MODE_ICMP, seg)
    return ip, l4


class _C:
    def __init__(self, path: str = LIB_PATH):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        lib = ctypes.CDLL(path)
        u8p, u16p, u64p = (ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_uint16),
                           ctypes.POINTER(ctypes.c_uint64))
        lib.or_checksum.restype = ctypes.c_uint16
        lib.or_checksum.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint16]
        lib.or_checksum_combine.restype = ctypes.c_uint16
        lib.or_checksum_combine.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
        lib.or_pseudo_header_checksum.restype = ctypes.c_uint16
        lib.or_pseudo_header_checksum.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                                  ctypes.c_void_p, ctypes.c_size_t]
        lib.or_batch_mt.restype = ctypes.c_int
        lib.or_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                    ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint16,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        del u8p, u16p, u64p
        self.lib = lib

    def checksum(self, buf: bytes, initial: int) -> int:
        b = bytes(buf)
        return self.lib.or_checksum(b, len(b), initial & 0xFFFF)

    def combine(self, a: int, b: int) -> int:
        return self.lib.or_checksum_combine(a, b)

    def pseudo_header_checksum(self, proto: int, src: bytes, dst: bytes) -> int:
        return self.lib.or_pseudo_header_checksum(proto, bytes(src), len(src), bytes(dst), len(dst))

    def batch(self, data: np.ndarray, mode: int, *, stride: int = 0, length: int = 0, n: int | None = None,
              offsets: np.ndarray | None = None, initial_arr: np.ndarray | None = None, initial: int = 0,
              addrs: np.ndarray | None = None, threads: int = 1) -> np.ndarray:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        if offsets is not None:
            offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
            n = len(offsets) - 1
        assert n is not None
        k = outputs(mode)
        out = np.zeros(max(n * k, 1), dtype=np.uint16)
        ia = None if initial_arr is None else np.ascontiguousarray(initial_arr, dtype=np.uint16)
        ad = None if addrs is None else np.ascontiguousarray(addrs, dtype=np.uint8)
        rc = self.lib.or_batch_mt(data.ctypes.data, None if offsets is None else offsets.ctypes.data,
                                  stride, length, n, mode, None if ia is None else ia.ctypes.data,
                                  initial & 0xFFFF, None if ad is None else ad.ctypes.data,
                                  out.ctypes.data, threads)
        if rc != 0:
            raise RuntimeError("oracle batch failed")
        return out[:n * k]


_c_singleton = None
LIB_OPT_PATH = os.path.join(HERE, "build", "libcsum_oracle_opt.so")


def C() -> _C:
    global _c_singleton
    if _c_singleton is None:
        _c_singleton = _C()
    return _c_singleton


def C_opt() -> _C:
    """The same C restatement built -O3 -march=x86-64-v3 (vectorised): the
    "optimised CPU" baseline of SURVEY.md §8d. bench.py's cpu_baseline only."""
    return _C(LIB_OPT_PATH)

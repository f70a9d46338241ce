#!/usr/bin/env python3
"""Generate tests/golden/refexec.json: known answers produced by EXECUTING the
reference's own Go source for the checksum path.

The reference is Go and this image has no Go toolchain. tests/golden/goexec.py is a
minimal interpreter for the Go subset these files use; it loads, at generation time
only, the reference's files under /root/reference (nothing is copied into this repo)
and runs them:

* checksum.Checksum, ChecksumCombine, PseudoHeaderChecksum (checksum/checksum.go);
* the senders, end to end: sendUDP (transport/udp/endpoint.go:164-187), sendTCP and
  sendTCPWithOptions (transport/tcp/connect.go:556-586, :288-322), sendICMPv4
  (network/ipv4/icmp.go:36-45), each through types.Route (types/route.go) into the
  ipv4 endpoint's WritePacket (network/ipv4/ipv4.go:80-97), with the UDP / TCP /
  IPv4 Encode, CalculateChecksum and SetChecksum methods of header/ and the
  Prependable of buffer/prependable.go. A stub link endpoint takes what WritePacket
  hands it (hdr.UsedBytes() + payload, as tundev's writev does,
  link/tundev/tundev.go:56-58,171-196): the datagram the reference would put on the
  wire. Its stored checksum fields are the expected TX values;
* the checker: checker.IPv4 (checker/checker.go:25-40) and the function checker.TCP
  returns (:71-99), with a stub *testing.T whose Fatalf ends the check as
  runtime.Goexit does. The sum each computes (`xsum`) is read from the interpreter's
  frame of that function, so the verify values are the checker's own.

Restated (not executed), each marked "src": "restated" in the fixture, because no
reference function computes them:
* VERIFY_UDP and the UDP / ICMP parts of VERIFY_RX — the reference never verifies UDP
  or ICMP (transport/udp/endpoint.go:191-229); this repo applies checker.TCP's formula
  (and sendICMPv4's sum) to them;
* IPv4 headers WritePacket never encodes (IHL other than 5) and TX_DATAGRAM's results
  outside its contract (include/yucsum.h) — the field value is still the executed
  IPv4.CalculateChecksum, only the `^` and the contract rule are restated;
* RAW vectors call checksum.Checksum directly (executed; there is no glue).
The generator asserts that oracle/ (C and Python) agrees on every vector;
tests/test_oracle.py re-checks that on every CPU run, and tests/test_gpu_parity.py
checks the HIP path against the same vectors.

Run from the repo root: python tests/golden/make_refexec.py [out.json]
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import goexec as G  # noqa: E402
from oracle import oracle as O  # noqa: E402

REF = "/root/reference"
U16 = lambda v: G.Int(v, "uint16")  # noqa: E731
U32 = lambda v: G.Int(v, "uint32")  # noqa: E731


class TestingT:
    """Stub *testing.T: Fatalf records the message and its arguments and ends the
    check (runtime.Goexit in Go; an exception here)."""

    def __init__(self):
        self.failed = []

    def Fatalf(self, fmt, *args):  # noqa: N802 (Go method name)
        self.failed.append((fmt.b.decode(), [a.v if isinstance(a, G.Int) else a for a in args]))
        raise G.GoFatal(fmt.b.decode())


class LinkStub:
    """The link endpoint under the ipv4 endpoint: what tundev's WritePacket would
    write (hdr.UsedBytes() then the payload, link/tundev/tundev.go:56-58)."""

    def __init__(self, it):
        self.it, self.sent = it, []

    def MaxHeaderLength(self):  # noqa: N802
        return G.Int(0, "uint16")

    def WritePacket(self, r, hdr, payload, protocol):  # noqa: N802
        used = self.it.method("buffer", hdr, "UsedBytes")
        self.sent.append(used.bytes() + (payload.bytes() if payload is not None else b""))
        return None


class Ref:
    """The reference's functions, executed by goexec."""

    def __init__(self, it=None):
        """it: an interpreter from G.load_path; by default the reference's own files
        (the fixture). tests/test_go_shim_exec.py passes one whose package checksum is
        the cgo shim, to run these same callers unchanged on it."""
        self.it = it or G.load_path(REF)
        self.it.watch |= {("checker", "IPv4"), ("checker", "TCP.func")}
        self.link = LinkStub(self.it)

    def checksum(self, b: bytes, initial: int) -> int:
        return self.it.call("checksum", "Checksum", G.from_bytes(b), U16(initial)).v

    def combine(self, a: int, b: int) -> int:
        return self.it.call("checksum", "ChecksumCombine", U16(a), U16(b)).v

    def pseudo(self, proto: int, src: bytes, dst: bytes) -> int:
        return self.it.call("checksum", "PseudoHeaderChecksum", G.Int(proto, "uint32"),
                            G.Str(src), G.Str(dst)).v

    def m(self, typ: str, b: bytes, name: str, *args):
        return self.it.method("header", G.from_bytes(b, typ), name, *args)

    # --- the senders, executed end to end -----------------------------------------
    def route(self, src: bytes, dst: bytes):
        """A types.Route from src to dst over an ipv4 endpoint whose address is src
        (network/ipv4/ipv4.go:31-38 fields; types/route.go:14-36)."""
        ep = self.it._zero("endpoint", self.it.pkgs["ipv4"])
        ep.f["address"] = G.from_bytes(src, "address")
        ep.f["linkEp"] = self.link
        r = self.it._zero("Route", self.it.pkgs["types"])
        r.f["LocalAddress"], r.f["RemoteAddress"] = G.Str(src, "Address"), G.Str(dst, "Address")
        r.f["NetEp"] = ep
        return r

    def _sent(self):
        return self.link.sent.pop()

    @staticmethod
    def _view(data):
        return None if data is None else G.from_bytes(data, "View")

    def send_udp(self, src, dst, data, lport, rport) -> bytes:
        """transport/udp/endpoint.go:164-187 -> network/ipv4/ipv4.go:80-97."""
        self.it.call("udp", "sendUDP", self.route(src, dst), self._view(data), U16(lport), U16(rport))
        return self._sent()

    def send_tcp(self, src, dst, data, lport, rport, flags, seq, ack, wnd, opts=None) -> bytes:
        """transport/tcp/connect.go:556-586 (sendTCP) or, with options, :288-322
        (sendTCPWithOptions, as sendSynTCP calls it)."""
        tid = self.it._zero("TransportEndpointId", self.it.pkgs["types"])
        tid.f["LocalPort"], tid.f["RemotePort"] = U16(lport), U16(rport)
        args = [self.route(src, dst), tid, self._view(data), G.Int(flags, "uint8"), U32(seq), U32(ack), U32(wnd)]
        if opts is None:
            self.it.call("tcp", "sendTCP", *args)
        else:
            self.it.call("tcp", "sendTCPWithOptions", *args, G.from_bytes(opts))
        return self._sent()

    def send_icmp(self, src, dst, typ, code, data) -> bytes:
        """network/ipv4/icmp.go:36-45."""
        self.it.call("ipv4", "sendICMPv4", self.route(src, dst), G.Int(typ, "uint8"), G.Int(code, "uint8"),
                     self._view(data))
        return self._sent()

    # --- the checker, executed ----------------------------------------------------
    def checker_ipv4(self, pkt: bytes):
        """checker.IPv4(t, b) (checker/checker.go:25-40): (passed, xsum it computed)."""
        t = TestingT()
        self.it.frames.pop(("checker", "IPv4"), None)
        try:
            self.it.call("checker", "IPv4", t, G.from_bytes(pkt))
        except G.GoFatal:
            pass
        x = self.it.frames.get(("checker", "IPv4"), {}).get("xsum")
        return not t.failed, (None if x is None else x.v)

    def checker_tcp(self, pkt: bytes):
        """The function checker.TCP() returns (checker/checker.go:71-99), run on the
        datagram's IPv4 header as checker.IPv4 would pass it: (passed, xsum)."""
        t = TestingT()
        f = self.it.call("checker", "TCP")
        net = G.GoList([G.from_bytes(pkt, "IPv4")], "[]Network")
        self.it.frames.pop(("checker", "TCP.func"), None)
        try:
            self.it._invoke_closure(f, [t, net])
        except G.GoFatal:
            pass
        x = self.it.frames.get(("checker", "TCP.func"), {}).get("xsum")
        return not t.failed, (None if x is None else x.v)

    # --- restated glue (no reference function computes these) ---------------------
    def ipv4_field(self, pkt: bytes) -> int:
        """network/ipv4/ipv4.go:85-94 for a header WritePacket never encodes (any IHL):
        ^IPv4.CalculateChecksum() (executed) with the field 0."""
        b = bytearray(pkt)
        b[10:12] = b"\x00\x00"
        return ~self.m("IPv4", bytes(b), "CalculateChecksum").v & 0xFFFF

    def verify_l4(self, seg: bytes, src: bytes, dst: bytes, proto: int) -> int:
        """checker.TCP's formula (checker/checker.go:84-88) for a UDP datagram: the
        reference never verifies UDP."""
        l = len(seg) & 0xFFFF
        x = self.checksum(src, 0)
        x = self.checksum(dst, x)
        x = self.checksum(bytes([0, proto & 0xFF]), x)
        x = self.checksum(bytes([l >> 8, l & 0xFF]), x)
        return self.checksum(seg, x)

    def rx_flags(self, pkt: bytes):
        """YU_MODE_VERIFY_RX (include/yucsum.h): IPv4.IsValid (header/ipv4.go:126-138,
        executed), checker.IPv4's header sum and, for TCP, checker.TCP's transport sum
        (both executed); UDP and ICMP restated (the reference verifies neither).
        Returns (flags, "exec" | "restated")."""
        if not self.m("IPv4", pkt, "IsValid", G.Int(len(pkt), "int")):
            return 8, "exec"
        _, s = self.checker_ipv4(pkt)
        r = 1 if s in (0, 0xFFFF) else 0
        proto = self.m("IPv4", pkt, "Protocol").v
        src = "exec"
        if proto == 6:
            r |= 2
            _, s = self.checker_tcp(pkt)
            r |= 4 if s in (0, 0xFFFF) else 0
        elif proto in (1, 17):
            r |= 2
            src = "restated"
            payload = self.m("IPv4", pkt, "Payload").bytes()
            s = self.checksum(payload, 0) if proto == 1 else self.verify_l4(payload, pkt[12:16], pkt[16:20], 17)
            r |= 4 if s in (0, 0xFFFF) else 0
        return r, src

    def tx_contract(self, pkt: bytes) -> list:
        """TX_DATAGRAM's rule for datagrams no sender built (include/yucsum.h): {0, 0}
        outside 20 <= HeaderLength() <= TotalLength() <= len; the transport value 0 for
        another protocol or a segment shorter than its header; otherwise the
        executed header methods and the sender formulas on the segment."""
        if len(pkt) < 20:
            return [0, 0]
        hl = self.m("IPv4", pkt, "HeaderLength").v
        if hl < 20 or not self.m("IPv4", pkt, "IsValid", G.Int(len(pkt), "int")):
            return [0, 0]
        ip = self.ipv4_field(pkt)
        proto = self.m("IPv4", pkt, "Protocol").v
        seg = self.m("IPv4", pkt, "Payload").bytes()
        src, dst = pkt[12:16], pkt[16:20]
        l4 = 0
        if proto == 17 and len(seg) >= 8:
            u = bytearray(seg)
            u[6:8] = b"\x00\x00"
            x = self.checksum(bytes(seg[8:]), self.pseudo(17, src, dst))
            l4 = ~self.m("UDP", bytes(u), "CalculateChecksum", U16(x), U16(len(seg) & 0xFFFF)).v & 0xFFFF
        elif proto == 6 and len(seg) >= 20:
            t = bytearray(seg)
            t[16:18] = b"\x00\x00"
            doff = self.m("TCP", bytes(t), "DataOffset").v
            x = self.checksum(bytes(seg[doff:]), self.pseudo(6, src, dst))
            l4 = ~self.m("TCP", bytes(t), "CalculateChecksum", U16(x), U16(len(seg) & 0xFFFF)).v & 0xFFFF
        elif proto == 1 and len(seg) >= 4:
            h = bytearray(seg[:4])
            h[2:4] = b"\x00\x00"
            l4 = ~self.checksum(bytes(h), self.checksum(bytes(seg[4:]), 0)) & 0xFFFF
        return [ip, l4]


def vec_bytes(v):
    """A checksum vector's input: hex, or all-0x00 / all-0xFF of a length."""
    if "hex" in v:
        return bytes.fromhex(v["hex"])
    return bytes(v["len"]) if v["kind"] == "zero" else b"\xff" * v["len"]


def rnd(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def build(ref: Ref) -> dict:
    """The fixture's content, computed by `ref`'s interpreter (seeded: the same inputs
    on every run)."""
    rng = random.Random(20261016)
    C = O.C()
    out = {"generator": "tests/golden/make_refexec.py: reference Go source executed by tests/golden/goexec.py"}

    # checksum.Checksum
    cs = []
    lens = list(range(0, 70)) + [127, 128, 129, 255, 256, 1499, 1500, 1501, 4097, 9000]
    for n in lens:
        for kind in ("rand", "ff", "zero"):
            d = rnd(rng, n) if kind == "rand" else (b"\xff" * n if kind == "ff" else bytes(n))
            init = rng.choice([0, 0xFFFF, 1, rng.getrandbits(16)])
            v = {"hex": d.hex()} if kind == "rand" else {"len": n, "kind": kind}
            cs.append(dict(v, initial=init, want=ref.checksum(d, init)))
    cs.append({"hex": "0001f203f4f5f6f7", "initial": 0, "want": ref.checksum(bytes.fromhex("0001f203f4f5f6f7"), 0)})
    assert cs[-1]["want"] == 0xDDF2  # RFC 1071 section 3, from the reference's code
    for v in cs:
        d = vec_bytes(v)
        assert O.checksum(d, v["initial"]) == C.checksum(d, v["initial"]) == v["want"], v
    out["checksum"] = cs

    # the uint32 wrap above 131072 bytes (checksum.go:5,14): fill byte, length, initial
    wrap = []
    for n, fill, init in ((131072, 0xFF, 0xFFFF), (131073, 0xFF, 0xFFFF), (131074, 0xFF, 0xFFFF),
                          (131075, 0xFE, 0x00FF), (140000, 0xAB, 0x8000)):
        d = bytes([fill]) * n
        want = ref.checksum(d, init)
        assert O.checksum(d, init) == C.checksum(d, init) == want
        wrap.append({"len": n, "fill": fill, "initial": init, "want": want})
    assert wrap[2]["want"] == 65534
    out["wrap"] = wrap

    comb = []
    for a, b in [(0, 0), (0xFFFF, 0xFFFF), (0xFFFF, 1), (0x8000, 0x8000)] + \
            [(rng.getrandbits(16), rng.getrandbits(16)) for _ in range(100)]:
        want = ref.combine(a, b)
        assert O.checksum_combine(a, b) == C.combine(a, b) == want
        comb.append([a, b, want])
    out["combine"] = comb

    pseudo = []
    for proto in (0, 1, 6, 17, 255, 0x106, 0xFFFFFFFF):
        for sl, dl in ((4, 4), (4, 4), (16, 16), (0, 4), (3, 5)):
            src, dst = rnd(rng, sl), rnd(rng, dl)
            want = ref.pseudo(proto, src, dst)
            assert O.pseudo_header_checksum(proto, src, dst) == C.pseudo_header_checksum(proto, src, dst) == want
            pseudo.append({"proto": proto, "src": src.hex(), "dst": dst.hex(), "want": want})
    out["pseudo"] = pseudo

    # batch-mode vectors: packet bytes (TX modes: the checksum fields overwritten with
    # garbage, which the modes take as 0), addresses {src, dst}, the expected value,
    # and where it came from ("exec": the reference's sender / checker run end to end;
    # "restated": see the module doc)
    modes = {}

    def add(mode, pkt, addrs, want, src="exec"):
        modes.setdefault(str(mode), []).append({"hex": pkt.hex(), "addrs": addrs.hex(), "want": want,
                                                "src": src})

    def garble(b, at):
        b = bytearray(b)
        b[at:at + 2] = rnd(rng, 2)
        return bytes(b)

    def flip(b, lo=0):
        b = bytearray(b)
        i = rng.randrange(lo, len(b)) if len(b) > lo else None
        if i is not None:
            b[i] ^= 1 << rng.randrange(8)
        return bytes(b)

    be16 = lambda b, at: b[at] << 8 | b[at + 1]  # noqa: E731
    sent = []  # (datagram, proto) the senders put on the wire

    # TCP: sendTCP (DataOffset 20) and sendTCPWithOptions (options of 4..40 bytes, as
    # sendSynTCP passes them) with random ports, sequence numbers, flags and windows
    # (some above 0xffff: the clamp at connect.go:559-561), payloads of 0..1600 bytes
    for k in range(70):
        a = rnd(rng, 8)
        n = rng.choice([0, 1, 2, 3, 40, 41, 1460, 1480, rng.randint(0, 1600)])
        data = rnd(rng, n) if n or k % 2 else None
        opts = None if k % 3 == 0 else rnd(rng, 4 * rng.randint(0, 10))
        dg = ref.send_tcp(a[:4], a[4:], data, rng.getrandbits(16), rng.getrandbits(16), rng.getrandbits(8),
                          rng.getrandbits(32), rng.getrandbits(32), rng.getrandbits(17), opts)
        seg = dg[20:]
        add(O.MODE_TCP, garble(seg, 16), a, be16(seg, 16))
        sent.append((dg, 6))
        # checker.TCP over the segment as sent, or with a bit flipped: its own xsum
        sg = seg if k % 2 else flip(seg)
        ok, x = ref.checker_tcp(dg[:20] + sg)
        assert ok == (x in (0, 0xFFFF))
        add(O.MODE_VERIFY_TCP, sg, a, x)
    # UDP: sendUDP, payloads of 0..1600 bytes (nil and empty views included)
    for k in range(70):
        a = rnd(rng, 8)
        n = rng.choice([0, 1, 2, 3, 64, 65, 1472, rng.randint(0, 1600)])
        data = rnd(rng, n) if n or k % 2 else None
        dg = ref.send_udp(a[:4], a[4:], data, rng.getrandbits(16), rng.getrandbits(16))
        seg = dg[20:]
        add(O.MODE_UDP, garble(seg, 6), a, be16(seg, 6))
        sent.append((dg, 17))
        sg = seg if k % 2 else flip(seg)
        add(O.MODE_VERIFY_UDP, sg, a, ref.verify_l4(sg, a[:4], a[4:], 17), "restated")
    # the UDP field 0x0000 (no RFC 768 0 -> 0xFFFF substitution, header/udp.go:60-62 via
    # transport/udp/endpoint.go:184): the payload's last word moved by the field value
    # (one's complement) so that the sum comes to 0xFFFF, then sent again; the executed
    # sender stores 0x0000. The same for sendTCP, where 0x0000 is legal anyway.
    def zero_field(send, seg_off, n):
        data = bytearray(rnd(rng, n))
        dg = send(bytes(data))
        f = be16(dg, seg_off)
        w = (data[-2] << 8 | data[-1]) + f
        w = w - 0xFFFF if w > 0xFFFF else w
        data[-2:] = bytes([w >> 8, w & 0xFF])
        dg = send(bytes(data))
        assert be16(dg, seg_off) == 0, hex(be16(dg, seg_off))
        return dg
    for k in range(6):
        a = rnd(rng, 8)
        ports = (rng.getrandbits(16), rng.getrandbits(16))
        dg = zero_field(lambda d: ref.send_udp(a[:4], a[4:], d, *ports), 26, 2 * rng.randint(1, 40))
        add(O.MODE_UDP, garble(dg[20:], 6), a, 0)
        sent.append((dg, 17))
    for k in range(2):
        a = rnd(rng, 8)
        hdr = (rng.getrandbits(16), rng.getrandbits(16), 0x18, rng.getrandbits(32), rng.getrandbits(32), 4096)
        dg = zero_field(lambda d: ref.send_tcp(a[:4], a[4:], d, *hdr), 36, 2 * rng.randint(1, 40))
        add(O.MODE_TCP, garble(dg[20:], 16), a, 0)
        sent.append((dg, 6))
    # ICMP: sendICMPv4 (echo replies and other types), payloads of 0..1600 bytes
    for k in range(50):
        a = rnd(rng, 8)
        n = rng.choice([0, 1, 4, 5, 56, 64, 65, rng.randint(0, 1600)])
        data = rnd(rng, n) if n or k % 2 else None
        dg = ref.send_icmp(a[:4], a[4:], rng.choice([0, 3, 8, 11, rng.getrandbits(8)]), rng.getrandbits(8), data)
        add(O.MODE_ICMP, garble(dg[20:], 2), bytes(8), be16(dg, 22))
        sent.append((dg, 1))
    # IPv4 header field: every datagram a sender built (WritePacket's value), as the
    # header alone and as the whole datagram; checker.IPv4 on them as sent and damaged
    for i, (dg, _) in enumerate(sent):
        if i % 2 == 0:
            add(O.MODE_IPV4, garble(dg if i % 4 == 0 else dg[:20], 10), bytes(8), be16(dg, 10))
        if i % 3 == 0:
            d2 = dg if i % 2 else flip(dg[:20]) + dg[20:]
            ok, x = ref.checker_ipv4(d2)
            if x is not None:  # IsValid held: checker.IPv4's own sum
                assert ok == (x in (0, 0xFFFF))
                add(O.MODE_VERIFY_IPV4, d2, bytes(8), x)
    # headers WritePacket never encodes: any IHL 0..15 (restated ^, executed sum)
    for _ in range(60):
        ihl = rng.randint(0, 15)
        n = max(1, 4 * ihl) + rng.choice([0, 0, 1, 3, 100])
        p = bytearray(rnd(rng, n))
        p[0] = 0x40 | ihl
        add(O.MODE_IPV4, bytes(p), bytes(8), ref.ipv4_field(bytes(p)), "restated")
        # VERIFY_IPV4 is the sum checker.IPv4 computes (checker.go:32): the executed
        # IPv4.CalculateChecksum, which checker.IPv4 reaches only when IsValid holds
        add(O.MODE_VERIFY_IPV4, bytes(p), bytes(8), ref.m("IPv4", bytes(p), "CalculateChecksum").v, "exec")
    for _ in range(40):
        n = rng.choice([0, 1, 2, 3, 63, 64, 65, 1500, rng.randint(0, 1600)])
        d = rnd(rng, n)
        init = rng.getrandbits(16)
        add(O.MODE_RAW, d, init.to_bytes(2, "little") + bytes(6), ref.checksum(d, init))
    # whole outgoing datagrams (TX_DATAGRAM): as the senders built them, both fields
    # then overwritten with garbage; the values are the fields the senders stored
    for dg, proto in sent:
        f = {17: 6, 6: 16, 1: 2}[proto]
        add(O.MODE_TX_DATAGRAM, garble(garble(dg, 10), 20 + f), bytes(8), [be16(dg, 10), be16(dg, 20 + f)])
    # whole received datagrams (VERIFY_RX): as sent, with a bit flipped in the header
    # or the payload, and rxgen's malformed and damaged ones
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rxgen  # tests/rxgen.py: datagrams built like the reference senders
    for i, (dg, _) in enumerate(sent):
        if i % 2:
            d2 = dg if i % 3 else flip(dg, 0 if i % 5 else 20)
            f, src = ref.rx_flags(d2)
            add(O.MODE_VERIFY_RX, d2, bytes(8), f, src)
    nrng = np.random.default_rng(16)
    blob, offs = rxgen.rx_batch(nrng, 120, lo=0, hi=1480)
    for i in range(len(offs) - 1):
        pk = bytes(blob[int(offs[i]):int(offs[i + 1])])
        f, src = ref.rx_flags(pk)
        add(O.MODE_VERIFY_RX, pk, bytes(8), f, src)
    # TX_DATAGRAM outside what the senders build: rxgen datagrams (any protocol, some
    # damaged or out of contract), under the mode's contract rule (restated)
    for i in range(60):
        pk = bytearray(rxgen.make_packet(nrng, int(nrng.integers(0, 1480)),
                                         ihl=5 if i % 3 else None))
        hl = (pk[0] & 0xF) * 4
        pk[10:12] = rnd(rng, 2)
        f = {17: 6, 6: 16, 1: 2}.get(pk[9])
        if f is not None:
            pk[hl + f: hl + f + 2] = rnd(rng, 2)
        if i % 10 == 9:
            pk = rxgen.tcp_contract(rxgen.damage(nrng, pk))
        add(O.MODE_TX_DATAGRAM, bytes(pk), bytes(8), ref.tx_contract(bytes(pk)), "restated")
    for ihl in (0, 1, 4):  # HeaderLength() under 20: outside the contract
        pk = bytearray(rxgen.make_packet(nrng, 40, proto=17, ihl=5))
        pk[0] = 0x40 | ihl
        add(O.MODE_TX_DATAGRAM, bytes(pk), bytes(8), ref.tx_contract(bytes(pk)), "restated")
    # the executed senders' fields agree with the restated contract rule where both apply
    for dg, proto in sent:
        f = {17: 6, 6: 16, 1: 2}[proto]
        assert ref.tx_contract(garble(garble(dg, 10), 20 + f)) == [be16(dg, 10), be16(dg, 20 + f)]
    out["modes"] = modes

    # oracle agreement on every mode vector (ragged batch through the C oracle)
    for mode, vecs in modes.items():
        m = int(mode)
        pk = [bytes.fromhex(v["hex"]) for v in vecs]
        offs = np.zeros(len(pk) + 1, np.uint64)
        offs[1:] = np.cumsum([len(x) for x in pk])
        data = np.frombuffer(b"".join(pk) + b"\0", np.uint8)
        ad = np.frombuffer(b"".join(bytes.fromhex(v["addrs"]) for v in vecs), np.uint8)
        init = np.array([int.from_bytes(bytes.fromhex(v["addrs"])[:2], "little") for v in vecs], np.uint16)
        got = C.batch(data, m, offsets=offs, addrs=ad if m in (1, 2, 6, 7) else None,
                      initial_arr=init if m == O.MODE_RAW else None)
        want = np.array([v["want"] for v in vecs], np.uint16).reshape(-1)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mode, bad[:5], got[bad[:5]], want[bad[:5]])

    return out


def main() -> None:
    out = build(Ref())
    modes, cs, pseudo, comb, wrap = out["modes"], out["checksum"], out["pseudo"], out["combine"], out["wrap"]
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "refexec.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {path}: {sum(len(v) for v in modes.values())} mode vectors, {len(cs)} checksum, "
          f"{len(pseudo)} pseudo, {len(comb)} combine, {len(wrap)} wrap")


if __name__ == "__main__":
    main()

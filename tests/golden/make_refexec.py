#!/usr/bin/env python3
"""Generate tests/golden/refexec.json: known answers produced by EXECUTING the
reference's own Go source for the checksum path.

The reference is Go and this image has no Go toolchain. tests/golden/goexec.py is a
minimal interpreter for the Go subset these files use; it loads, at generation time
only, /root/reference/checksum/checksum.go and /root/reference/header/{ipv4,tcp,udp}.go
(nothing is copied into this repo) and runs their functions and methods:

* checksum.Checksum, checksum.ChecksumCombine, checksum.PseudoHeaderChecksum;
* header.IPv4.{CalculateChecksum, IsValid, HeaderLength, TotalLength, Protocol,
  Payload, SourceAddress...}, header.TCP.{CalculateChecksum, DataOffset},
  header.UDP.CalculateChecksum.

The few lines that glue them together per batch mode are restated below from the
reference call sites they follow (file:line in each helper). Expected values in the
fixture therefore come from the reference's code, not from oracle/. The generator
asserts that oracle/ (C and Python) agrees on every vector; tests/test_oracle.py
re-checks that on every CPU run, and tests/test_gpu_parity.py checks the HIP path
against the same vectors.

Run from the repo root: python tests/golden/make_refexec.py
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


class Ref:
    """The reference's functions, executed by goexec."""

    def __init__(self):
        self.it = G.load_reference(REF)

    def checksum(self, b: bytes, initial: int) -> int:
        return self.it.call("checksum", "Checksum", G.from_bytes(b), U16(initial)).v

    def combine(self, a: int, b: int) -> int:
        return self.it.call("checksum", "ChecksumCombine", U16(a), U16(b)).v

    def pseudo(self, proto: int, src: bytes, dst: bytes) -> int:
        return self.it.call("checksum", "PseudoHeaderChecksum", G.Int(proto, "uint32"),
                            G.Str(src), G.Str(dst)).v

    def m(self, typ: str, b: bytes, name: str, *args):
        return self.it.method("header", G.from_bytes(b, typ), name, *args)

    # --- TX compositions (field value the sender stores) --------------------------
    def tcp_field(self, seg: bytes, src: bytes, dst: bytes) -> int:
        """transport/tcp/connect.go:576-583 (sendTCP) and :310-317 (with options):
        the header is Encode()d with checksum 0 (header/tcp.go:176-186), the data
        follows DataOffset(); route.PseudoHeaderChecksum(6) = checksum.
        PseudoHeaderChecksum(6, local, remote) (types/route.go:90-92)."""
        hdr = bytearray(seg)
        hdr[16:18] = b"\x00\x00"
        doff = self.m("TCP", bytes(hdr), "DataOffset").v
        data = bytes(seg[doff:])
        xsum = self.pseudo(6, src, dst)
        length = len(seg) & 0xFFFF
        xsum = self.checksum(data, xsum)
        r = self.m("TCP", bytes(hdr), "CalculateChecksum", U16(xsum), U16(length)).v
        return ~r & 0xFFFF

    def udp_field(self, dgram: bytes, src: bytes, dst: bytes) -> int:
        """transport/udp/endpoint.go:171-184 (sendUDP): Encode() leaves the checksum
        field 0 (header/udp.go:78-83), data follows the 8-byte header."""
        hdr = bytearray(dgram)
        hdr[6:8] = b"\x00\x00"
        xsum = self.pseudo(17, src, dst)
        xsum = self.checksum(bytes(dgram[8:]), xsum)
        r = self.m("UDP", bytes(hdr), "CalculateChecksum", U16(xsum), U16(len(dgram) & 0xFFFF)).v
        return ~r & 0xFFFF

    def ipv4_field(self, pkt: bytes) -> int:
        """network/ipv4/ipv4.go:85-94: Encode() with checksum 0 (header/ipv4.go:146-157),
        then SetChecksum(^CalculateChecksum())."""
        b = bytearray(pkt)
        b[10:12] = b"\x00\x00"
        return ~self.m("IPv4", bytes(b), "CalculateChecksum").v & 0xFFFF

    def icmp_field(self, msg: bytes) -> int:
        """network/ipv4/icmp.go:36-45: ^Checksum(icmpv4 header (field 0), Checksum(data, 0))."""
        hdr = bytearray(msg[:4])
        hdr[2:4] = b"\x00\x00"
        return ~self.checksum(bytes(hdr), self.checksum(bytes(msg[4:]), 0)) & 0xFFFF

    def tx_datagram(self, pkt: bytes) -> list:
        """YU_MODE_TX_DATAGRAM (include/yucsum.h): a whole outgoing datagram's two
        fields — ipv4.WritePacket's header field (network/ipv4/ipv4.go:85-94) and the
        transport field its sender stored before (sendUDP / sendTCP / sendICMPv4),
        with the route addresses = the header's SourceAddress / DestinationAddress
        (ipv4.go:84-92 encodes them from the same route) over Payload()."""
        if len(pkt) < 20:
            return [0, 0]
        hl = self.m("IPv4", pkt, "HeaderLength").v
        tl = self.m("IPv4", pkt, "TotalLength").v
        if hl < 20 or not self.m("IPv4", pkt, "IsValid", G.Int(len(pkt), "int")):
            return [0, 0]
        ip = self.ipv4_field(pkt)
        proto = self.m("IPv4", pkt, "Protocol").v
        seg = self.m("IPv4", pkt, "Payload").bytes()
        assert len(seg) == tl - hl
        # SourceAddress() / DestinationAddress() are b[12:16] / b[16:20]
        # (header/ipv4.go:111-118; their types.Address is outside goexec's packages)
        src, dst = pkt[12:16], pkt[16:20]
        l4 = 0
        if proto == 17 and len(seg) >= 8:
            l4 = self.udp_field(seg, src, dst)
        elif proto == 6 and len(seg) >= 20:
            l4 = self.tcp_field(seg, src, dst)
        elif proto == 1 and len(seg) >= 4:
            l4 = self.icmp_field(seg)
        return [ip, l4]

    # --- receive-side verification (checker semantics) ------------------------------
    def verify_ipv4(self, pkt: bytes) -> int:
        """checker/checker.go:32-35: the sum over b[:HeaderLength()] incl. the field."""
        return self.m("IPv4", pkt, "CalculateChecksum").v

    def verify_l4(self, seg: bytes, src: bytes, dst: bytes, proto: int) -> int:
        """checker/checker.go:80-92 (checker.TCP), the same formula for UDP."""
        l = len(seg) & 0xFFFF
        x = self.checksum(src, 0)
        x = self.checksum(dst, x)
        x = self.checksum(bytes([0, proto & 0xFF]), x)
        x = self.checksum(bytes([l >> 8, l & 0xFF]), x)
        return self.checksum(seg, x)

    def rx_flags(self, pkt: bytes) -> int:
        """YU_MODE_VERIFY_RX (include/yucsum.h): IPv4.IsValid (header/ipv4.go:126-138),
        checker.IPv4's header test and checker.TCP's transport test over
        Payload() = b[HeaderLength():][:PayloadLength()] (header/ipv4.go:181-189) with
        the addresses and protocol read from the packet; ICMP without the pseudo
        header (network/ipv4/icmp.go:36-45)."""
        if not self.m("IPv4", pkt, "IsValid", G.Int(len(pkt), "int")):
            return 8
        r = 0
        s = self.verify_ipv4(pkt)
        if s in (0, 0xFFFF):
            r |= 1
        proto = self.m("IPv4", pkt, "Protocol").v
        if proto in (1, 6, 17):
            r |= 2
            payload = self.m("IPv4", pkt, "Payload").bytes()
            if proto == 1:
                s = self.checksum(payload, 0)
            else:
                s = self.verify_l4(payload, pkt[12:16], pkt[16:20], proto)
            if s in (0, 0xFFFF):
                r |= 4
        return r


def vec_bytes(v):
    """A checksum vector's input: hex, or all-0x00 / all-0xFF of a length."""
    if "hex" in v:
        return bytes.fromhex(v["hex"])
    return bytes(v["len"]) if v["kind"] == "zero" else b"\xff" * v["len"]


def rnd(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def main() -> None:
    ref = Ref()
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

    # batch-mode vectors: packet bytes (checksum fields left random: TX modes take
    # them as 0), addresses {src, dst}, expected value from the reference
    modes = {}

    def add(mode, pkt, addrs, want):
        modes.setdefault(str(mode), []).append({"hex": pkt.hex(), "addrs": addrs.hex(), "want": want})

    for _ in range(60):
        n = rng.choice([20, 21, 24, 40, 41, 60, 61, 200, 1460, 1500, rng.randint(20, 1600)])
        doff = 4 * rng.randint(5, min(15, n // 4))
        seg = bytearray(rnd(rng, n))
        seg[12] = (doff // 4) << 4 | (seg[12] & 0x0F)
        a = rnd(rng, 8)
        add(O.MODE_TCP, bytes(seg), a, ref.tcp_field(bytes(seg), a[:4], a[4:]))
        add(O.MODE_VERIFY_TCP, bytes(seg), a, ref.verify_l4(bytes(seg), a[:4], a[4:], 6))
    for _ in range(60):
        n = rng.choice([8, 9, 10, 72, 73, 1472, rng.randint(8, 1600)])
        d = rnd(rng, n)
        a = rnd(rng, 8)
        add(O.MODE_UDP, d, a, ref.udp_field(d, a[:4], a[4:]))
        add(O.MODE_VERIFY_UDP, d, a, ref.verify_l4(d, a[:4], a[4:], 17))
    for _ in range(60):
        ihl = rng.randint(0, 15)
        n = max(1, 4 * ihl) + rng.choice([0, 0, 1, 3, 100])
        p = bytearray(rnd(rng, n))
        p[0] = 0x40 | ihl
        add(O.MODE_IPV4, bytes(p), bytes(8), ref.ipv4_field(bytes(p)))
        add(O.MODE_VERIFY_IPV4, bytes(p), bytes(8), ref.verify_ipv4(bytes(p)))
    for _ in range(40):
        n = rng.choice([4, 5, 8, 64, 65, rng.randint(4, 1600)])
        d = rnd(rng, n)
        add(O.MODE_ICMP, d, bytes(8), ref.icmp_field(d))
    for _ in range(40):
        n = rng.choice([0, 1, 2, 3, 63, 64, 65, 1500, rng.randint(0, 1600)])
        d = rnd(rng, n)
        init = rng.getrandbits(16)
        add(O.MODE_RAW, d, init.to_bytes(2, "little") + bytes(6), ref.checksum(d, init))
    # whole received datagrams: well-formed (the reference's senders), damaged, malformed
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import rxgen  # tests/rxgen.py: datagrams built like the reference senders
    nrng = np.random.default_rng(16)
    blob, offs = rxgen.rx_batch(nrng, 120, lo=0, hi=1480)
    for i in range(len(offs) - 1):
        pk = bytes(blob[int(offs[i]):int(offs[i + 1])])
        add(O.MODE_VERIFY_RX, pk, bytes(8), ref.rx_flags(pk))
    # whole outgoing datagrams (TX_DATAGRAM): built like the reference senders, their
    # checksum fields then overwritten with garbage (the mode takes them as 0), plus
    # out-of-contract ones (IHL < 5, lengths that do not fit, other protocols)
    for i in range(120):
        pk = bytearray(rxgen.make_packet(nrng, int(nrng.integers(0, 1480)),
                                         ihl=5 if i % 3 else None))
        hl = (pk[0] & 0xF) * 4
        pk[10:12] = rnd(rng, 2)
        f = {17: 6, 6: 16, 1: 2}.get(pk[9])
        if f is not None:
            pk[hl + f: hl + f + 2] = rnd(rng, 2)
        if i % 10 == 9:
            pk = rxgen.tcp_contract(rxgen.damage(nrng, pk))
        add(O.MODE_TX_DATAGRAM, bytes(pk), bytes(8), ref.tx_datagram(bytes(pk)))
    for ihl in (0, 1, 4):  # HeaderLength() under 20: outside the contract
        pk = bytearray(rxgen.make_packet(nrng, 40, proto=17, ihl=5))
        pk[0] = 0x40 | ihl
        add(O.MODE_TX_DATAGRAM, bytes(pk), bytes(8), ref.tx_datagram(bytes(pk)))
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

    path = os.path.join(HERE, "refexec.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {path}: {sum(len(v) for v in modes.values())} mode vectors, {len(cs)} checksum, "
          f"{len(pseudo)} pseudo, {len(comb)} combine, {len(wrap)} wrap")


if __name__ == "__main__":
    main()

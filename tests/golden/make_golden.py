#!/usr/bin/env python3
"""Generate tests/golden/golden.json — known-answer vectors for the checksum path.

The reference (Go) cannot run in this image and ships no known-answer vectors
(SURVEY.md §8c), so the expected values come from the oracle's pure-Python twin
(oracle/oracle.py, a literal restatement of checksum/checksum.go and its call
sites), cross-checked here against the C restatement (oracle/csum_oracle.c) and the
closed form. Pins carried in the file that do NOT depend on our restatements:

* RFC 1071 §3's published example: 00 01 f2 03 f4 f5 f6 f7 -> 0xddf2;
* the IPv4 header of RFC 1071-style worked examples with a known field value
  (4500 0073 0000 4000 4011 .... c0a8 0001 c0a8 00c7 -> field 0xb861);
* the reference's own test-side property (checker/checker.go:32-35,80-92): every
  packet built the way the reference's test harnesses build them
  (transport/tcp/testing/context/context.go:164-209,
  transport/udp/udp_test.go:105-144) sums to 0 or 0xFFFF.

Inputs are generated from a fixed seed; random byte strings are stored as hex.
Run from the repo root: python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import random
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402

EDGE_LENS = [0, 1, 2, 3, 15, 16, 17, 63, 64, 65, 1499, 1500, 1501, 8999, 9000]
INITIALS = [0, 0xFFFF, 0x1234]


def pattern(kind: str, n: int, rng: random.Random) -> bytes:
    if kind == "zero":
        return bytes(n)
    if kind == "ff":
        return b"\xff" * n
    return bytes(rng.getrandbits(8) for _ in range(n))


def tcp_harness_packet(payload: bytes, src_port, dst_port, seq, ack, flags, wnd, opts=b"",
                       test_addr=b"\x0a\x00\x00\x02", stack_addr=b"\x0a\x00\x00\x01") -> bytes:
    """context.go:164-209 (SendPacket), restated with the oracle's functions."""
    buf = bytearray(20 + 20 + len(opts) + len(payload))
    buf[len(buf) - len(payload):] = payload
    buf[len(buf) - len(payload) - len(opts): len(buf) - len(payload)] = opts
    # IPv4 Encode (header/ipv4.go:146-157) + SetChecksum(^CalculateChecksum())
    buf[0] = 0x45
    struct.pack_into(">HHH", buf, 2, len(buf), 0, 0)
    buf[8], buf[9] = 64, 6
    buf[12:16], buf[16:20] = test_addr, stack_addr
    struct.pack_into(">H", buf, 10, ~O.ipv4_calculate_checksum(bytes(buf[:20])) & 0xFFFF)
    # TCP Encode (header/tcp.go:176-186)
    t = 20
    struct.pack_into(">HHII", buf, t, src_port, dst_port, seq, ack)
    buf[t + 12] = ((20 + len(opts)) // 4) << 4
    buf[t + 13] = flags
    struct.pack_into(">HHH", buf, t + 14, wnd, 0, 0)
    xsum = O.checksum(test_addr, 0)
    xsum = O.checksum(stack_addr, xsum)
    xsum = O.checksum(bytes([0, 6]), xsum)
    length = 20 + len(opts) + len(payload)
    xsum = O.checksum(payload, xsum)
    struct.pack_into(">H", buf, t + 16, ~O.tcp_calculate_checksum(bytes(buf[t:]), xsum, length) & 0xFFFF)
    return bytes(buf)


def udp_harness_packet(payload: bytes, src_port, dst_port,
                       test_addr=b"\x0a\x01\x00\x01", stack_addr=b"\x0a\x01\x00\x02") -> bytes:
    """udp_test.go:105-144 (sendPacket), restated with the oracle's functions."""
    buf = bytearray(8 + 20 + len(payload))
    buf[len(buf) - len(payload):] = payload
    buf[0] = 0x45
    struct.pack_into(">HHH", buf, 2, len(buf), 0, 0)
    buf[8], buf[9] = 64, 17
    buf[12:16], buf[16:20] = test_addr, stack_addr
    struct.pack_into(">H", buf, 10, ~O.ipv4_calculate_checksum(bytes(buf[:20])) & 0xFFFF)
    struct.pack_into(">HHHH", buf, 20, src_port, dst_port, 8 + len(payload), 0)
    xsum = O.checksum(test_addr, 0)
    xsum = O.checksum(stack_addr, xsum)
    xsum = O.checksum(bytes([0, 17]), xsum)
    length = 8 + len(payload)
    xsum = O.checksum(payload, xsum)
    struct.pack_into(">H", buf, 26, ~O.udp_calculate_checksum(bytes(buf[20:]), xsum, length) & 0xFFFF)
    return bytes(buf)


def main() -> None:
    rng = random.Random(20261015)
    C = O.C()
    raw = []
    for n in EDGE_LENS:
        for kind in ("zero", "ff", "rand"):
            data = pattern(kind, n, rng)
            for init in INITIALS:
                want = O.checksum(data, init)
                assert want == O.checksum_loop(data, init) == C.checksum(data, init) == \
                    O.checksum_closed_form(data, init)
                raw.append({"len": n, "kind": kind, "initial": init,
                            "hex": data.hex() if kind == "rand" else None, "want": want})

    published = [
        {"what": "RFC 1071 section 3 example", "hex": "0001f203f4f5f6f7", "initial": 0, "want": 0xDDF2},
        {"what": "IPv4 header (field zeroed) -> stored field ^Checksum",
         "hex": "450000730000400040110000c0a80001c0a800c7", "initial": 0, "want_field": 0xB861},
    ]
    for p in published:
        d = bytes.fromhex(p["hex"])
        if "want" in p:
            assert O.checksum(d, p["initial"]) == p["want"] == C.checksum(d, p["initial"])
        else:
            assert (~O.checksum(d, 0) & 0xFFFF) == p["want_field"]

    wrap = []
    for n, fill, init in ((131072, 0xFF, 0xFFFF), (131073, 0xFF, 0xFFFF), (131074, 0xFF, 0xFFFF),
                          (262144, 0xFF, 0), (200001, 0xAB, 0x8000)):
        d = bytes([fill]) * n
        want = O.checksum(d, init)
        assert want == C.checksum(d, init)
        wrap.append({"len": n, "fill": fill, "initial": init, "want": want})
    assert wrap[2]["want"] == 65534  # the reference's uint32 wrap (exact sum would be 65535)

    pseudo = []
    for src, dst, proto in ((b"\x0a\x00\x00\x02", b"\x0a\x00\x00\x01", 6),
                            (b"\x0a\x01\x00\x01", b"\x0a\x01\x00\x02", 17),
                            (b"\xff\xff\xff\xff", b"\xff\xff\xff\xff", 17),
                            (b"\x00\x00\x00\x00", b"\x00\x00\x00\x00", 0x106)):
        want = O.pseudo_header_checksum(proto, src, dst)
        assert want == C.pseudo_header_checksum(proto, src, dst)
        pseudo.append({"proto": proto, "src": src.hex(), "dst": dst.hex(), "want": want})

    # packets as the reference's test harnesses build them; fields + checker sums
    harness = []
    tcp_payloads = [b"", bytes([1, 2, 3]), bytes(range(256)) * 4, pattern("rand", 1460, rng)]
    for i, pl in enumerate(tcp_payloads):
        opts = b"\x02\x04\x05\xb4\x01\x03\x03\x07" if i == 1 else b""  # MSS + WS, as in SYN options
        pk = tcp_harness_packet(pl, 4096, 1234, 790 + i, 1000, 0x18, 30000, opts)
        seg = pk[20:]
        harness.append({"proto": "tcp", "hex": pk.hex(),
                        "ipv4_field": struct.unpack_from(">H", pk, 10)[0],
                        "transport_field": struct.unpack_from(">H", pk, 36)[0],
                        "verify_ipv4": O.ipv4_calculate_checksum(pk),
                        "verify_transport": O.packet(O.MODE_VERIFY_TCP, seg, addrs=pk[12:20], p=0)})
    for n in (30, 64, 129):
        pk = udp_harness_packet(pattern("rand", n, rng), 4096, 1234)
        seg = pk[20:]
        harness.append({"proto": "udp", "hex": pk.hex(),
                        "ipv4_field": struct.unpack_from(">H", pk, 10)[0],
                        "transport_field": struct.unpack_from(">H", pk, 26)[0],
                        "verify_ipv4": O.ipv4_calculate_checksum(pk),
                        "verify_transport": O.packet(O.MODE_VERIFY_UDP, seg, addrs=pk[12:20], p=0)})
    for h in harness:  # checker/checker.go:32-35, 84-92
        assert h["verify_ipv4"] in (0, 0xFFFF) and h["verify_transport"] in (0, 0xFFFF)

    # batch compositions (every mode) over a small ragged batch
    lens = [60, 61, 62, 63, 64, 100, 1500, 1501, 20, 24, 28, 40]
    blob = bytearray()
    offs = [0]
    for n in lens:
        pk = bytearray(pattern("rand", n, rng))
        pk[0] = 0x45 + (len(offs) % 3)          # IHL 5..7 for the IPv4 modes
        pk[12] = (5 + (len(offs) % 3)) << 4     # DataOffset 20..28 for the TCP modes
        blob += pk
        offs.append(len(blob))
    addrs = pattern("rand", 8 * len(lens), rng)
    init = [rng.getrandbits(16) for _ in lens]
    modes = {}
    for m, name in O.MODE_NAMES.items():
        want_a = O.batch_ragged_py(bytes(blob), offs, m, addrs=addrs if m in (1, 2, 6, 7) else None)
        want_i = O.batch_ragged_py(bytes(blob), offs, m, initial_arr=init)
        c_a = C.batch(np.frombuffer(bytes(blob), np.uint8), m, offsets=np.array(offs, np.uint64),
                      addrs=np.frombuffer(addrs, np.uint8) if m in (1, 2, 6, 7) else None)
        c_i = C.batch(np.frombuffer(bytes(blob), np.uint8), m, offsets=np.array(offs, np.uint64),
                      initial_arr=np.array(init, np.uint16))
        assert (want_a == c_a).all() and (want_i == c_i).all(), name
        modes[name] = {"with_addrs": [int(x) for x in want_a], "with_initial": [int(x) for x in want_i]}

    # VERIFY_RX (whole received datagrams): the harness packets above are what the
    # reference's tests feed checker.IPv4/checker.TCP, so each must come out
    # IP_OK | L4 | L4_OK; damaged copies and the published header pin the rest.
    rx = []
    for h in harness:
        pk = bytes.fromhex(h["hex"])
        variants = [("as built", pk)]
        b = bytearray(pk); b[25] ^= 0x01; variants.append(("transport byte flipped", bytes(b)))
        b = bytearray(pk); b[8] ^= 0x80; variants.append(("ttl flipped", bytes(b)))
        variants.append(("trailing bytes", pk + b"\x00\x01\x02"))
        variants.append(("truncated", pk[:-1]))
        for what, d in variants:
            want = O.packet(O.MODE_VERIFY_RX, d)
            assert want == C.batch(np.frombuffer(d, np.uint8), O.MODE_VERIFY_RX,
                                   offsets=np.array([0, len(d)], np.uint64))[0]
            rx.append({"what": f"{h['proto']} harness, {what}", "hex": d.hex(), "want": want})
    assert all(r["want"] == 7 for r in rx if r["what"].endswith("as built"))
    hdr = bytes.fromhex("4500007300004000" "4011b861c0a80001c0a800c7")
    rx.append({"what": "published header + 95 zero bytes", "hex": (hdr + bytes(95)).hex(),
               "want": O.packet(O.MODE_VERIFY_RX, hdr + bytes(95))})
    assert rx[-1]["want"] & O.RX_IP_OK

    out = {
        "generator": "tests/golden/make_golden.py (oracle/oracle.py twin, cross-checked vs oracle/csum_oracle.c)",
        "published": published, "raw": raw, "wrap": wrap, "pseudo": pseudo, "harness": harness,
        "batch": {"hex": bytes(blob).hex(), "offsets": offs, "addrs": addrs.hex(), "initial": init,
                  "modes": modes},
        "rx": rx,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(raw)} raw, {len(wrap)} wrap, {len(pseudo)} pseudo, {len(harness)} harness, "
          f"{len(modes)} batch-mode, {len(rx)} rx vectors")


if __name__ == "__main__":
    main()

"""Generates tests/golden/kernel_verified.npz: datagrams whose checksums the Linux
kernel verified, and datagrams the Linux kernel built itself (data only; run in a
container that may create tun devices: python tests/golden/make_kernel_verified.py).

* sent_*: IPv4 datagrams built by this repo's send compositions (sendTCP, sendICMPv4,
  ipv4.WritePacket over the scalar C ABI; tests/tun_probe.py) that the kernel accepted
  over a tun link: it answered every echo request and SYN, and delivered every data
  segment to the accepted socket. Their stored fields are what TX_DATAGRAM must give.
* kernel_*: what the kernel wrote back (echo replies, SYN-ACK, ACKs with TCP options)
  and datagrams a kernel UDP socket sent: checksums computed by Linux, an
  implementation independent of this repo and of the reference. VERIFY_RX must pass
  them.

Both sets are ragged batches: blob (uint8) + offsets (uint64, n+1).
"""
import os
import socket
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import tun_probe  # noqa: E402


def _pack(dgrams):
    offs = np.zeros(len(dgrams) + 1, np.uint64)
    offs[1:] = np.cumsum([len(d) for d in dgrams])
    return np.frombuffer(b"".join(dgrams), np.uint8), offs


def main(out=os.path.join(HERE, "kernel_verified.npz")):
    rng = np.random.default_rng(2026)
    rb = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()  # noqa: E731
    p = tun_probe.Probe()
    try:
        for seq, n in enumerate([0, 1, 2, 3, 7, 8, 55, 56, 63, 64, 65, 127, 255, 511, 999, 1400, 1472]):
            assert p.ping(0x5959, seq, rb(n)), n
        sizes = [1, 2, 3, 5, 63, 64, 65, 511, 1000, 1399, 1400] + [int(x) for x in rng.integers(1, 1401, 20)]
        payloads = [rb(n) for n in sizes]
        r = p.tcp_session(24680, payloads)
        assert r["synack"] and r["received"] == b"".join(payloads)
        udp = [rb(n) for n in (1, 2, 3, 7, 8, 63, 64, 65, 511, 1000, 1472)]
        assert p.kernel_udp(udp) == len(udp)
        assert p.oracle_mismatch == 0 and p.bad_replies == 0
    finally:
        p.close()
    # the closing RST is not answered, so nothing shows the kernel took it
    sent = [d for d in p.sent_ok if not (d[9] == 6 and d[20 + 13] & tun_probe.RST)]
    sb, so = _pack(sent)
    kb, ko = _pack(p.from_kernel)
    np.savez(out, sent_blob=sb, sent_offs=so, kernel_blob=kb, kernel_offs=ko)
    protos = lambda ds: {pr: sum(1 for d in ds if d[9] == pr) for pr in (1, 6, 17)}  # noqa: E731
    print(f"{out}: {len(sent)} accepted datagrams {protos(sent)}, {len(p.from_kernel)} kernel "
          f"datagrams {protos(p.from_kernel)}")


if __name__ == "__main__":
    main()

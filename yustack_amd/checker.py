"""Verification semantics of the reference's test-only ``checker`` package.

``checker.IPv4`` (checker/checker.go:25-40) and ``checker.TCP`` (:71-99) are the only
place the reference *verifies* a checksum: a packet is valid iff the sum over the
header/segment INCLUDING the stored field (plus pseudo-header and length for TCP) is
0 or 0xFFFF. The scalar functions below restate that with the scalar C ABI; the
batched GPU form is ``yustack_amd.batch`` modes VERIFY_IPV4 / VERIFY_TCP / VERIFY_UDP.
"""
from __future__ import annotations

from .checksum import Checksum
from .header import IPv4, TCP


class CheckError(AssertionError):
    pass


def valid_sum(x: int) -> bool:
    return x == 0 or x == 0xFFFF


def check_ipv4(b: bytes) -> int:
    """checker/checker.go:25-35. Returns the verified sum; raises CheckError."""
    ip = IPv4(bytearray(b))
    if len(b) < 20 or ip.HeaderLength() > len(b):
        raise CheckError("Not a valid IPv4 packet")
    xsum = ip.CalculateChecksum()
    if not valid_sum(xsum):
        raise CheckError(f"Bad checksum: 0x{xsum:x}, checksum in packet: 0x{ip.Checksum():x}")
    return xsum


def transport_sum(b: bytes) -> int:
    """checker/checker.go:80-88 — pseudo ‖ len ‖ segment for the IPv4 packet b."""
    ip = IPv4(bytearray(b))
    seg = bytes(ip.Payload())
    l = len(seg) & 0xFFFF
    xsum = Checksum(ip.SourceAddress(), 0)
    xsum = Checksum(ip.DestinationAddress(), xsum)
    xsum = Checksum(bytes([0, ip.Protocol()]), xsum)
    xsum = Checksum(bytes([l >> 8, l & 0xFF]), xsum)
    return Checksum(seg, xsum)


def check_tcp(b: bytes) -> int:
    """checker/checker.go:71-99 (protocol and checksum parts)."""
    check_ipv4(b)
    ip = IPv4(bytearray(b))
    if ip.Protocol() != 6:
        raise CheckError(f"Bad protocol, got {ip.Protocol()}, want 6")
    xsum = transport_sum(b)
    if not valid_sum(xsum):
        raise CheckError(f"Bad checksum: 0x{xsum:x}, checksum in segment: "
                         f"0x{TCP(bytearray(ip.Payload())).Checksum():x}")
    return xsum

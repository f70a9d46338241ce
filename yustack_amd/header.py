"""Checksum-facing subset of yustack's ``header`` package, over Python bytearrays.

Only the methods on the checksum path (SURVEY.md §8a rows A5–A8) plus the ``Encode``
helpers needed to lay packets out the way the reference does; field parsing and TCP
option handling are out of scope. Every ``CalculateChecksum`` calls the C ABI
through :mod:`yustack_amd.checksum`, exactly as the Go methods call package
``checksum``:

* ``IPv4.CalculateChecksum``  header/ipv4.go:177-179 (``HeaderLength`` :91-93)
* ``TCP.CalculateChecksum``   header/tcp.go:165-173 (``DataOffset``, ``Encode`` :176-186)
* ``UDP.CalculateChecksum``   header/udp.go:67-75 (``Encode`` :78-83)
* ``ICMPv4.SetChecksum``      header/icmpv4.go:46-48
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

from .checksum import Checksum

IPv4MinimumSize = 20
TCPMinimumSize = 20
UDPMinimumSize = 8
ICMPv4MinimumSize = 4
IPv4ProtocolNumber = 0x0800
TCPProtocolNumber = 6
UDPProtocolNumber = 17
ICMPv4ProtocolNumber = 1


class IPv4:
    """header/ipv4.go — view over a bytearray starting at the IPv4 header."""

    def __init__(self, b: bytearray, off: int = 0):
        self.b, self.o = b, off

    def HeaderLength(self) -> int:  # noqa: N802
        return (self.b[self.o] & 0xF) * 4

    def TotalLength(self) -> int:  # noqa: N802
        return struct.unpack_from(">H", self.b, self.o + 2)[0]

    def Protocol(self) -> int:  # noqa: N802
        return self.b[self.o + 9]

    def Checksum(self) -> int:  # noqa: N802
        return struct.unpack_from(">H", self.b, self.o + 10)[0]

    def SetChecksum(self, v: int) -> None:  # noqa: N802
        struct.pack_into(">H", self.b, self.o + 10, v & 0xFFFF)

    def SourceAddress(self) -> bytes:  # noqa: N802
        return bytes(self.b[self.o + 12: self.o + 16])

    def DestinationAddress(self) -> bytes:  # noqa: N802
        return bytes(self.b[self.o + 16: self.o + 20])

    def Payload(self) -> bytearray:  # noqa: N802
        return self.b[self.o + self.HeaderLength(): self.o + self.TotalLength()]

    def CalculateChecksum(self) -> int:  # noqa: N802
        """header/ipv4.go:177-179"""
        return Checksum(bytes(self.b[self.o: self.o + self.HeaderLength()]), 0)

    def Encode(self, IHL: int, TotalLength: int, Protocol: int, SrcAddr: bytes, DstAddr: bytes,  # noqa: N803
               TTL: int = 64, TOS: int = 0, ID: int = 0, Flags: int = 0, FragmentOffset: int = 0,
               Checksum: int = 0) -> None:
        """header/ipv4.go:146-157"""
        b, o = self.b, self.o
        b[o] = (4 << 4) | ((IHL // 4) & 0xF)
        b[o + 1] = TOS
        struct.pack_into(">HH", b, o + 2, TotalLength, ID)
        struct.pack_into(">H", b, o + 6, ((Flags << 13) | (FragmentOffset >> 3)) & 0xFFFF)
        b[o + 8] = TTL
        b[o + 9] = Protocol
        struct.pack_into(">H", b, o + 10, Checksum)
        b[o + 12: o + 16] = SrcAddr
        b[o + 16: o + 20] = DstAddr


class TCP:
    """header/tcp.go"""

    def __init__(self, b: bytearray, off: int = 0):
        self.b, self.o = b, off

    def DataOffset(self) -> int:  # noqa: N802
        return (self.b[self.o + 12] >> 4) * 4

    def Checksum(self) -> int:  # noqa: N802
        return struct.unpack_from(">H", self.b, self.o + 16)[0]

    def SetChecksum(self, v: int) -> None:  # noqa: N802
        struct.pack_into(">H", self.b, self.o + 16, v & 0xFFFF)

    def CalculateChecksum(self, partialChecksum: int, totalLen: int) -> int:  # noqa: N802,N803
        """header/tcp.go:165-173"""
        cksm = Checksum(struct.pack(">H", totalLen & 0xFFFF), partialChecksum)
        return Checksum(bytes(self.b[self.o: self.o + self.DataOffset()]), cksm)

    def Encode(self, SrcPort: int, DstPort: int, SeqNum: int, AckNum: int, DataOffset: int,  # noqa: N803
               Flags: int, WindowSize: int, Checksum: int = 0, UrgentPointer: int = 0) -> None:
        """header/tcp.go:176-186"""
        b, o = self.b, self.o
        struct.pack_into(">HHII", b, o, SrcPort, DstPort, SeqNum & 0xFFFFFFFF, AckNum & 0xFFFFFFFF)
        b[o + 12] = ((DataOffset // 4) << 4) & 0xFF
        b[o + 13] = Flags & 0xFF
        struct.pack_into(">HHH", b, o + 14, WindowSize & 0xFFFF, Checksum, UrgentPointer)


class UDP:
    """header/udp.go"""

    def __init__(self, b: bytearray, off: int = 0):
        self.b, self.o = b, off

    def Length(self) -> int:  # noqa: N802
        return struct.unpack_from(">H", self.b, self.o + 4)[0]

    def Checksum(self) -> int:  # noqa: N802
        return struct.unpack_from(">H", self.b, self.o + 6)[0]

    def SetChecksum(self, v: int) -> None:  # noqa: N802
        struct.pack_into(">H", self.b, self.o + 6, v & 0xFFFF)

    def CalculateChecksum(self, partialChecksum: int, totalLength: int) -> int:  # noqa: N802,N803
        """header/udp.go:67-75"""
        c = Checksum(struct.pack(">H", totalLength & 0xFFFF), partialChecksum)
        return Checksum(bytes(self.b[self.o: self.o + UDPMinimumSize]), c)

    def Encode(self, SrcPort: int, DstPort: int, Length: int, Checksum: int = 0) -> None:  # noqa: N803
        """header/udp.go:78-83"""
        struct.pack_into(">HHHH", self.b, self.o, SrcPort, DstPort, Length, Checksum)


class ICMPv4:
    """header/icmpv4.go"""

    def __init__(self, b: bytearray, off: int = 0):
        self.b, self.o = b, off

    def SetType(self, t: int) -> None:  # noqa: N802
        self.b[self.o] = t

    def SetCode(self, c: int) -> None:  # noqa: N802
        self.b[self.o + 1] = c

    def Checksum(self) -> int:  # noqa: N802
        return struct.unpack_from(">H", self.b, self.o + 2)[0]

    def SetChecksum(self, v: int) -> None:  # noqa: N802
        struct.pack_into(">H", self.b, self.o + 2, v & 0xFFFF)


@dataclass
class Route:
    """The two fields of types.Route that the checksum path reads (types/route.go:90-92)."""
    LocalAddress: bytes
    RemoteAddress: bytes

    def PseudoHeaderChecksum(self, protocol: int) -> int:  # noqa: N802
        from .checksum import PseudoHeaderChecksum
        return PseudoHeaderChecksum(protocol, self.LocalAddress, self.RemoteAddress)

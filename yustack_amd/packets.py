"""Scalar packet composition, mirroring the reference's send paths call for call.

These are the compositions the batched TX modes reproduce on the GPU; they run on
the host through the scalar C ABI, like the reference runs them per packet:

* :func:`send_udp`    transport/udp/endpoint.go:164-187 (sendUDP) + network/ipv4/ipv4.go:80-97
* :func:`send_tcp`    transport/tcp/connect.go:556-586 (sendTCP), :288-322 (with options)
* :func:`send_icmpv4` network/ipv4/icmp.go:36-45 (sendICMPv4)
* :func:`ipv4_write`  network/ipv4/ipv4.go:80-97 (endpoint.WritePacket)

and the test harnesses' inbound builders:

* :func:`tcp_test_packet` transport/tcp/testing/context/context.go:164-209 (SendPacket)
* :func:`udp_test_packet` transport/udp/udp_test.go:105-144 (sendPacket)
"""
from __future__ import annotations

from .checksum import Checksum
from .header import (ICMPv4, ICMPv4MinimumSize, IPv4, IPv4MinimumSize, Route, TCP, TCPMinimumSize,
                     TCPProtocolNumber, UDP, UDPMinimumSize, UDPProtocolNumber, ICMPv4ProtocolNumber)


def ipv4_write(r: Route, transport_hdr: bytes, payload: bytes, protocol: int) -> bytearray:
    """network/ipv4/ipv4.go:80-97: prepend the IPv4 header (IHL 20, TTL 64, ID 0) and
    set its checksum."""
    b = bytearray(IPv4MinimumSize) + bytearray(transport_hdr) + bytearray(payload)
    ip = IPv4(b)
    ip.Encode(IHL=IPv4MinimumSize, TotalLength=len(b), ID=0, TTL=64, Protocol=protocol,
              SrcAddr=r.LocalAddress, DstAddr=r.RemoteAddress)
    ip.SetChecksum(~ip.CalculateChecksum() & 0xFFFF)
    return b


def send_udp(r: Route, data: bytes | None, local_port: int, remote_port: int) -> bytearray:
    """transport/udp/endpoint.go:164-187"""
    hdr = bytearray(UDPMinimumSize)
    udp = UDP(hdr)
    length = UDPMinimumSize
    xsum = r.PseudoHeaderChecksum(UDPProtocolNumber)
    if data is not None:
        length = (length + len(data)) & 0xFFFF
        xsum = Checksum(data, xsum)
    udp.Encode(SrcPort=local_port, DstPort=remote_port, Length=length)
    udp.SetChecksum(~udp.CalculateChecksum(xsum, length) & 0xFFFF)
    return ipv4_write(r, bytes(hdr), data or b"", UDPProtocolNumber)


def send_tcp(r: Route, local_port: int, remote_port: int, data: bytes | None, flags: int,
             seq: int, ack: int, rcv_wnd: int, options: bytes = b"") -> bytearray:
    """transport/tcp/connect.go:556-586 (options form: :288-322)"""
    hdr = bytearray(TCPMinimumSize + len(options))
    hdr[TCPMinimumSize:] = options
    rcv_wnd = min(rcv_wnd, 0xFFFF)
    tcp = TCP(hdr)
    tcp.Encode(SrcPort=local_port, DstPort=remote_port, SeqNum=seq, AckNum=ack,
               DataOffset=TCPMinimumSize + len(options), Flags=flags, WindowSize=rcv_wnd)
    length = len(hdr)
    xsum = r.PseudoHeaderChecksum(TCPProtocolNumber)
    if data is not None:
        length = (length + len(data)) & 0xFFFF
        xsum = Checksum(data, xsum)
    tcp.SetChecksum(~tcp.CalculateChecksum(xsum, length) & 0xFFFF)
    return ipv4_write(r, bytes(hdr), data or b"", TCPProtocolNumber)


def send_icmpv4(r: Route, typ: int, code: int, data: bytes) -> bytearray:
    """network/ipv4/icmp.go:36-45"""
    hdr = bytearray(ICMPv4MinimumSize)
    icmp = ICMPv4(hdr)
    icmp.SetType(typ)
    icmp.SetCode(code)
    icmp.SetChecksum(~Checksum(bytes(hdr), Checksum(data, 0)) & 0xFFFF)
    return ipv4_write(r, bytes(hdr), data, ICMPv4ProtocolNumber)


def tcp_test_packet(payload: bytes, src_port: int, dst_port: int, seq: int, ack: int, flags: int,
                    rcv_wnd: int, tcp_opts: bytes = b"",
                    test_addr: bytes = b"\x0a\x00\x00\x02",
                    stack_addr: bytes = b"\x0a\x00\x00\x01") -> bytearray:
    """transport/tcp/testing/context/context.go:164-209 (Context.SendPacket)"""
    buf = bytearray(TCPMinimumSize + IPv4MinimumSize + len(tcp_opts) + len(payload))
    buf[len(buf) - len(payload):] = payload
    buf[len(buf) - len(payload) - len(tcp_opts): len(buf) - len(payload)] = tcp_opts
    ip = IPv4(buf)
    ip.Encode(IHL=IPv4MinimumSize, TotalLength=len(buf), TTL=64, Protocol=TCPProtocolNumber,
              SrcAddr=test_addr, DstAddr=stack_addr)
    ip.SetChecksum(~ip.CalculateChecksum() & 0xFFFF)
    t = TCP(buf, IPv4MinimumSize)
    t.Encode(SrcPort=src_port, DstPort=dst_port, SeqNum=seq, AckNum=ack,
             DataOffset=TCPMinimumSize + len(tcp_opts), Flags=flags, WindowSize=rcv_wnd & 0xFFFF)
    xsum = Checksum(test_addr, 0)
    xsum = Checksum(stack_addr, xsum)
    xsum = Checksum(bytes([0, TCPProtocolNumber]), xsum)
    length = TCPMinimumSize + len(tcp_opts) + len(payload)
    xsum = Checksum(payload, xsum)
    t.SetChecksum(~t.CalculateChecksum(xsum, length) & 0xFFFF)
    return buf


def udp_test_packet(payload: bytes, src_port: int, dst_port: int,
                    test_addr: bytes = b"\x0a\x01\x00\x01",
                    stack_addr: bytes = b"\x0a\x01\x00\x02") -> bytearray:
    """transport/udp/udp_test.go:105-144 (testContext.sendPacket)"""
    buf = bytearray(UDPMinimumSize + IPv4MinimumSize + len(payload))
    buf[len(buf) - len(payload):] = payload
    ip = IPv4(buf)
    ip.Encode(IHL=IPv4MinimumSize, TotalLength=len(buf), TTL=64, Protocol=UDPProtocolNumber,
              SrcAddr=test_addr, DstAddr=stack_addr)
    ip.SetChecksum(~ip.CalculateChecksum() & 0xFFFF)
    u = UDP(buf, IPv4MinimumSize)
    u.Encode(SrcPort=src_port, DstPort=dst_port, Length=UDPMinimumSize + len(payload))
    xsum = Checksum(test_addr, 0)
    xsum = Checksum(stack_addr, xsum)
    xsum = Checksum(bytes([0, UDPProtocolNumber]), xsum)
    length = UDPMinimumSize + len(payload)
    xsum = Checksum(payload, xsum)
    u.SetChecksum(~u.CalculateChecksum(xsum, length) & 0xFFFF)
    return buf

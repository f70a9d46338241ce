"""BASELINE config 1 harness: sample/tun_udp_echo's data path over a real tun device,
with the Linux kernel as the independent checker (TEST INFRASTRUCTURE).

The reference sample (sample/tun_udp_echo/main.go) runs yustack on a tun device at
10.1.0.1 and echoes every UDP datagram sent to port 12345. Its per-datagram checksum
work is what this repo replaces: on receive, nothing (the reference does not verify,
network/ipv4/ipv4.go:62-77, transport/udp/endpoint.go:191-229); on send,
sendUDP's UDP checksum and ipv4.WritePacket's header checksum
(transport/udp/endpoint.go:164-187, network/ipv4/ipv4.go:80-97).

This harness keeps exactly that data path and nothing else of the stack (sockets,
routing and the state machines are out of scope):

* the echo thread reads whole IPv4 datagrams from the tun fd, checks them with this
  repo's checker mirror (the kernel computed those checksums), and answers each
  with yustack_amd.packets.send_udp — the sendUDP + WritePacket composition over the
  scalar C ABI (yu_checksum / yu_pseudo_header_checksum, the cgo shim's targets);
* a UDP socket in the kernel sends the datagrams and receives the echoes. Linux
  verifies the UDP checksum of every echo before delivering it (a tun frame arrives
  CHECKSUM_NONE), so each received echo is a kernel-verified checksum.

Needs CAP_NET_ADMIN (tun creation and interface setup through ioctls; no `ip` tool
is needed). Callers skip when that is refused.
"""
from __future__ import annotations

import fcntl
import os
import select
import socket
import struct
import threading
import time

from yustack_amd import checker, packets
from yustack_amd.header import IPv4, Route

TUNSETIFF = 0x400454CA
IFF_TUN, IFF_NO_PI = 0x0001, 0x1000
SIOCSIFADDR, SIOCSIFNETMASK, SIOCGIFFLAGS, SIOCSIFFLAGS = 0x8916, 0x891C, 0x8913, 0x8914
IFF_UP, IFF_RUNNING = 0x1, 0x40

STACK_ADDR = "10.1.0.1"   # sample/tun_udp_echo/main.go:18 (stackAddr)
STACK_PORT = 12345        # :19 (stackPort)
HOST_ADDR = "10.1.0.10"   # the kernel side of the tun link


def _ifreq_addr(name: bytes, addr: str) -> bytes:
    sin = struct.pack("HH4s8x", socket.AF_INET, 0, socket.inet_aton(addr))
    return struct.pack("16s16s", name, sin)


def open_tun(name: str) -> tuple[int, str]:
    """Create a tun device and configure HOST_ADDR/24 on it (raises OSError when
    the sandbox refuses)."""
    fd = os.open("/dev/net/tun", os.O_RDWR)
    try:
        ifr = fcntl.ioctl(fd, TUNSETIFF, struct.pack("16sH", name.encode(), IFF_TUN | IFF_NO_PI))
        real = ifr[:16].rstrip(b"\0")
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            fcntl.ioctl(s, SIOCSIFADDR, _ifreq_addr(real, HOST_ADDR))
            fcntl.ioctl(s, SIOCSIFNETMASK, _ifreq_addr(real, "255.255.255.0"))
            flags = struct.unpack("16sH", fcntl.ioctl(s, SIOCGIFFLAGS, struct.pack("16sH", real, 0))[:18])[1]
            fcntl.ioctl(s, SIOCSIFFLAGS, struct.pack("16sH", real, flags | IFF_UP | IFF_RUNNING))
        finally:
            s.close()
        return fd, real.decode()
    except Exception:
        os.close(fd)
        raise


class Echo(threading.Thread):
    """The echo side: tun frames in, sendUDP-built replies out."""

    def __init__(self, fd: int, corrupt_every: int = 0):
        super().__init__(daemon=True)
        self.fd, self.corrupt_every = fd, corrupt_every
        self.stop = threading.Event()
        self.seen = self.echoed = self.bad_in = self.corrupted = 0
        self.stack = socket.inet_aton(STACK_ADDR)

    def run(self):
        while not self.stop.is_set():
            r, _, _ = select.select([self.fd], [], [], 0.05)
            if not r:
                continue
            pkt = os.read(self.fd, 65535)
            if len(pkt) < 28 or pkt[0] >> 4 != 4:
                continue  # not IPv4 (e.g. router solicitations are IPv6)
            ip = IPv4(bytearray(pkt))
            if ip.Protocol() != 17 or ip.DestinationAddress() != self.stack:
                continue
            self.seen += 1
            # the kernel filled these checksums: the checker semantics
            # (checker/checker.go:32-35,80-92) over our scalar path must accept them
            if not (checker.valid_sum(ip.CalculateChecksum()) and
                    checker.valid_sum(checker.transport_sum(pkt))):
                self.bad_in += 1
            hl = ip.HeaderLength()
            src_port, dst_port = struct.unpack_from(">HH", pkt, hl)
            if dst_port != STACK_PORT:
                continue
            payload = pkt[hl + 8: ip.TotalLength()]
            r = Route(LocalAddress=self.stack, RemoteAddress=ip.SourceAddress())
            reply = packets.send_udp(r, payload, STACK_PORT, src_port)
            if self.corrupt_every and self.seen % self.corrupt_every == 0:
                reply[26] ^= 0x01  # damage the UDP checksum: the kernel must drop it
                self.corrupted += 1
            os.write(self.fd, bytes(reply))
            self.echoed += 1


def run_echo(n: int, size: int = 64, name: str = "yuecho%d", corrupt_every: int = 0,
             timeout: float = 0.5) -> dict:
    """Send n datagrams of `size` bytes to the echo, one at a time (the sample's
    request/response pattern), and count the kernel-verified echoes."""
    fd, ifname = open_tun(name)
    echo = Echo(fd, corrupt_every)
    echo.start()
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind((HOST_ADDR, 0))
    s.settimeout(timeout)
    got = lost = mismatched = 0
    t0 = time.perf_counter()
    try:
        for i in range(n):
            msg = struct.pack(">I", i) + os.urandom(size - 4)
            s.sendto(msg, (STACK_ADDR, STACK_PORT))
            try:
                back, peer = s.recvfrom(65535)
            except socket.timeout:
                lost += 1
                continue
            got += 1
            if back != msg or peer != (STACK_ADDR, STACK_PORT):
                mismatched += 1
    finally:
        dt = time.perf_counter() - t0
        echo.stop.set()
        echo.join(2)
        s.close()
        os.close(fd)
    return {"interface": ifname, "sent": n, "echoed_verified_by_kernel": got, "lost": lost,
            "mismatched": mismatched, "seen_by_echo": echo.seen, "bad_inbound_checksums": echo.bad_in,
            "corrupted_on_purpose": echo.corrupted, "seconds": dt,
            "round_trips_per_s": got / dt if dt else 0.0}


if __name__ == "__main__":
    import json
    print(json.dumps(run_echo(20000)))

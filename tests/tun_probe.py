"""The Linux kernel as an independent checker of TCP, ICMP and IPv4 checksums
(TEST INFRASTRUCTURE; tests/test_tun_probe.py).

tests/tun_echo.py lets the kernel verify the UDP path (sendUDP + WritePacket). This
harness covers the other send compositions the batched TX modes reproduce, by
writing datagrams built with them into a tun device, addressed to the kernel's own
address on the link (HOST_ADDR), and watching what the kernel answers:

* ICMP: an echo request built with ``packets.send_icmpv4`` (sendICMPv4,
  network/ipv4/icmp.go:36-45) gets an echo reply only if the kernel's icmp_rcv
  accepted its checksum (and ip_rcv the IPv4 header's, ipv4.WritePacket,
  network/ipv4/ipv4.go:80-97);
* TCP: a SYN built with ``packets.send_tcp`` (sendTCP, transport/tcp/connect.go:556-586)
  to a listening kernel socket gets a SYN-ACK only if tcp_v4_rcv accepted its
  checksum; after the handshake, data segments of any length reach the accepted
  socket only if their checksums pass (a tun frame arrives CHECKSUM_NONE, so the
  kernel verifies every one in software).

Damaged datagrams must go unanswered. Every datagram the kernel accepted is also
checked against the C oracle's TX_DATAGRAM fields, and every datagram the kernel sent
back against the oracle's VERIFY_RX: the oracle is what the GPU parity tests pin the
HIP kernels to, so this ties the kernel's verdict to theirs.

Needs CAP_NET_ADMIN; callers skip when tun creation is refused.
"""
from __future__ import annotations

import os
import select
import socket
import struct
import time

import numpy as np

from oracle import oracle as O
from tun_echo import HOST_ADDR, STACK_ADDR, open_tun
from yustack_amd import packets
from yustack_amd.header import Route

SYN, ACK, PSH, RST = 0x02, 0x10, 0x08, 0x04
RX_OK = 0x2 | 0x4  # YU_RX_IP_OK | YU_RX_L4_OK (include/yucsum.h)


def oracle_fields(dgram: bytes) -> tuple[int, int]:
    """The oracle's TX_DATAGRAM values ({IPv4 field, transport field}) for a datagram,
    computed with both fields left out."""
    out = O.C().batch(np.frombuffer(bytes(dgram), np.uint8), O.MODE_TX_DATAGRAM,
                      stride=len(dgram), length=len(dgram), n=1)
    return int(out[0]), int(out[1])


def oracle_rx(dgram: bytes) -> int:
    """The oracle's VERIFY_RX result bits for a received datagram."""
    return int(O.C().batch(np.frombuffer(bytes(dgram), np.uint8), O.MODE_VERIFY_RX,
                           stride=len(dgram), length=len(dgram), n=1)[0])


def stored_fields(dgram: bytes) -> tuple[int, int]:
    """The IPv4 and transport checksum fields a datagram carries."""
    hl = (dgram[0] & 0xF) * 4
    fo = {6: 16, 17: 6, 1: 2}[dgram[9]]
    return (struct.unpack_from(">H", dgram, 10)[0], struct.unpack_from(">H", dgram, hl + fo)[0])


class Probe:
    """One tun link: datagrams in from the stack side, the kernel's answers out."""

    def __init__(self, name: str = "yuprobe%d"):
        self.fd, self.ifname = open_tun(name)
        self.stack, self.host = socket.inet_aton(STACK_ADDR), socket.inet_aton(HOST_ADDR)
        self.route = Route(LocalAddress=self.stack, RemoteAddress=self.host)
        self.sent = self.oracle_mismatch = self.bad_replies = 0
        # what the fixture generator keeps (tests/golden/make_kernel_verified.py)
        self.sent_ok: list[bytes] = []      # undamaged datagrams written to the kernel
        self.from_kernel: list[bytes] = []  # datagrams the kernel wrote back

    def close(self) -> None:
        os.close(self.fd)

    def _send(self, dgram: bytearray, corrupt_at: int | None) -> None:
        if corrupt_at is None:
            if stored_fields(dgram) != oracle_fields(dgram):
                self.oracle_mismatch += 1
            self.sent_ok.append(bytes(dgram))
        else:
            dgram[corrupt_at] ^= 0x01
        os.write(self.fd, bytes(dgram))
        self.sent += 1

    def _recv(self, want, timeout: float) -> bytes | None:
        end = time.monotonic() + timeout
        while (left := end - time.monotonic()) > 0:
            r, _, _ = select.select([self.fd], [], [], left)
            if not r:
                continue
            pkt = os.read(self.fd, 65535)
            if len(pkt) >= 20 and pkt[0] >> 4 == 4 and pkt[16:20] == self.stack and want(pkt):
                if oracle_rx(pkt) & RX_OK != RX_OK:
                    self.bad_replies += 1
                self.from_kernel.append(pkt)
                return pkt
        return None

    # ICMP --------------------------------------------------------------
    def ping(self, ident: int, seq: int, payload: bytes, corrupt_at: int | None = None,
             timeout: float = 0.5) -> bool:
        """An echo request from sendICMPv4; True when the kernel's echo reply came back
        with the same identifier, sequence number and payload. corrupt_at: a byte to
        damage (10/11: the IPv4 field, 22/23: the ICMP field)."""
        data = struct.pack(">HH", ident, seq) + payload
        self._send(packets.send_icmpv4(self.route, 8, 0, data), corrupt_at)
        rep = self._recv(lambda p: p[9] == 1 and p[20] == 0 and p[24:28] == data[:4], timeout)
        return rep is not None and rep[28:struct.unpack_from(">H", rep, 2)[0]] == payload

    # UDP ---------------------------------------------------------------
    def kernel_udp(self, payloads: list[bytes], port: int = 12345, timeout: float = 0.5) -> int:
        """Datagrams a kernel UDP socket sends to the stack side (their checksums are
        the kernel's); returns how many came through the tun."""
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            s.bind((HOST_ADDR, 0))
            got = 0
            for data in payloads:
                s.sendto(data, (STACK_ADDR, port))
                if self._recv(lambda p: p[9] == 17 and p[28:] == data, timeout) is not None:
                    got += 1
            return got
        finally:
            s.close()

    # TCP ---------------------------------------------------------------
    def tcp_session(self, port: int, payloads: list[bytes], corrupt_syn: bool = False,
                    timeout: float = 1.0) -> dict:
        """Handshake with a listening kernel socket on HOST_ADDR:port, then the payloads
        as PSH|ACK data segments from sendTCP; returns what the accepted socket read."""
        ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        ls.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        ls.bind((HOST_ADDR, port))
        ls.listen(1)
        ls.settimeout(timeout)
        sport, iss = 40000 + port % 1000, 0x1000_0000 + port
        res = {"synack": False, "received": b"", "acked": 0}
        conn = None
        try:
            self._send(packets.send_tcp(self.route, sport, port, None, SYN, iss, 0, 65535),
                       36 if corrupt_syn else None)
            synack = self._recv(lambda p: p[9] == 6 and p[33] & (SYN | ACK) == SYN | ACK, timeout)
            if synack is None:
                return res
            res["synack"] = True
            irs = struct.unpack_from(">I", synack, 24)[0]
            snd, rcv = iss + 1, irs + 1
            self._send(packets.send_tcp(self.route, sport, port, None, ACK, snd, rcv, 65535), None)
            conn, _ = ls.accept()
            conn.settimeout(timeout)
            for data in payloads:
                self._send(packets.send_tcp(self.route, sport, port, data, PSH | ACK, snd, rcv, 65535), None)
                snd += len(data)
                ack = self._recv(lambda p: p[9] == 6 and p[33] & ACK and
                                 struct.unpack_from(">I", p, 28)[0] == snd & 0xFFFFFFFF, timeout)
                if ack is not None:
                    res["acked"] += 1
            want = sum(len(d) for d in payloads)
            buf = b""
            while len(buf) < want:
                try:
                    chunk = conn.recv(65536)
                except socket.timeout:
                    break
                if not chunk:
                    break
                buf += chunk
            res["received"] = buf
            # end the session without a FIN exchange
            self._send(packets.send_tcp(self.route, sport, port, None, RST | ACK, snd, rcv, 0), None)
            return res
        except socket.timeout:
            return res
        finally:
            if conn is not None:
                conn.close()
            ls.close()

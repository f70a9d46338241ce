"""The Linux kernel verifies the TCP, ICMP and IPv4 checksums of datagrams built by
this repo's send compositions (sendTCP, sendICMPv4, ipv4.WritePacket over the scalar
C ABI), and every accepted datagram's fields equal the C oracle's TX_DATAGRAM values
(tests/tun_probe.py). CPU only; skipped where creating a tun device is refused (the
GPU boxes run unprivileged)."""
import os

import numpy as np
import pytest

import tun_probe


@pytest.fixture
def probe():
    try:
        p = tun_probe.Probe()
    except OSError as e:  # no /dev/net/tun or no CAP_NET_ADMIN here
        pytest.skip(f"tun device unavailable: {e}")
    yield p
    p.close()


@pytest.mark.parametrize("size", [0, 1, 2, 7, 56, 63, 64, 999, 1400, 1472])
def test_icmp_echo_kernel_verified(probe, size):
    for seq in range(10):
        assert probe.ping(0x4242, seq, os.urandom(size)), (size, seq)
    assert probe.oracle_mismatch == 0 and probe.bad_replies == 0


@pytest.mark.parametrize("at", [10, 11, 22, 23])
def test_damaged_icmp_or_ipv4_field_is_dropped(probe, at):
    assert not probe.ping(0x4343, 1, os.urandom(33), corrupt_at=at, timeout=0.3)
    assert probe.ping(0x4343, 2, os.urandom(33))  # the same link still answers


def test_tcp_handshake_and_segments_kernel_verified(probe):
    rng = np.random.default_rng(5)
    sizes = [1, 2, 3, 63, 64, 65, 511, 1000, 1399, 1400] + [int(x) for x in rng.integers(1, 1401, 30)]
    payloads = [os.urandom(n) for n in sizes]
    r = probe.tcp_session(23456, payloads)
    assert r["synack"], r
    assert r["received"] == b"".join(payloads), (len(r["received"]), sum(sizes))
    assert probe.oracle_mismatch == 0 and probe.bad_replies == 0


def test_damaged_tcp_syn_is_dropped(probe):
    r = probe.tcp_session(23457, [], corrupt_syn=True, timeout=0.4)
    assert not r["synack"]
    assert probe.tcp_session(23458, [b"after"])["received"] == b"after"

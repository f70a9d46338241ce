"""BASELINE config 1 (sample/tun_udp_echo over a tun device) with the Linux kernel as
the checker: every echo the kernel delivers passed its UDP checksum verification, and
every deliberately damaged one is dropped (tests/tun_echo.py). CPU only; skipped where
creating a tun device is refused (the GPU boxes run unprivileged)."""
import pytest

import tun_echo


def _run(*a, **k):
    try:
        return tun_echo.run_echo(*a, **k)
    except OSError as e:  # no /dev/net/tun or no CAP_NET_ADMIN here
        pytest.skip(f"tun device unavailable: {e}")


@pytest.mark.parametrize("size", [64, 5, 63, 1400])
def test_udp_echo_kernel_verified(size):
    r = _run(400, size=size)
    assert r["echoed_verified_by_kernel"] == 400 and r["lost"] == 0 and r["mismatched"] == 0, r
    assert r["bad_inbound_checksums"] == 0, r  # the kernel's checksums pass our checker


def test_damaged_checksums_are_dropped_by_kernel():
    r = _run(60, corrupt_every=10, timeout=0.2)
    assert r["corrupted_on_purpose"] == 6
    assert r["lost"] == 6 and r["echoed_verified_by_kernel"] == 54, r

"""GPU parity: the HIP kernels (through the C ABI) against the C oracle, bit-exact.

Small cases cover every mode × layout × alignment × edge length; the full BASELINE
configs (2, 3, 4) are compared packet-for-packet against the multithreaded C oracle
on the same bytes.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O
from yustack_amd import batch

# a measurement run that forces the ragged kernel (YU_TUNING=1 YU_RAGGED=...) checks
# parity only: the default ragged kernel choice is not asserted then. The library
# reads its knobs only under the YU_TUNING=1 gate, and so do these flags.
TUNING = os.environ.get("YU_TUNING") == "1"
FORCED = TUNING and bool(os.environ.get("YU_RAGGED"))
# TX_DATAGRAM in place from 64K datagrams on: 40-packet chunks
DG_FILL_CH = 40
DG_FILL = f"k_seg<8,dg,c{DG_FILL_CH}>"

pytestmark = pytest.mark.gpu

EDGE_LENS = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 20, 31, 32, 33, 60, 63, 64, 65, 127, 128, 129,
             255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 1499, 1500, 1501, 1535, 1536, 2047,
             2048, 2049, 3071, 3072, 4095, 4096, 4097, 8999, 9000, 9001]


def _to(dev, a):
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:  # e.g. golden vectors from np.frombuffer
        a = a.copy()
    return torch.from_numpy(a).to(dev)


def _rand(rng, n, kind="rand"):
    if kind == "zero":
        return np.zeros(n, np.uint8)
    if kind == "ff":
        return np.full(n, 255, np.uint8)
    return rng.integers(0, 256, size=n, dtype=np.uint8)


def _uniform_case(dev, oracle_c, rng, length, stride, n, mode, base_off=0, kind="rand",
                  use_addrs=False, use_init_arr=False, initial=0):
    total = base_off + (n - 1) * stride + length + 64
    host = _rand(rng, total, kind)
    if mode in (O.MODE_TCP, O.MODE_VERIFY_TCP) and length >= 20:
        for p in range(n):  # DataOffset in [20, min(60, len)], a multiple of 4
            doff = 4 * int(rng.integers(5, min(60, length) // 4 + 1))
            host[base_off + p * stride + 12] = (doff // 4) << 4
    if mode in (O.MODE_IPV4, O.MODE_VERIFY_IPV4) and length >= 1:
        for p in range(n):
            ihl = int(rng.integers(0, 16))
            host[base_off + p * stride] = 0x40 | ihl if ihl * 4 <= length else 0x40 | (length // 4)
    addrs = _rand(rng, 8 * n) if use_addrs else None
    init = rng.integers(0, 65536, size=n, dtype=np.uint16) if use_init_arr else None
    d = _to(dev, host)
    view = d[base_off:]
    got = batch.checksum_uniform(view, stride, length, n, mode, initial=initial,
                                 initial_arr=None if init is None else _to(dev, init),
                                 addrs=None if addrs is None else _to(dev, addrs)).cpu().numpy()
    want = oracle_c.batch(host[base_off:], mode, stride=stride, length=length, n=n,
                          initial_arr=init, initial=initial, addrs=addrs)
    return got, want


@pytest.mark.parametrize("length", EDGE_LENS)
def test_raw_uniform_edge_lengths(dev, oracle_c, length):
    rng = np.random.default_rng(length)
    for base_off in (0, 1, 2, 3, 5, 8, 13):
        for stride in {length, length + 1, length + 3, max(length, 1) * 2 + 7}:
            for kind in ("rand", "zero", "ff"):
                got, want = _uniform_case(dev, oracle_c, rng, length, stride, 37, O.MODE_RAW,
                                          base_off=base_off, kind=kind, use_init_arr=(kind == "rand"),
                                          initial=0xFFFF if kind == "ff" else 0)
                assert np.array_equal(got, want), (length, stride, base_off, kind)


@pytest.mark.parametrize("mode", [O.MODE_UDP, O.MODE_TCP, O.MODE_VERIFY_TCP, O.MODE_VERIFY_UDP])
@pytest.mark.parametrize("length", [20, 21, 63, 64, 65, 1499, 1500, 1501, 4097, 9000, 65535])
def test_transport_uniform(dev, oracle_c, mode, length):
    rng = np.random.default_rng(1000 + length + 17 * mode)
    n = 8 if length > 9000 else 41
    for base_off, stride_pad, use_addrs in ((0, 0, True), (3, 5, False), (2, 1, True), (1, 0, False)):
        got, want = _uniform_case(dev, oracle_c, rng, length, length + stride_pad, n, mode,
                                  base_off=base_off, use_addrs=use_addrs, use_init_arr=not use_addrs)
        assert np.array_equal(got, want), (mode, length, base_off, stride_pad)


@pytest.mark.parametrize("mode", [O.MODE_RAW, O.MODE_UDP, O.MODE_TCP, O.MODE_ICMP,
                                  O.MODE_VERIFY_TCP, O.MODE_VERIFY_UDP])
def test_lane_kernel_shapes(dev, oracle_c, mode):
    """k_lane (dense uniform packets up to 112 bytes, strides to 128): tails of 1-3 bytes,
    gaps between packets (stride > len), every LDS read width, partial last wave
    steps, and the TX field; k_tiny<8> takes over above 112 bytes."""
    rng = np.random.default_rng(3000 + mode)
    use_addrs = mode in (O.MODE_UDP, O.MODE_TCP, O.MODE_VERIFY_TCP, O.MODE_VERIFY_UDP)
    seen = set()
    lo = {O.MODE_UDP: 8, O.MODE_TCP: 20, O.MODE_VERIFY_TCP: 20, O.MODE_VERIFY_UDP: 8, O.MODE_ICMP: 4}
    for length, stride in ((3, 4), (8, 8), (20, 20), (21, 24), (33, 36), (48, 48), (60, 64), (64, 64),
                           (65, 68), (66, 68), (67, 68), (68, 68), (71, 72), (72, 72), (72, 80),
                           (80, 80), (81, 96), (96, 96), (100, 100), (104, 104), (112, 112),
                           (100, 128), (112, 128), (127, 128), (128, 128)):
        if length < lo.get(mode, 1):
            continue
        seen.add(batch.variant(stride, length, mode, 0))
        for n in (1, 63, 64, 65, 1000):
            got, want = _uniform_case(dev, oracle_c, rng, length, stride, n, mode,
                                      use_addrs=use_addrs, use_init_arr=not use_addrs)
            assert np.array_equal(got, want), (mode, length, stride, n)
    assert {"k_lane<2>", "k_lane<3>", "k_lane<4>", "k_lane<5>", "k_lane<6>", "k_lane<7>", "k_lane<8>",
            "k_tiny<8>"} <= seen, seen


def test_lane_kernel_grid_stride(dev, oracle_c):
    """More packets than one pass of the k_lane grid: 1.3M x 72-B UDP datagrams."""
    rng = np.random.default_rng(5)
    n, L = 1_300_000, 72
    assert batch.variant(L, L, "udp", 0) == "k_lane<5>"
    host = _rand(rng, n * L)
    addrs = _rand(rng, 8 * n)
    got = batch.checksum_uniform(_to(dev, host), L, L, n, "udp", addrs=_to(dev, addrs)).cpu().numpy()
    want = oracle_c.batch(host, O.MODE_UDP, stride=L, length=L, n=n, addrs=addrs)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", [O.MODE_IPV4, O.MODE_VERIFY_IPV4, O.MODE_ICMP])
@pytest.mark.parametrize("length", [4, 20, 21, 24, 60, 61, 64, 100, 1500, 1501])
def test_ipv4_icmp_uniform(dev, oracle_c, mode, length):
    rng = np.random.default_rng(2000 + length + 31 * mode)
    for base_off in (0, 1, 2, 7):
        got, want = _uniform_case(dev, oracle_c, rng, length, length + base_off, 53, mode, base_off=base_off)
        assert np.array_equal(got, want), (mode, length, base_off)


def _ragged(rng, lens, base_off=0, kind="rand"):
    offs = np.zeros(len(lens) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += base_off
    return _rand(rng, int(offs[-1]) + 32, kind), offs


@pytest.mark.parametrize("npk", [600, 4500])  # a small burst (k_loop) and k_seg
@pytest.mark.parametrize("mode", list(range(8)))
def test_ragged_all_modes(dev, oracle_c, mode, npk):
    rng = np.random.default_rng(3000 + mode + npk)
    lo = {O.MODE_UDP: 8, O.MODE_TCP: 60, O.MODE_VERIFY_TCP: 60, O.MODE_ICMP: 4,
          O.MODE_IPV4: 60, O.MODE_VERIFY_IPV4: 60}.get(mode, 0)
    if mode not in (O.MODE_IPV4, O.MODE_VERIFY_IPV4):
        assert FORCED or batch.ragged_variant(mode, npk).startswith("k_loop" if npk <= 4096 else "k_seg")
    lens = rng.integers(lo, 9001, size=npk)
    lens[:len(EDGE_LENS)] = np.maximum(np.array(EDGE_LENS), lo)
    blob, offs = _ragged(rng, lens, base_off=3)
    n = len(lens)
    for p in range(n):
        s = int(offs[p])
        if mode in (O.MODE_TCP, O.MODE_VERIFY_TCP):
            blob[s + 12] = int(rng.integers(5, 16)) << 4
        if mode in (O.MODE_IPV4, O.MODE_VERIFY_IPV4):
            blob[s] = 0x40 | int(rng.integers(0, 16))
    addrs = _rand(rng, 8 * n)
    init = rng.integers(0, 65536, size=n, dtype=np.uint16)
    for use_addrs in (False, True):
        got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), mode,
                                    initial_arr=None if use_addrs else _to(dev, init),
                                    addrs=_to(dev, addrs) if use_addrs else None).cpu().numpy()
        want = oracle_c.batch(blob, mode, offsets=offs, initial_arr=None if use_addrs else init,
                              addrs=addrs if use_addrs else None)
        assert np.array_equal(got, want), (mode, use_addrs, np.nonzero(got != want)[0][:10])


def _ragged_headers(rng, blob, offs, mode):
    for p in range(len(offs) - 1):
        s = int(offs[p])
        if mode in (O.MODE_TCP, O.MODE_VERIFY_TCP):
            blob[s + 12] = int(rng.integers(5, 16)) << 4
        if mode in (O.MODE_IPV4, O.MODE_VERIFY_IPV4):
            blob[s] = 0x40 | int(rng.integers(0, 16))


@pytest.mark.parametrize("lo,hi", [(0, 64), (40, 200), (64, 1500)])
@pytest.mark.parametrize("mode", list(range(8)))
def test_ragged_small_packets(dev, oracle_c, mode, lo, hi):
    """tun-style RX bursts: mostly short packets (k_rag's group path) with a
    few long ones sprinkled in (its whole-wave phase 2), every start alignment."""
    rng = np.random.default_rng(7000 + 17 * mode + hi)
    mn = {O.MODE_UDP: 8, O.MODE_TCP: 60, O.MODE_VERIFY_TCP: 60, O.MODE_ICMP: 4,
          O.MODE_IPV4: 60, O.MODE_VERIFY_IPV4: 60}.get(mode, 0)
    n = 5000
    lens = rng.integers(max(lo, mn), max(hi, mn) + 1, size=n)
    long_at = rng.choice(n, size=24, replace=False)
    lens[long_at[:20]] = rng.integers(1537, 9001, size=20)
    # RAW: past the LE-sum limit; transport/IPv4 modes are capped at 65535
    lens[long_at[20:]] = rng.integers(131073, 140000, size=4) if mode == O.MODE_RAW else 65535
    for base_off in (0, 1, 2, 3):
        blob, offs = _ragged(rng, lens, base_off=base_off)
        _ragged_headers(rng, blob, offs, mode)
        addrs = _rand(rng, 8 * n)
        init = rng.integers(0, 65536, size=n, dtype=np.uint16)
        got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), mode,
                                    initial_arr=_to(dev, init), addrs=_to(dev, addrs)).cpu().numpy()
        want = oracle_c.batch(blob, mode, offsets=offs, initial_arr=init, addrs=addrs)
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])


@pytest.mark.parametrize("mode", [O.MODE_RAW])
def test_ragged_far_from_step_base(dev, oracle_c, mode):
    """A 2.1 GiB packet followed by short ones: the short packets of its step lie
    more than 1 GiB past the step's first packet, which k_rag's 32-bit lane
    offsets cannot reach, so they take the whole-wave path; the later steps sit
    at offsets with bit 31 set (a sign-extension trap for 32-bit lane reads)."""
    big = (2 << 30) + (100 << 20) + 3
    lens = np.array([big, 64, 65, 20, 100, 7] + [60] * 10, dtype=np.int64)
    offs = np.zeros(len(lens) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += 1
    blob = np.zeros(int(offs[-1]) + 32, np.uint8)
    rng = np.random.default_rng(77)
    blob[:1 << 20] = _rand(rng, 1 << 20)
    blob[-(1 << 20):] = _rand(rng, 1 << 20)
    _ragged_headers(rng, blob, offs, mode)
    got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), mode,
                                initial=0x1234).cpu().numpy()
    want = oracle_c.batch(blob, mode, offsets=offs, initial=0x1234)
    assert np.array_equal(got, want), np.nonzero(got != want)[0]


@pytest.mark.parametrize("npk", [3000, 4500])  # a burst (k_loop_rx) and k_seg's RX kind
@pytest.mark.parametrize("lo,hi", [(0, 40), (0, 300), (0, 1480), (1000, 9000)])
def test_verify_rx_ragged(dev, oracle_c, lo, hi, npk):
    """Whole received datagrams (tun RX bursts): header + transport verification
    bits against the oracle, every start alignment, valid and damaged packets."""
    import rxgen
    assert FORCED or batch.ragged_variant("verify_rx", npk) == ("k_loop<4,rx>" if npk <= 4096 else "k_seg<8,rx,c16>")
    rng = np.random.default_rng(9100 + hi + npk)
    blob, offs = rxgen.rx_batch(rng, npk, lo=lo, hi=min(hi, 65535 - 80))
    for base_off in (0, 1, 2, 3):
        b = np.concatenate([np.zeros(base_off, np.uint8), blob, np.zeros(32, np.uint8)])
        o = offs + base_off
        got = batch.checksum_ragged(_to(dev, b), _to(dev, o.view(np.int64)), "verify_rx").cpu().numpy()
        want = oracle_c.batch(b, O.MODE_VERIFY_RX, offsets=o)
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])
    assert len(np.unique(want)) >= 5


def test_verify_rx_fuzz(dev, oracle_c):
    """Seeded RX batches whose sizes straddle every VERIFY_RX kernel cut-over (a wave
    per datagram up to 4096, 16-datagram k_seg chunks up to 65535, 64-datagram chunks
    from 65536): verification bits against the oracle at a random start alignment.
    YU_RX_FUZZ_SEED / YU_RX_FUZZ_ITERS for longer runs by hand."""
    import os
    import rxgen
    rng = np.random.default_rng(int(os.environ.get("YU_RX_FUZZ_SEED", "4242")))
    seen = set()
    sizes = [1, 2, 63, 64, 65, 4096, 4097, 65535, 65536, 70000]
    for it in range(int(os.environ.get("YU_RX_FUZZ_ITERS", "12"))):
        npk = sizes[it] if it < len(sizes) else int(rng.integers(1, 20000))
        lo, hi = [(0, 40), (0, 300), (0, 1480), (1000, 9000)][int(rng.integers(0, 4))]
        bad = float(rng.random())
        if npk > 10000:
            # mostly short datagrams (keeps the Python packet generator to seconds),
            # with 64 of 1000..9000 bytes among them: at 64 datagrams per chunk those
            # reach past a tile, in the small-packet grid's regime too
            lo, hi = min(lo, 100), min(hi, 300)
            blob, offs = rxgen.rx_batch(rng, npk - 64, lo=lo, hi=hi, bad=bad)
            bblob, boffs = rxgen.rx_batch(rng, 64, lo=1000, hi=9000, bad=bad)
            pk = [blob[int(offs[i]):int(offs[i + 1])] for i in range(npk - 64)]
            for j, at in enumerate(sorted(rng.choice(npk - 63, size=64, replace=False))[::-1]):
                pk.insert(int(at), bblob[int(boffs[j]):int(boffs[j + 1])])
            offs = np.zeros(npk + 1, np.uint64)
            offs[1:] = np.cumsum([len(x) for x in pk])
            blob = np.concatenate(pk)
        else:
            blob, offs = rxgen.rx_batch(rng, npk, lo=lo, hi=hi, bad=bad)
        base_off = int(rng.integers(0, 16))
        b = np.concatenate([np.zeros(base_off, np.uint8), blob, np.zeros(32, np.uint8)])
        o = offs + base_off
        seen.add(batch.ragged_variant("verify_rx", npk))
        got = batch.checksum_ragged(_to(dev, b), _to(dev, o.view(np.int64)), "verify_rx").cpu().numpy()
        want = oracle_c.batch(b, O.MODE_VERIFY_RX, offsets=o)
        assert np.array_equal(got, want), (it, npk, lo, hi, base_off, np.nonzero(got != want)[0][:10])
    if int(os.environ.get("YU_RX_FUZZ_ITERS", "12")) >= len(sizes) and not FORCED:
        assert {"k_loop<4,rx>", "k_seg<8,rx,c16>", "k_seg<8,rx>"} <= seen, seen


def _tx_expected(blob, offs, want, length=None):
    """The bytes TX_DATAGRAM's in-place writer must leave: every byte as before,
    except the two fields of each datagram where they are defined (the oracle's
    values, include/yucsum.h YU_MODE_TX_DATAGRAM). Datagram i starts at offs[i]
    and ends at offs[i+1], or after `length` bytes (uniform slots). Also returns
    which datagrams got an IPv4 and which a transport field."""
    exp = blob.copy()
    n = len(offs) - 1
    ip_def, l4_def = np.zeros(n, bool), np.zeros(n, bool)
    for i in range(n):
        a = int(offs[i])
        e = int(offs[i + 1]) if length is None else a + length
        pk = blob[a:e]
        if e - a < 20:
            continue
        hl, tl = (int(pk[0]) & 15) * 4, (int(pk[2]) << 8) | int(pk[3])
        if hl < 20 or hl > tl or tl > e - a:
            continue
        exp[a + 10], exp[a + 11] = want[2 * i] >> 8, want[2 * i] & 0xFF
        ip_def[i] = True
        fo, mn = {17: (6, 8), 6: (16, 20), 1: (2, 4)}.get(int(pk[9]), (0, 0))
        if fo and tl - hl >= mn:
            exp[a + hl + fo], exp[a + hl + fo + 1] = want[2 * i + 1] >> 8, want[2 * i + 1] & 0xFF
            l4_def[i] = True
    return exp, ip_def, l4_def


@pytest.mark.parametrize("npk", [1, 64, 4096, 4097, 65535, 65536, 70000])
def test_tx_datagram_ragged(dev, oracle_c, npk):
    """TX_DATAGRAM over ragged batches of outgoing datagrams on both sides of every
    kernel cut-over (a wave per datagram up to 4096, 16-datagram k_seg chunks up to
    65535, 64-datagram chunks from 65536): both fields against the oracle at an odd
    start, then in place at 4-aligned offsets, where afterwards only the defined
    fields differ from the input and the filled datagrams pass VERIFY_RX."""
    import rxgen
    rng = np.random.default_rng(9500 + npk)
    hi = 1480 if npk <= 4097 else 200
    blob, offs = rxgen.tx_batch(rng, npk, lo=0, hi=hi, bad=0.15, pad4=True)
    if npk > 1000:  # a few jumbo datagrams among the small ones (past a tile)
        jb, jo = rxgen.tx_batch(rng, 8, lo=5000, hi=9000, bad=0.0, pad4=True)
        blob = np.concatenate([jb, blob])
        offs = np.concatenate([jo[:-1], offs + jo[-1]])
        npk += 8
    want = oracle_c.batch(blob, O.MODE_TX_DATAGRAM, offsets=offs)
    assert want.size == 2 * npk
    assert (want[0::2] != 0).mean() > 0.8 and (want[1::2] != 0).mean() > 0.5
    for base_off in (1, 3):
        b = np.concatenate([np.zeros(base_off, np.uint8), blob, np.zeros(32, np.uint8)])
        got = batch.checksum_ragged(_to(dev, b), _to(dev, (offs + base_off).view(np.int64)),
                                    "tx_datagram").cpu().numpy()
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])
    d = _to(dev, np.concatenate([blob, np.zeros(32, np.uint8)]))
    o = _to(dev, offs.view(np.int64))
    got = batch.checksum_ragged(d, o, "tx_datagram", fill=True).cpu().numpy()
    assert np.array_equal(got, want)
    filled = d.cpu().numpy()[:blob.size]
    exp, ip_def, l4_def = _tx_expected(blob, offs, want)
    bad = np.nonzero(filled != exp)[0]
    assert bad.size == 0, bad[:10]
    assert ip_def.mean() > 0.8 and l4_def.mean() > 0.5
    # what was filled now verifies (checker.IPv4 / checker.TCP semantics)
    rx = batch.checksum_ragged(d, o, "verify_rx").cpu().numpy()
    assert (rx[ip_def] & O.RX_IP_OK).all()
    assert (rx[l4_def] & (O.RX_L4 | O.RX_L4_OK) == (O.RX_L4 | O.RX_L4_OK)).all()


@pytest.mark.parametrize("packed,shift", [(False, 0), (False, 68), (True, 0), (True, 1), (True, 67),
                                          (True, 130)])
@pytest.mark.parametrize("npk", [5000, 70000])
@pytest.mark.parametrize("mode,lo", [(O.MODE_UDP, 8), (O.MODE_TCP, 20), (O.MODE_ICMP, 4)])
def test_fill_ragged_small_packets(dev, oracle_c, mode, lo, npk, packed, shift):
    """In place on ragged small packets with a few large ones among them, in 16- and
    48-packet k_seg chunks: only the fields change, chunk edges included, and the
    results equal the oracle's. The TX kind's whole-line write-back (YU_FILL_WB)
    stores the 128-byte lines of each chunk's last tile; shift 68 starts the batch
    off a line boundary, so the first chunk's line begins before the batch.
    `packed`: lengths as drawn (not rounded to 4) and the batch at an odd address
    (shift 1, 67) or 2 bytes past a line (130) — a packed, unaligned tun burst, which
    yu_csum_fill_ragged takes as it lies (include/yucsum.h, Preconditions): fields at
    odd addresses and fields straddling a 128-byte line, in the TXW kind's 48-packet
    chunks from 70000 packets."""
    rng = np.random.default_rng(9900 + 7 * mode + npk + (1000 if packed else 0))
    lens = rng.integers(lo, 201, size=npk)
    if not packed:
        lens = (lens + 3) & ~3
    lens[rng.choice(npk, size=npk // 500, replace=False)] = 4 * rng.integers(1000, 2500, size=npk // 500)
    offs = np.zeros(npk + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = _rand(rng, int(offs[-1]) + 64)
    if mode == O.MODE_TCP:
        blob[offs[:-1].astype(np.int64) + 12] = 0x50
    addrs = _rand(rng, 8 * npk)
    want = oracle_c.batch(blob, mode, offsets=offs, addrs=addrs if mode != O.MODE_ICMP else None)
    # the write-back off (YU_FILL_WB=0): the TX kind; from 64K packets on the TXW kind
    # takes 48-packet chunks
    wb = not (TUNING and os.environ.get("YU_FILL_WB") == "0")
    big = "k_seg<8,txw,c48>" if wb else "k_seg<8,tx>"
    assert FORCED or batch.ragged_variant(mode, npk, fill=True) == (
        f"k_seg<8,{'txw' if wb else 'tx'},c16>" if npk < 65536 else big)
    pre = _rand(rng, shift)
    whole = _to(dev, np.concatenate([pre, blob]))
    d = whole[shift:]
    got = batch.checksum_ragged(d, _to(dev, offs.view(np.int64)), mode,
                                addrs=_to(dev, addrs) if mode != O.MODE_ICMP else None, fill=True).cpu().numpy()
    assert np.array_equal(got, want)
    f = {O.MODE_UDP: 6, O.MODE_TCP: 16, O.MODE_ICMP: 2}[mode]
    exp = blob.copy()
    fi = offs[:-1].astype(np.int64) + f
    exp[fi] = (want >> 8).astype(np.uint8)
    exp[fi + 1] = (want & 0xFF).astype(np.uint8)
    bad = np.nonzero(d.cpu().numpy() != exp)[0]
    assert bad.size == 0, bad[:10]
    assert np.array_equal(whole[:shift].cpu().numpy(), pre)  # the bytes before the batch
    if packed:  # the layout did put fields on odd addresses and across 128-byte lines
        fa = fi + shift
        assert (fa & 1).any() and ((fa & 127) == 127).any()


def test_tx_datagram_fuzz(dev, oracle_c):
    """Seeded TX_DATAGRAM batches of 1 to 70000 datagrams: random sizes (tiny, MTU,
    jumbo), protocols, IHL 5..15, a share damaged or out of contract, random start
    alignment (values, and in place, where only the defined fields may change). YU_TX_FUZZ_SEED / YU_TX_FUZZ_ITERS for longer runs by hand."""
    import os
    import rxgen
    rng = np.random.default_rng(int(os.environ.get("YU_TX_FUZZ_SEED", "5151")))
    sizes = [1, 2, 63, 64, 65, 4096, 4097, 65535, 65536, 70000]
    seen = set()
    for it in range(int(os.environ.get("YU_TX_FUZZ_ITERS", "12"))):
        npk = sizes[it] if it < len(sizes) else int(rng.integers(1, 20000))
        lo, hi = [(0, 40), (0, 300), (0, 1480), (1000, 9000)][int(rng.integers(0, 4))]
        if npk > 10000:
            lo, hi = min(lo, 100), min(hi, 300)
        blob, offs = rxgen.tx_batch(rng, npk, lo=lo, hi=hi, bad=float(rng.random()) * 0.5, pad4=True)
        seen.add(batch.ragged_variant("tx_datagram", npk))
        seen.add("fill:" + batch.ragged_variant("tx_datagram", npk, fill=True))
        want = oracle_c.batch(blob, O.MODE_TX_DATAGRAM, offsets=offs)
        base_off = int(rng.integers(0, 16))
        b = np.concatenate([np.zeros(base_off, np.uint8), blob, np.zeros(32, np.uint8)])
        got = batch.checksum_ragged(_to(dev, b), _to(dev, (offs + base_off).view(np.int64)),
                                    "tx_datagram").cpu().numpy()
        assert np.array_equal(got, want), (it, npk, lo, hi, base_off, np.nonzero(got != want)[0][:10])
        pad = int(rng.integers(0, 16))  # in place at any alignment (include/yucsum.h)
        d = _to(dev, np.concatenate([np.zeros(pad, np.uint8), blob, np.zeros(32, np.uint8)]))
        got = batch.checksum_ragged(d, _to(dev, (offs + pad).view(np.int64)), "tx_datagram",
                                    fill=True).cpu().numpy()
        assert np.array_equal(got, want), (it, npk, "fill")
        filled = d.cpu().numpy()[pad:pad + blob.size]
        assert np.array_equal(filled, _tx_expected(blob, offs, want)[0]), (it, npk, "fill bytes")
    if int(os.environ.get("YU_TX_FUZZ_ITERS", "12")) >= len(sizes) and not FORCED:
        assert {"k_loop<4,dg>", "k_seg<8,dg,c16>", "k_seg<8,dg>", "fill:k_seg<8,dg,c16>",
                "fill:" + DG_FILL} <= seen, seen


@pytest.mark.parametrize("npk,kern", [(5000, "k_seg<8,dg,c16>"), (66000, "k_seg<8,dg>")])
def test_tx_datagram_header_straddles_tile(dev, oracle_c, npk, kern):
    """k_seg's DG kind gathers each datagram's first 20 header bytes across tiles: IHL-5
    datagrams start with floor4(start) 4..20 bytes before a 4 KiB and an 8 KiB tile
    boundary of their chunk (rxgen.tile_edge_batch), at every start alignment."""
    import rxgen
    assert FORCED or batch.ragged_variant("tx_datagram", npk) == kern
    chunk = 16 if "c16" in kern else 64
    rng = np.random.default_rng(9600 + npk)
    special = lambda r, total: rxgen.tx_packet(r, max(0, total - 20), ihl=5)  # noqa: E731
    for base_off in (0, 1, 2, 3):
        blob, offs = rxgen.tile_edge_batch(rng, npk, chunk, base_off, special=special)
        for i in range(npk):  # fillers with protocol 6: keep their TCP segments in contract
            a, e = int(offs[i]), int(offs[i + 1])
            blob[a:e] = np.frombuffer(bytes(rxgen.tcp_contract(bytearray(blob[a:e].tobytes()))), np.uint8)
        got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), "tx_datagram").cpu().numpy()
        want = oracle_c.batch(blob, O.MODE_TX_DATAGRAM, offsets=offs)
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])
        assert (want[0::2] != 0).mean() > 0.9  # in contract: fillers and specials alike


@pytest.mark.parametrize("npk,kern", [(5000, "k_seg<8,dg,c16>"), (66000, DG_FILL)])
def test_tx_datagram_fill_header_straddles_tile(dev, oracle_c, npk, kern):
    """The same tile-straddling headers written in place: TX_DATAGRAM's fill takes
    40-packet chunks from 64K datagrams on (16 below), so the batch is laid out on
    that chunk's tile boundaries; values, both fields, and no other byte changed."""
    import rxgen
    assert FORCED or batch.ragged_variant("tx_datagram", npk, fill=True) == kern
    chunk = 16 if "c16" in kern else DG_FILL_CH
    rng = np.random.default_rng(9650 + npk)
    special = lambda r, total: rxgen.tx_packet(r, max(0, total - 20), ihl=5)  # noqa: E731
    for base_off in (0, 3):
        blob, offs = rxgen.tile_edge_batch(rng, npk, chunk, base_off, tile=8192, special=special)
        for i in range(npk):
            a, e = int(offs[i]), int(offs[i + 1])
            blob[a:e] = np.frombuffer(bytes(rxgen.tcp_contract(bytearray(blob[a:e].tobytes()))), np.uint8)
        want = oracle_c.batch(blob, O.MODE_TX_DATAGRAM, offsets=offs)
        d = _to(dev, blob)
        got = batch.checksum_ragged(d, _to(dev, offs.view(np.int64)), "tx_datagram", fill=True).cpu().numpy()
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])
        exp = _tx_expected(blob, offs, want)[0]
        bad = np.nonzero(d.cpu().numpy() != exp)[0]
        assert bad.size == 0, (base_off, bad[:10])


@pytest.mark.parametrize("npk", [777, 70000])
@pytest.mark.parametrize("length", [20, 28, 64, 576, 1500])
def test_tx_datagram_uniform(dev, oracle_c, length, npk):
    """Fixed-size outgoing datagrams in uniform slots (stride > length), values and
    in-place fields."""
    import rxgen
    rng = np.random.default_rng(9700 + length + npk)
    n, stride = npk, (length + 7) // 4 * 4
    host = np.zeros(n * stride + 64, np.uint8)
    for p in range(n if n < 5000 else 3000):
        pk = bytes(rxgen.tx_packet(rng, length - 20, ihl=5))[:length].ljust(length, b"\0")
        host[p * stride: p * stride + length] = np.frombuffer(pk, np.uint8)
    if n >= 5000:  # replicate the first 3000 slots
        reps = -(-n // 3000)
        host[: n * stride] = np.tile(host[: 3000 * stride], reps)[: n * stride]
    want = oracle_c.batch(host, O.MODE_TX_DATAGRAM, stride=stride, length=length, n=n)
    d = _to(dev, host)
    got = batch.checksum_uniform(d, stride, length, n, "tx_datagram").cpu().numpy()
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]
    got = batch.checksum_uniform(d, stride, length, n, "tx_datagram", fill=True).cpu().numpy()
    assert np.array_equal(got, want)
    exp = _tx_expected(host, np.arange(n + 1, dtype=np.uint64) * stride, want, length=length)
    filled = d.cpu().numpy()
    # slot i = [i*stride, i*stride+length): the gap bytes after each datagram stay
    assert np.array_equal(filled, exp[0])


def test_tx_datagram_host_paths(dev, oracle_c):
    """TX_DATAGRAM through the host entry points (direct burst, pipelined slices, the
    scatter-gather form) with fill: two results per packet, fields in host memory."""
    import rxgen
    rng = np.random.default_rng(9800)
    for n in (64, 30000):
        blob, offs = rxgen.tx_batch(rng, n, lo=0, hi=1480, bad=0.1, pad4=True)
        want = oracle_c.batch(blob, O.MODE_TX_DATAGRAM, offsets=offs)
        got = batch.checksum_host_ragged(blob, offs, "tx_datagram")
        assert np.array_equal(got, want), n
        buf = blob.copy()
        got = batch.checksum_host_ragged(buf, offs, "tx_datagram", fill=True)
        assert np.array_equal(got, want)
        assert np.array_equal(buf, _tx_expected(blob, offs, want)[0])
        pk = [bytearray(blob[int(offs[i]):int(offs[i + 1])].tobytes()) for i in range(n)]
        views = [[np.frombuffer(p, np.uint8)[:7].copy(), np.frombuffer(p, np.uint8)[7:].copy()] for p in pk]
        got = batch.checksum_host_iov(views, "tx_datagram", fill=True)
        assert np.array_equal(got, want)
        joined = np.concatenate([np.concatenate(v) for v in views])
        assert np.array_equal(joined, _tx_expected(blob, offs, want)[0])


@pytest.mark.parametrize("npk", [777, 5000])
@pytest.mark.parametrize("length", [20, 40, 64, 576, 1500])
def test_verify_rx_uniform(dev, oracle_c, length, npk):
    """Fixed-size received datagrams in uniform slots (stride >= length)."""
    import rxgen
    rng = np.random.default_rng(9200 + length + npk)
    n, stride = npk, length + 5
    host = np.zeros(n * stride + 64, np.uint8)
    for p in range(n):
        pk = rxgen.make_packet(rng, length - 20, ihl=5)
        if rng.random() < 0.4:
            pk = rxgen.damage(rng, pk)
        pk = bytes(pk[:length]).ljust(length, b"\0")
        host[p * stride: p * stride + length] = np.frombuffer(pk, np.uint8)
    for base_off in (0, 2):
        got = batch.checksum_uniform(_to(dev, host[base_off:]), stride, length, n - 1, "verify_rx").cpu().numpy()
        want = oracle_c.batch(host[base_off:], O.MODE_VERIFY_RX, stride=stride, length=length, n=n - 1)
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])


@pytest.mark.parametrize("npk,kern", [(5000, "k_seg<8,rx,c16>"), (66000, "k_seg<8,rx>")])
def test_verify_rx_header_straddles_tile(dev, oracle_c, npk, kern):
    """k_seg's RX kind parses a header that straddles two tiles in the second one.
    IHL 0..4 headers (and total lengths under 20) put the header and transport end
    points inside the first tile; they must still be evaluated. Every short-header
    datagram here starts with floor4(start) 4..20 bytes before a 4 KiB or 8 KiB tile
    boundary of its chunk, at each start alignment (ragged), and the same with
    uniform slots of 8188 / 4092 bytes (packet k of a chunk then sits 4k bytes before
    the k-th 8 / 4 KiB boundary)."""
    import rxgen
    assert FORCED or batch.ragged_variant("verify_rx", npk) == kern
    chunk = 16 if "c16" in kern else 64
    rng = np.random.default_rng(9300 + npk)
    for base_off in (0, 1, 2, 3):
        blob, offs = rxgen.tile_edge_batch(rng, npk, chunk, base_off)
        got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), "verify_rx").cpu().numpy()
        want = oracle_c.batch(blob, O.MODE_VERIFY_RX, offsets=offs)
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])
        assert (want[1::2] & O.RX_IP_OK).any() and (want[1::2] & O.RX_L4_OK).any()
    # uniform slots
    stride = 8188 if npk < 65536 else 4092
    length = 48
    pk = np.frombuffer(b"".join(bytes(rxgen.short_header_packet(rng, length)) for _ in range(npk)),
                       np.uint8).reshape(npk, length)
    for base_off in (0, 1, 3):
        host = np.zeros(npk * stride + 64, np.uint8)
        host[base_off:base_off + npk * stride].reshape(npk, stride)[:, :length] = pk
        view = host[base_off:]
        got = batch.checksum_uniform(_to(dev, view), stride, length, npk - 1, "verify_rx").cpu().numpy()
        want = oracle_c.batch(view, O.MODE_VERIFY_RX, stride=stride, length=length, n=npk - 1)
        assert np.array_equal(got, want), (base_off, np.nonzero(got != want)[0][:10])
        assert (want & O.RX_IP_OK).any() and (want & O.RX_L4_OK).any()


def test_ragged_zero_ff_and_empty(dev, oracle_c):
    rng = np.random.default_rng(5)
    lens = np.array([0, 0, 1, 0, 2, 3, 0, 5, 17, 0] + list(rng.integers(0, 300, size=300)))
    for kind in ("zero", "ff", "rand"):
        for base_off in (0, 1, 2, 3):
            blob, offs = _ragged(rng, lens, base_off=base_off, kind=kind)
            for initial in (0, 0xFFFF, 1234):
                got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), "raw",
                                            initial=initial).cpu().numpy()
                want = oracle_c.batch(blob, O.MODE_RAW, offsets=offs, initial=initial)
                assert np.array_equal(got, want), (kind, base_off, initial)
    # the 0x0000-vs-0xFFFF representation: all-zero bytes with initial 0 must give 0
    blob, offs = _ragged(rng, lens, kind="zero")
    got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), "raw").cpu().numpy()
    assert (got == 0).all()


def test_raw_uint32_wrap(dev, oracle_c):
    """Buffers > 131072 B wrap the reference's uint32 accumulator (checksum.go:5,14)."""
    rng = np.random.default_rng(9)
    for length in (131072, 131073, 131074, 200001, 1 << 20):
        for kind in ("ff", "rand"):
            for initial in (0, 0xFFFF):
                got, want = _uniform_case(dev, oracle_c, rng, length, length + 1, 3, O.MODE_RAW,
                                          base_off=1, kind=kind, initial=initial)
                assert np.array_equal(got, want), (length, kind, initial)
    host = np.full(131074, 255, np.uint8)
    got = batch.checksum_uniform(_to(dev, host), 131074, 131074, 1, "raw", initial=0xFFFF).cpu().numpy()
    assert got[0] == 65534  # the reference's wrapped value (exact sum would give 65535)


@pytest.mark.parametrize("L,pad", [(132, 0), (136, 0), (200, 4), (300, 0), (700, 0), (1500, 0), (1500, 8), (2000, 0),
                                   (3000, 4), (4000, 0), (1500, 36)])
@pytest.mark.parametrize("mode", [O.MODE_UDP, O.MODE_TCP, O.MODE_ICMP])
def test_fill_k_small_every_alignment(dev, oracle_c, mode, L, pad):
    """The in-place writer on every k_small shape it reaches (132..4000-byte packets,
    dense and sparse): packets start at every 4-aligned offset mod 64 (device views
    at base 0/4/36/60 plus the stride's steps); afterwards every byte but the fields
    equals the input, first and last packet included, and the fields and results
    equal the oracle's. (Written for a whole-64-byte-block writer that was measured
    and rejected, profiles/r02/kbench_ab_fill_block64_rejected.log.)"""
    rng = np.random.default_rng(5100 + 7 * L + pad + mode)
    stride = L + pad
    n = 777
    rand = _rand(rng, n * stride + 64)
    addrs = _rand(rng, 8 * n)
    for base in (0, 4, 36, 60):
        host = rand.copy()
        if mode == O.MODE_TCP:  # DataOffset 5 (sendTCP's segments)
            host[base + np.arange(n, dtype=np.int64) * stride + 12] = 0x50
        assert batch.variant(stride, L, {1: "udp", 2: "tcp", 4: "icmp"}[mode], base, n=n).startswith("k_small<")
        dfull = _to(dev, host)
        assert dfull.data_ptr() % 64 == 0
        d = dfull[base:]  # packets start at base mod 64 (plus the stride's steps)
        a = _to(dev, addrs) if mode in (1, 2) else None
        out = batch.checksum_uniform(d, stride, L, n, mode, addrs=a, fill=True).cpu().numpy()
        want = oracle_c.batch(host[base:], mode, stride=stride, length=L, n=n,
                              addrs=addrs if mode in (1, 2) else None)
        assert np.array_equal(out, want), (base, np.nonzero(out != want)[0][:8])
        got = dfull.cpu().numpy()
        f = {O.MODE_UDP: 6, O.MODE_TCP: 16, O.MODE_ICMP: 2}[mode]
        fidx = base + np.arange(n, dtype=np.int64) * stride + f
        expect = host.copy()
        expect[fidx] = (want >> 8).astype(np.uint8)
        expect[fidx + 1] = (want & 0xFF).astype(np.uint8)
        bad = np.nonzero(got != expect)[0]
        assert bad.size == 0, (base, bad[:8])


@pytest.mark.parametrize("L", [1500, 124, 100, 72, 64, 20])  # k_small / k_hdr, k_tiny<8>, k_lane<7,5,4,2>
@pytest.mark.parametrize("mode", [O.MODE_UDP, O.MODE_TCP, O.MODE_IPV4, O.MODE_ICMP])
def test_fill_in_place(dev, oracle_c, mode, L):
    """fill=True writes the TX field (SetChecksum); re-verifying gives 0/0xFFFF."""
    rng = np.random.default_rng(77 + mode + L)
    n = 333
    host = _rand(rng, n * L)
    pk = host.reshape(n, L)
    if mode == O.MODE_TCP:
        pk[:, 12] = 0x50
    if mode == O.MODE_IPV4:
        pk[:, 0] = 0x45
    addrs = _rand(rng, 8 * n)
    d = _to(dev, host)
    a = _to(dev, addrs)
    out = batch.checksum_uniform(d, L, L, n, mode, addrs=a if mode in (1, 2) else None, fill=True)
    want = oracle_c.batch(host, mode, stride=L, length=L, n=n, addrs=addrs if mode in (1, 2) else None)
    assert np.array_equal(out.cpu().numpy(), want)
    filled = d.cpu().numpy().reshape(n, L)
    f = {O.MODE_UDP: 6, O.MODE_TCP: 16, O.MODE_IPV4: 10, O.MODE_ICMP: 2}[mode]
    assert np.array_equal((filled[:, f].astype(np.uint16) << 8) | filled[:, f + 1], want)
    if mode in (O.MODE_UDP, O.MODE_TCP):
        vmode = O.MODE_VERIFY_UDP if mode == O.MODE_UDP else O.MODE_VERIFY_TCP
        v = batch.checksum_uniform(d, L, L, n, vmode, addrs=a)
        assert bool(batch.verified(v).all())
    if mode == O.MODE_IPV4:
        v = batch.checksum_uniform(d, L, L, n, O.MODE_VERIFY_IPV4)
        assert bool(batch.verified(v).all())


def test_reference_harness_packets_verify(dev):
    """Packets built exactly like the reference test harnesses
    (context.go:164-209, udp_test.go:105-144) pass the batched checker modes."""
    from yustack_amd import packets
    rng = np.random.default_rng(11)
    pk = [packets.tcp_test_packet(bytes(rng.integers(0, 256, int(rng.integers(0, 1460)), dtype=np.uint8)),
                                  4096, 1234, 790, 1000, 0x18, 30000) for _ in range(64)]
    offs = np.zeros(len(pk) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(p) for p in pk])
    blob = np.frombuffer(b"".join(bytes(p) for p in pk), dtype=np.uint8)
    v = batch.checksum_ragged(_to(dev, blob), _to(dev, offs), "verify_ipv4")
    assert bool(batch.verified(v).all())
    segs = [bytes(p[20:]) for p in pk]
    soffs = np.zeros(len(segs) + 1, dtype=np.int64)
    soffs[1:] = np.cumsum([len(s) for s in segs])
    sblob = np.frombuffer(b"".join(segs), dtype=np.uint8)
    addrs = np.frombuffer(b"".join(bytes(p[12:20]) for p in pk), dtype=np.uint8)
    v = batch.checksum_ragged(_to(dev, sblob), _to(dev, soffs), "verify_tcp", addrs=_to(dev, addrs))
    assert bool(batch.verified(v).all())
    # one corrupted byte must fail verification
    bad = sblob.copy()
    bad[soffs[3] + 25] ^= 0x10
    v = batch.checksum_ragged(_to(dev, bad), _to(dev, soffs), "verify_tcp", addrs=_to(dev, addrs))
    ok = batch.verified(v).cpu().numpy()
    assert not ok[3] and ok[np.arange(len(segs)) != 3].all()


def test_host_uniform_path(dev, oracle_c):
    rng = np.random.default_rng(21)
    for n, L, stride in ((100000, 1500, 1500), (70000, 64, 64), (1000, 9000, 9003), (3, 5, 7)):
        host = _rand(rng, (n - 1) * stride + L)
        host[12::stride] = 0x50 if L >= 20 else host[12::stride]
        addrs = _rand(rng, 8 * n)
        mode = O.MODE_TCP if L >= 20 else O.MODE_RAW
        got = batch.checksum_host_uniform(host, stride, L, n, mode, addrs=addrs)
        want = oracle_c.batch(host, mode, stride=stride, length=L, n=n, addrs=addrs, threads=8)
        assert np.array_equal(got, want), (n, L, stride)
    # pinned input goes straight to the copy engine (6 MB: pipelined path) or,
    # for a small burst, is read by the kernel in place (direct path), also from
    # an interior, odd address of the pinned allocation, results into pinned memory
    pinned = torch.from_numpy(_rand(rng, 4096 * 1500)).pin_memory()
    got = batch.checksum_host_uniform(pinned, 1500, 1500, 4096, "raw")
    want = oracle_c.batch(pinned.numpy(), O.MODE_RAW, stride=1500, length=1500, n=4096)
    assert np.array_equal(got, want)
    pout = torch.zeros(64, dtype=torch.int16).pin_memory()
    for start, n in ((0, 64), (1501, 63), (7, 1)):
        sub = pinned[start:start + n * 1500]
        got = batch.checksum_host_uniform(sub, 1500, 1500, n, "raw", out=pout[:n])
        want = oracle_c.batch(sub.numpy(), O.MODE_RAW, stride=1500, length=1500, n=n)
        assert np.array_equal(got.numpy().view(np.uint16), want), (start, n)
    lens = rng.integers(0, 1501, size=300)
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += 5
    pr = torch.from_numpy(_rand(rng, int(offs[-1]) + 3)).pin_memory()
    got = batch.checksum_host_ragged(pr, offs, "raw", initial=0x1234)
    assert np.array_equal(got, oracle_c.batch(pr.numpy(), O.MODE_RAW, offsets=offs, initial=0x1234))


def test_host_ragged_and_iov_paths(dev, oracle_c):
    """Host-memory ragged bursts and scatter-gather packets (tundev's 4-view readv,
    link/tundev/tundev.go:116-125) through the pinned pipeline, against the oracle."""
    import rxgen
    rng = np.random.default_rng(23)
    lens = rng.integers(0, 9001, size=20000)
    lens[::997] = 40 << 20  # a few packets longer than a 32 MiB slice
    offs = np.zeros(lens.size + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    offs += 3
    blob = _rand(rng, int(offs[-1]) + 5)
    init = rng.integers(0, 65536, size=lens.size, dtype=np.uint16)
    got = batch.checksum_host_ragged(blob, offs, "raw", initial_arr=init)
    want = oracle_c.batch(blob, O.MODE_RAW, offsets=offs, initial_arr=init, threads=8)
    assert np.array_equal(got, want)
    # RX datagrams split at the tun view boundaries 128/384/896 (tundev.go:20)
    rblob, roffs = rxgen.rx_batch(rng, 4000, lo=0, hi=1480)
    want = oracle_c.batch(rblob, O.MODE_VERIFY_RX, offsets=roffs)
    got = batch.checksum_host_ragged(rblob, roffs, "verify_rx")
    assert np.array_equal(got, want)
    cuts = [128, 128 + 384, 128 + 384 + 896]
    pkts = []
    for i in range(roffs.size - 1):
        pk = rblob[int(roffs[i]):int(roffs[i + 1])]
        edges = [0] + [c for c in cuts if c < pk.size] + [pk.size]
        pkts.append([pk[a:b] for a, b in zip(edges[:-1], edges[1:])])
    got = batch.checksum_host_iov(pkts, "verify_rx")
    assert np.array_equal(got, want)


def test_host_multi_device_paths(dev, oracle_c):
    """Multi-GPU host calls (yu_csum_batch_host_*_multi): one shard per listed
    device on its own worker thread. On a one-GPU box the list repeats device 0,
    which exercises the split, the per-worker staging and the result placement."""
    import rxgen
    rng = np.random.default_rng(29)
    ndev = max(1, torch.cuda.device_count())
    for devs in ([0], [0, 0], [0, 0, 0], list(range(ndev)) * 2):
        n, L = 50001, 1500
        host = _rand(rng, n * L)
        host[12::L] = 0x50
        addrs = _rand(rng, 8 * n)
        got = batch.checksum_host_uniform(host, L, L, n, "tcp", addrs=addrs, device=devs)
        want = oracle_c.batch(host, O.MODE_TCP, stride=L, length=L, n=n, addrs=addrs, threads=8)
        assert np.array_equal(got, want), devs
        lens = rng.integers(0, 9001, size=7777)
        lens[:5] = 0  # empty packets at a shard edge
        offs = np.zeros(lens.size + 1, np.uint64)
        offs[1:] = np.cumsum(lens)
        blob = _rand(rng, int(offs[-1]))
        init = rng.integers(0, 65536, size=lens.size, dtype=np.uint16)
        got = batch.checksum_host_ragged(blob, offs, "raw", initial_arr=init, device=devs)
        want = oracle_c.batch(blob, O.MODE_RAW, offsets=offs, initial_arr=init, threads=8)
        assert np.array_equal(got, want), devs
        rblob, roffs = rxgen.rx_batch(rng, 999, lo=0, hi=1480)
        pkts = [[rblob[int(roffs[i]):int(roffs[i + 1])]] for i in range(roffs.size - 1)]
        got = batch.checksum_host_iov(pkts, "verify_rx", device=devs)
        assert np.array_equal(got, oracle_c.batch(rblob, O.MODE_VERIFY_RX, offsets=roffs)), devs
        # two results per packet: each shard's results land at 2 x its first packet
        tblob, toffs = rxgen.tx_batch(rng, 3001, lo=0, hi=1480)
        want = oracle_c.batch(tblob, O.MODE_TX_DATAGRAM, offsets=toffs)
        assert np.array_equal(batch.checksum_host_ragged(tblob, toffs, "tx_datagram", device=devs), want), devs
        tpk = [[tblob[int(toffs[i]):int(toffs[i + 1])]] for i in range(toffs.size - 1)]
        assert np.array_equal(batch.checksum_host_iov(tpk, "tx_datagram", device=devs), want), devs
    # more shards than packets: empty shards are skipped
    host = _rand(rng, 3 * 64)
    got = batch.checksum_host_uniform(host, 64, 64, 3, "raw", device=[0] * 5)
    assert np.array_equal(got, oracle_c.batch(host, O.MODE_RAW, stride=64, length=64, n=3))
    from yustack_amd._lib import YuError
    with pytest.raises(YuError):
        batch.checksum_host_uniform(host, 64, 64, 3, "raw", device=[0, 99])


def test_side_stream_and_graph_replay(dev, oracle_c):
    """The device entry points run on the caller's stream and, allocating and
    synchronising nothing, can be captured in a HIP graph (include/yucsum.h):
    replaying the graph over new bytes in the same buffers gives the new sums."""
    rng = np.random.default_rng(31)
    n, L = 4096, 1500
    lens = rng.integers(40, 1501, size=n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    addrs = _rand(rng, 8 * n)
    a_d = _to(dev, addrs)
    d_u = torch.empty(n * L, dtype=torch.uint8, device=dev)
    d_r = torch.empty(int(offs[-1]), dtype=torch.uint8, device=dev)
    o_r = _to(dev, offs.view(np.int64))
    out_u = torch.empty(n, dtype=torch.uint16, device=dev)
    out_r = torch.empty(n, dtype=torch.uint16, device=dev)

    def fresh():
        hu = _rand(rng, n * L)
        hu[12::L] = 0x50
        hr = _rand(rng, int(offs[-1]))
        d_u.copy_(torch.from_numpy(hu))
        d_r.copy_(torch.from_numpy(hr))
        return (oracle_c.batch(hu, O.MODE_TCP, stride=L, length=L, n=n, addrs=addrs),
                oracle_c.batch(hr, O.MODE_UDP, offsets=offs, addrs=addrs))

    def launch():
        batch.checksum_uniform(d_u, L, L, n, "tcp", addrs=a_d, out=out_u)
        batch.checksum_ragged(d_r, o_r, "udp", addrs=a_d, out=out_r, validate=False)

    want_u, want_r = fresh()
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        launch()
    s.synchronize()
    assert np.array_equal(out_u.cpu().numpy(), want_u)
    assert np.array_equal(out_r.cpu().numpy(), want_r)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        launch()
    for _ in range(2):
        want_u, want_r = fresh()
        out_u.zero_()
        out_r.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out_u.cpu().numpy(), want_u)
        assert np.array_equal(out_r.cpu().numpy(), want_r)


def test_empty_batches_are_no_ops(dev):
    """n == 0 is a no-op returning an empty result, through every front-end call
    (the C ABI takes a NULL results array then, include/yucsum.h [out])."""
    d = torch.zeros(64, dtype=torch.uint8, device=dev)
    assert batch.checksum_uniform(d, 16, 16, 0, "tcp").numel() == 0
    assert batch.checksum_ragged(d, torch.zeros(1, dtype=torch.int64, device=dev), "udp").numel() == 0
    assert batch.checksum_ragged(d, torch.zeros(1, dtype=torch.int64, device=dev), "tx_datagram",
                                 fill=True).numel() == 0
    h = np.zeros(64, np.uint8)
    assert batch.checksum_host_uniform(h, 16, 16, 0, "raw").size == 0
    assert batch.checksum_host_ragged(h, np.zeros(1, np.uint64), "verify_rx").size == 0
    assert batch.checksum_host_iov([], "raw").size == 0


def test_errors_are_loud(dev):
    from yustack_amd._lib import YuError
    d = torch.zeros(1 << 17, dtype=torch.uint8, device=dev)
    with pytest.raises(YuError):
        batch.checksum_uniform(d, 16, 70000, 1, "tcp")  # > 65535 in a transport mode
    with pytest.raises(YuError):
        batch.checksum_uniform(d, 16, 4, 1, "udp")  # shorter than the UDP header
    with pytest.raises(ValueError):
        batch.checksum_uniform(d, 1 << 17, 16, 2, "raw")  # runs past the buffer
    with pytest.raises(TypeError):
        batch.checksum_uniform(d.cpu(), 16, 16, 1, "raw")


# ------------------------------------------------------------------ full size
def _full_uniform(dev, oracle_c, n, L, mode, use_addrs, use_init):
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + L)
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    if mode == O.MODE_TCP:
        d.view(n, L)[:, 12] = 0x50
        d.view(n, L)[:, 16:18] = 0
    a = torch.randint(0, 256, (8 * n,), dtype=torch.uint8, device=dev, generator=g) if use_addrs else None
    i = torch.randint(0, 65536, (n,), dtype=torch.int32, device=dev, generator=g).to(torch.uint16) if use_init else None
    got = batch.checksum_uniform(d, L, L, n, mode, addrs=a, initial_arr=i).cpu().numpy()
    want = oracle_c.batch(d.cpu().numpy(), mode, stride=L, length=L, n=n,
                          addrs=None if a is None else a.cpu().numpy(),
                          initial_arr=None if i is None else i.cpu().numpy(), threads=16)
    return got, want


def test_full_config2_raw_64B(dev, oracle_c):
    got, want = _full_uniform(dev, oracle_c, 1 << 20, 64, O.MODE_RAW, False, True)
    assert np.array_equal(got, want)


def test_full_config3_tcp_1500B(dev, oracle_c):
    got, want = _full_uniform(dev, oracle_c, 1 << 20, 1500, O.MODE_TCP, True, False)
    assert np.array_equal(got, want)


def test_full_config4_ragged(dev, oracle_c):
    n = 1 << 20
    rng = np.random.default_rng(4)
    lens = rng.integers(64, 9001, size=n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    d = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device=dev, generator=g)
    init = rng.integers(0, 65536, size=n, dtype=np.uint16)
    got = batch.checksum_ragged(d, _to(dev, offs.view(np.int64)), "raw", initial_arr=_to(dev, init)).cpu().numpy()
    want = oracle_c.batch(d.cpu().numpy(), O.MODE_RAW, offsets=offs, initial_arr=init, threads=16)
    assert np.array_equal(got, want)


# ------------------------------------------------------------------ kernel-verified datagrams
def test_kernel_verified_datagrams_on_gpu(dev):
    """Datagrams whose checksums the Linux kernel verified over a tun link, and datagrams
    the kernel built itself (tests/golden/kernel_verified.npz,
    tests/golden/make_kernel_verified.py): the HIP TX_DATAGRAM path gives exactly the
    fields the kernel accepted, in place it restores every byte of them, and the HIP
    VERIFY_RX path passes the kernel's own checksums; at aligned and odd starts."""
    from test_kernel_verified import RX_OK, load, stored_fields
    sb, so, kb, ko = load()
    z, want = stored_fields(sb, so)
    for base in (0, 1, 3):
        pad = lambda b: np.concatenate([np.zeros(base, np.uint8), b, np.zeros(16, np.uint8)])  # noqa: E731
        got = batch.checksum_ragged(_to(dev, pad(z)), _to(dev, (so + base).view(np.int64)),
                                    "tx_datagram").cpu().numpy()
        assert np.array_equal(got, want), (base, np.nonzero(got != want)[0][:10])
        for blob, offs in ((kb, ko), (sb, so)):
            rx = batch.checksum_ragged(_to(dev, pad(blob)), _to(dev, (offs + base).view(np.int64)),
                                       "verify_rx").cpu().numpy()
            assert np.all(rx & RX_OK == RX_OK), (base, rx)
    d = _to(dev, np.concatenate([z, np.zeros(16, np.uint8)]))
    got = batch.checksum_ragged(d, _to(dev, so.view(np.int64)), "tx_datagram", fill=True).cpu().numpy()
    assert np.array_equal(got, want)
    assert np.array_equal(d.cpu().numpy()[:sb.size], sb)
    # every other batch mode on the same datagrams' segments and headers
    from test_kernel_verified import mode_cases
    for mode, blob, offs, addrs, check in mode_cases():
        got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), mode,
                                    addrs=None if addrs is None else _to(dev, addrs)).cpu().numpy()
        assert check(got), (mode, got)


@pytest.mark.parametrize("n", [5000, 70000])
def test_kernel_verified_datagrams_tiled_past_cutovers(dev, n):
    """The kernel-verified datagrams drawn at random (seeded) into batches past the
    4096-packet burst cut-over and past the 65536-packet chunk cut-over, so the default
    pick is k_seg<8,dg/rx,c16> and k_seg<8,dg/rx> rather than k_loop: mixed start
    alignments, headers across tile edges, 20-byte and optioned headers, and the
    fields the Linux kernel accepted (or built) as the expected values."""
    from test_kernel_verified import RX_OK, load, stored_fields
    sb, so, kb, ko = load()
    so, ko = so.astype(np.int64), ko.astype(np.int64)
    z, want = stored_fields(sb, so)
    rng = np.random.default_rng(n)

    def tile(blob, offs, pick):
        parts = [blob[offs[i]:offs[i + 1]] for i in pick]
        o = np.zeros(len(parts) + 1, np.int64)
        o[1:] = np.cumsum([len(p) for p in parts])
        return np.concatenate(parts), o

    pick = rng.integers(0, len(so) - 1, size=n)
    zb, to = tile(z, so, pick)
    sent, _ = tile(sb, so, pick)
    want_t = want.reshape(-1, 2)[pick].ravel()
    kname = batch.ragged_variant("tx_datagram", n)
    assert FORCED or kname.startswith("k_seg<8,dg") and (("c16" in kname) == (n < 65536)), kname
    for base in (0, 1, 3):
        pad = np.concatenate([np.zeros(base, np.uint8), zb, np.zeros(16, np.uint8)])
        got = batch.checksum_ragged(_to(dev, pad), _to(dev, to + base), "tx_datagram").cpu().numpy()
        assert np.array_equal(got, want_t), (base, np.nonzero(got != want_t)[0][:10])
    d = _to(dev, np.concatenate([zb, np.zeros(16, np.uint8)]))
    got = batch.checksum_ragged(d, _to(dev, to), "tx_datagram", fill=True).cpu().numpy()
    assert np.array_equal(got, want_t)
    assert np.array_equal(d.cpu().numpy()[:sent.size], sent)
    # received: the sent and the kernel-built datagrams mixed
    both = np.concatenate([sb, kb])
    bo = np.concatenate([so[:-1], ko[:-1] + sb.size, [sb.size + kb.size]])
    rb, ro = tile(both, bo, rng.integers(0, len(bo) - 1, size=n))
    assert FORCED or batch.ragged_variant("verify_rx", n).startswith("k_seg<8,rx")
    for base in (0, 2):
        pad = np.concatenate([np.zeros(base, np.uint8), rb, np.zeros(16, np.uint8)])
        rx = batch.checksum_ragged(_to(dev, pad), _to(dev, ro + base), "verify_rx").cpu().numpy()
        assert np.all(rx & RX_OK == RX_OK), (base, np.nonzero(rx & RX_OK != RX_OK)[0][:10])


# ------------------------------------------------------------------ reference-executed vectors
def test_refexec_vectors_on_gpu(dev):
    """The HIP path against known answers produced by executing the reference's own Go
    source (tests/golden/make_refexec.py, tests/golden/goexec.py): every batch mode as
    a ragged batch (odd offsets included) and the Checksum vectors as RAW packets."""
    import json
    import os
    from test_oracle import REFEXEC, _vec_bytes, refexec_mode_batch
    ref = json.load(open(REFEXEC))
    for mode, vecs in ref["modes"].items():
        m = int(mode)
        data, offs, addrs, init, want = refexec_mode_batch(vecs, m)
        got = batch.checksum_ragged(_to(dev, data), _to(dev, offs.view(np.int64)), m,
                                    addrs=None if addrs is None else _to(dev, addrs),
                                    initial_arr=None if init is None else _to(dev, init)).cpu().numpy()
        assert np.array_equal(got, want), (mode, np.nonzero(got != want)[0][:10])
    pk = [_vec_bytes(v) for v in ref["checksum"]]
    offs = np.zeros(len(pk) + 1, np.uint64)
    offs[1:] = np.cumsum([len(x) for x in pk])
    data = np.frombuffer(b"".join(pk) + b"\0", np.uint8).copy()
    init = np.array([v["initial"] for v in ref["checksum"]], np.uint16)
    got = batch.checksum_ragged(_to(dev, data), _to(dev, offs.view(np.int64)), "raw",
                                initial_arr=_to(dev, init)).cpu().numpy()
    assert np.array_equal(got, np.array([v["want"] for v in ref["checksum"]], np.uint16))
    for v in ref["wrap"]:
        d = np.full(v["len"], v["fill"], np.uint8)
        got = batch.checksum_uniform(_to(dev, d), v["len"], v["len"], 1, "raw", initial=v["initial"])
        assert int(got.cpu().numpy()[0]) == v["want"], v


def test_host_paths_concurrent_callers(dev, oracle_c):
    """The host entry points are thread-safe (include/yucsum.h): several threads,
    each with its own staging context, call the pipelined, direct and multi-device
    paths at once (the copy pool serves one of them at a time, the rest copy on
    their own threads), every result bit-exact."""
    import threading
    rng = np.random.default_rng(37)
    jobs = []
    for k in range(6):
        n, L = (20000, 1500) if k % 3 == 0 else ((300, 1500) if k % 3 == 1 else (5000, 700))
        host = _rand(rng, n * L)
        host[12::L] = 0x50
        addrs = _rand(rng, 8 * n)
        want = oracle_c.batch(host, O.MODE_TCP, stride=L, length=L, n=n, addrs=addrs, threads=4)
        jobs.append((host, L, n, addrs, want, [0, 0] if k % 3 == 2 else 0))
    errors = []

    def worker(job):
        host, L, n, addrs, want, devs = job
        try:
            for _ in range(3):
                got = batch.checksum_host_uniform(host, L, L, n, "tcp", addrs=addrs, device=devs)
                if not np.array_equal(got, want):
                    errors.append(("mismatch", n, L))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    ts = [threading.Thread(target=worker, args=(j,)) for j in jobs]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts), "host call hung"
    assert not errors, errors


# ------------------------------------------------------------------ full-size properties
@pytest.mark.parametrize("stride,length,mode,align,n,kern", [
    (200, 40, "raw", 1, (1 << 18) + 7, "k_small<4,1>"),
    (200, 60, "udp", 2, (1 << 18) + 7, "k_small<4,1>"),
    (256, 70, "raw", 2, (1 << 18) + 7, "k_small<8,1>"),
    (300, 136, "tcp", 0, (1 << 18) + 9, "k_small<8,2>"),
    (1600, 1500, "udp", 0, (1 << 20) + 7, "k_small<16,6>"),
    (2000, 2000, "raw", 0, (1 << 20) + 7, "k_small<32,4>"),
])
def test_k_small_runs_at_grid_size(dev, oracle_c, stride, length, mode, align, n, kern):
    """k_small hands each wave 16 consecutive packets (one side-record load, one
    result store per run) from 8 runs per CU up, and a wave takes further runs
    grid-stride once the grid is full (CUs x blocks per CU x 4 waves; 16 blocks per
    CU below G = 16 lanes per packet, 64 from there). These batches are past the
    full grid, with a partial last run, at unaligned starts, with initial arrays
    and address records; bit-exact against the oracle at full size. (Smaller
    batches in the other tests cover the interleaved mapping below 8 runs per CU.)"""
    mod = {"raw": O.MODE_RAW, "udp": O.MODE_UDP, "tcp": O.MODE_TCP}[mode]
    assert batch.variant(stride, length, mode, align, n=n) == kern
    G = int(kern.split("<")[1].split(",")[0])
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    assert n // 16 >= cus * (64 if G >= 16 else 16) * 4  # the run mapping applies
    g = torch.Generator(device=dev)
    g.manual_seed(n + stride)
    total = align + (n - 1) * stride + length
    d = torch.randint(0, 256, (total + 16,), dtype=torch.uint8, device=dev, generator=g)
    if mode == "tcp":  # DataOffset 5
        d[align + 12: align + 12 + (n - 1) * stride + 1: stride] = 0x50
    ia = torch.randint(0, 1 << 16, (n,), dtype=torch.int32, device=dev, generator=g).to(torch.uint16) \
        if mode == "raw" else None
    ad = torch.randint(0, 256, (8 * n,), dtype=torch.uint8, device=dev, generator=g) if mode != "raw" else None
    got = batch.checksum_uniform(d[align:], stride, length, n, mode, initial_arr=ia, addrs=ad).cpu().numpy()
    want = oracle_c.batch(d.cpu().numpy()[align:], mod, stride=stride, length=length, n=n,
                          initial_arr=None if ia is None else ia.cpu().numpy(),
                          addrs=None if ad is None else ad.cpu().numpy(), threads=8)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


@pytest.mark.parametrize("stride,length,mode,align,n,kern", [
    (3604, 3501, "raw", 0, 40000 + 5, "k_small<64,4>"),   # GPW 1, SPR 16: shfl src = step, lane 63 finishes
    (3602, 3600, "udp", 2, 32768 + 9, "k_small<64,4>"),
    (704, 700, "tcp", 0, 40000 + 3, "k_small<16,3>"),
    (1000, 1000, "raw", 3, 40000 + 11, "k_small<16,4>"),
    (3000, 2900, "udp", 0, 40000 + 1, "k_small<32,6>"),
])
def test_k_small_runs_every_shape(dev, oracle_c, stride, length, mode, align, n, kern):
    """The run mapping (16 consecutive packets per wave) in the k_small shapes the
    grid-size test does not reach: k_small<64,4> (one packet per wave step, so a
    run is 16 steps and the result of step k comes from lane 63 to lane k) and
    <16,3>, <16,4>, <32,6>; batches past 8 runs per CU (so runs apply) with a
    partial last run, initial arrays or address records, unaligned starts."""
    mod = {"raw": O.MODE_RAW, "udp": O.MODE_UDP, "tcp": O.MODE_TCP}[mode]
    assert batch.variant(stride, length, mode, align, n=n) == kern
    assert n // 16 >= 8 * torch.cuda.get_device_properties(dev).multi_processor_count and n % 16
    g = torch.Generator(device=dev)
    g.manual_seed(n * 3 + stride)
    total = align + (n - 1) * stride + length
    d = torch.randint(0, 256, (total + 16,), dtype=torch.uint8, device=dev, generator=g)
    if mode == "tcp":
        d[align + 12: align + 12 + (n - 1) * stride + 1: stride] = 0x50
    ia = torch.randint(0, 1 << 16, (n,), dtype=torch.int32, device=dev, generator=g).to(torch.uint16) \
        if mode == "raw" else None
    ad = torch.randint(0, 256, (8 * n,), dtype=torch.uint8, device=dev, generator=g) if mode != "raw" else None
    got = batch.checksum_uniform(d[align:], stride, length, n, mode, initial_arr=ia, addrs=ad).cpu().numpy()
    want = oracle_c.batch(d.cpu().numpy()[align:], mod, stride=stride, length=length, n=n,
                          initial_arr=None if ia is None else ia.cpu().numpy(),
                          addrs=None if ad is None else ad.cpu().numpy(), threads=8)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


@pytest.mark.parametrize("mode", ["tcp", "udp"])
@pytest.mark.parametrize("length,gap,n", [
    (1280, 0, 40000 + 3), (1281, 3, 40000 + 5), (1283, 1, 33000 + 1), (1390, 2, 40000 + 15),
    (1500, 0, 40000 + 9), (1500, 100, 65536 + 1), (1534, 2, 40000 + 7), (1535, 1, 32768 + 11),
])
def test_k_small_mtu_send_path(dev, oracle_c, mode, length, gap, n):
    """The MTU send path (config 3's shape: TCP or UDP with {src,dst} records, no
    initial array, 4-aligned packet starts, 1280..1535-byte packets on k_small<16,6>
    runs), at its edges: every length residue mod 4 (the last dword's tail mask),
    both ends of the length range where only the window's last step is partial,
    gaps between packets, partial last runs; bit-exact against the oracle."""
    mod = {"udp": O.MODE_UDP, "tcp": O.MODE_TCP}[mode]
    stride = (length + 3) // 4 * 4 + 4 * gap
    assert batch.variant(stride, length, mode, 0, n=n) == "k_small<16,6>"
    assert n // 16 >= 8 * torch.cuda.get_device_properties(dev).multi_processor_count  # runs
    g = torch.Generator(device=dev)
    g.manual_seed(length * 7 + gap)
    total = (n - 1) * stride + length
    d = torch.randint(0, 256, (total + 16,), dtype=torch.uint8, device=dev, generator=g)
    if mode == "tcp":  # DataOffset 5
        d[12: 12 + (n - 1) * stride + 1: stride] = 0x50
    ad = torch.randint(0, 256, (8 * n,), dtype=torch.uint8, device=dev, generator=g)
    got = batch.checksum_uniform(d, stride, length, n, mode, addrs=ad).cpu().numpy()
    want = oracle_c.batch(d.cpu().numpy(), mod, stride=stride, length=length, n=n,
                          addrs=ad.cpu().numpy(), threads=8)
    assert np.array_equal(got, want), np.nonzero(got != want)[0][:10]


def test_full_size_fill_then_verify_round_trip(dev):
    """Size-independent property at BASELINE config 3 and 4 sizes: writing the TX
    field in place (yu_csum_fill_*, SetChecksum semantics) and then verifying the same
    bytes (checker semantics) accepts every packet; flipping one bit in a chosen set
    of packets rejects exactly that set."""
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    n, L = 1 << 20, 1500  # config 3
    d = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=g)
    d.view(n, L)[:, 12] = 0x50
    a = torch.randint(0, 256, (8 * n,), dtype=torch.uint8, device=dev, generator=g)
    batch.checksum_uniform(d, L, L, n, "tcp", addrs=a, fill=True)
    ok = batch.verified(batch.checksum_uniform(d, L, L, n, "verify_tcp", addrs=a))
    assert bool(ok.all())
    bad = torch.randperm(n, device=dev, generator=g)[:1000]
    pos = bad * L + 20 + torch.randint(0, L - 20, (1000,), device=dev, generator=g)
    d[pos] ^= 0x04
    ok = batch.verified(batch.checksum_uniform(d, L, L, n, "verify_tcp", addrs=a))
    mask = torch.ones(n, dtype=torch.bool, device=dev)
    mask[bad] = False
    assert torch.equal(ok, mask)
    del d
    # config 4 shape, UDP datagrams packed back to back (4-aligned offsets for fill)
    rng = np.random.default_rng(4)
    lens = (rng.integers(64, 9001, size=n) + 3) & ~3
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    r = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device=dev, generator=g)
    o = _to(dev, offs)
    batch.checksum_ragged(r, o, "udp", addrs=a, fill=True)
    ok = batch.verified(batch.checksum_ragged(r, o, "verify_udp", addrs=a))
    assert bool(ok.all())


def test_raw_packets_beyond_2GiB(dev, oracle_c):
    """RAW packets longer than 2 GiB (buffer-descriptor extents are 2 GiB; windows and
    tiles re-base) with the reference's uint32 wrap, uniform and ragged, against the
    oracle."""
    big = (5 << 29) + 3  # 2.5 GiB + 3, odd
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    d = torch.randint(0, 256, (big + 1000,), dtype=torch.uint8, device=dev, generator=g)
    host = d.cpu().numpy()
    got = batch.checksum_uniform(d, big, big, 1, "raw", initial=0x1234).cpu().numpy()
    assert int(got[0]) == oracle_c.checksum(host[:big].tobytes(), 0x1234)
    offs = np.array([0, 17, 17 + big, 17 + big + 980], np.int64)
    got = batch.checksum_ragged(d, _to(dev, offs), "raw", initial=0xFFFF).cpu().numpy()
    want = oracle_c.batch(host, O.MODE_RAW, offsets=offs.astype(np.uint64), initial=0xFFFF)
    assert np.array_equal(got, want)


def test_more_than_2pow32_packets(dev):
    """A batch of 2^32 + 5 one-byte packets (stride 1): packet indices, side-array and
    result offsets past 32 bits. Checksum of one odd byte b with initial i is
    fold(i + (b << 8)) (checksum/checksum.go:8-11,17); checked on the device in
    slices against that closed form."""
    n = (1 << 32) + 5
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    d = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev, generator=g)
    out = batch.checksum_uniform(d, 1, 1, n, "raw", initial=0xFFF0)
    step = 1 << 28
    for a in range(0, n, step):
        b = min(n, a + step)
        x = (d[a:b].to(torch.int32) << 8) + 0xFFF0
        x = (x & 0xFFFF) + (x >> 16)
        assert torch.equal(out[a:b].view(torch.int16).to(torch.int32) & 0xFFFF, x), a
    assert int(out[-1].view(torch.int16)) & 0xFFFF == int(x[-1])


def test_direct_path_back_to_back_bursts(dev, oracle_c):
    """Hundreds of consecutive small bursts through the direct host path (results
    read back by polling a GPU-written completion flag), each with fresh bytes and a
    changing size, so a result read before it landed would show as a mismatch."""
    rng = np.random.default_rng(41)
    pin = torch.empty(64 * 1500, dtype=torch.uint8).pin_memory()
    for it in range(400):
        n = int(rng.integers(1, 65))
        L = int(rng.choice([40, 64, 576, 1500]))
        host = _rand(rng, n * L)
        addrs = _rand(rng, 8 * n)
        want = oracle_c.batch(host, O.MODE_UDP, stride=L, length=L, n=n, addrs=addrs)
        if it % 2:
            pin[: n * L].copy_(torch.from_numpy(host))
            got = batch.checksum_host_uniform(pin[: n * L], L, L, n, "udp", addrs=addrs)
        else:
            got = batch.checksum_host_uniform(host, L, L, n, "udp", addrs=addrs)
        assert np.array_equal(got, want), (it, n, L)


@pytest.mark.parametrize("packed,shift", [(False, 0), (True, 1), (True, 3)])
def test_fill_ragged_ipv4_headers(dev, oracle_c, packed, shift):
    """Ragged IPv4 TX in place (k_hdr): the header field written big-endian equals
    the oracle's value, and the filled headers verify (checker.IPv4). `packed`:
    lengths as drawn (not rounded to 4) and the batch 1 or 3 bytes past a dword, so
    fields lie at every address parity: only bytes 10-11 of each header
    change, and the bytes before the batch stay."""
    rng = np.random.default_rng(43 + shift)
    n = 3000
    lens = rng.integers(20, 1501, size=n)
    if not packed:
        lens = (lens + 3) & ~3
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = _rand(rng, int(offs[-1]))
    for i in range(n):
        s = int(offs[i])
        ihl = int(rng.integers(5, 16))
        blob[s] = 0x40 | (ihl if ihl * 4 <= lens[i] else 5)
    want = oracle_c.batch(blob, O.MODE_IPV4, offsets=offs)
    pre = _rand(rng, shift)
    whole = _to(dev, np.concatenate([pre, blob, np.zeros(16, np.uint8)]))
    d = whole[shift:]
    got = batch.checksum_ragged(d, _to(dev, offs.view(np.int64)), "ipv4", fill=True).cpu().numpy()
    assert np.array_equal(got, want)
    filled = d.cpu().numpy()[:blob.size]
    st = offs[:-1].astype(np.int64)
    exp = blob.copy()
    exp[st + 10] = (want >> 8).astype(np.uint8)
    exp[st + 11] = (want & 0xFF).astype(np.uint8)
    bad = np.nonzero(filled != exp)[0]
    assert bad.size == 0, bad[:10]
    assert np.array_equal(whole[:shift].cpu().numpy(), pre)
    if packed:
        assert ((st + 10 + shift) & 1).any() and (((st + 10 + shift) & 1) == 0).any()
    v = batch.checksum_ragged(d[:blob.size], _to(dev, offs.view(np.int64)), "verify_ipv4")
    assert bool(batch.verified(v).all())


_MIN_LEN = {O.MODE_UDP: 8, O.MODE_TCP: 20, O.MODE_VERIFY_TCP: 20, O.MODE_ICMP: 4,
            O.MODE_IPV4: 1, O.MODE_VERIFY_IPV4: 1}
_FIELD = {O.MODE_UDP: 6, O.MODE_TCP: 16, O.MODE_ICMP: 2}


def _fuzz_lens(rng, n, lo):
    kind = int(rng.integers(0, 4))
    if kind == 0:   # tiny
        hi = 80
    elif kind == 1:  # tun-like
        hi = 1600
    elif kind == 2:  # mixed with jumbo
        hi = 9100
    else:            # one size
        return np.full(n, int(rng.integers(lo, 2000)), np.int64)
    return rng.integers(lo, max(lo, hi) + 1, size=n)


def _fuzz_headers(rng, blob, starts, lens, mode):
    for s, ln in zip(starts, lens):
        s, ln = int(s), int(ln)
        if mode in (O.MODE_TCP, O.MODE_VERIFY_TCP):
            blob[s + 12] = (4 * int(rng.integers(5, min(60, ln) // 4 + 1)) // 4) << 4
        if mode in (O.MODE_IPV4, O.MODE_VERIFY_IPV4):
            ihl = int(rng.integers(0, 16))
            blob[s] = 0x40 | (ihl if ihl * 4 <= ln else ln // 4 & 0xF)


def test_random_batches_fuzz(dev, oracle_c):
    """Randomised geometry x mode x side data x fill: every kernel variant the
    selection can pick (k_tiny, k_lane, k_small, k_hdr, k_seg, k_loop), against the
    C oracle on the same bytes. Seeded, so a failure reproduces."""
    import os
    # YU_FUZZ_SEED / YU_FUZZ_ITERS: longer or different runs by hand; YU_FUZZ_NBIG
    # raises the largest batch size drawn (default 6000; 70000 reaches the 16-packet
    # k_seg chunks of ragged batches up to 65535 and the uniform k_seg choice at 64K)
    rng = np.random.default_rng(int(os.environ.get("YU_FUZZ_SEED", "2026")))
    nbig = int(os.environ.get("YU_FUZZ_NBIG", "6000"))
    iters = int(os.environ.get("YU_FUZZ_ITERS", "800"))
    seen = set()
    for it in range(iters):
        if iters > 800 and it % 100 == 0:
            print(f"fuzz {it}/{iters} variants so far: {sorted(seen)}", flush=True)
        mode = int(rng.integers(0, 8))  # VERIFY_RX has its own tests (real headers)
        lo = _MIN_LEN.get(mode, 0)
        n = int(rng.choice([1, 2, 63, 64, 65, int(rng.integers(1, 3000)), int(rng.integers(4097, nbig))]))
        ragged = bool(rng.integers(0, 2))
        side = int(rng.integers(0, 3))  # 0: scalar initial, 1: initial_arr, 2: addrs
        tx = mode in _FIELD or mode == O.MODE_IPV4
        fill = tx and bool(rng.integers(0, 2))
        init = rng.integers(0, 65536, size=n, dtype=np.uint16) if side == 1 else None
        addrs = _rand(rng, 8 * n) if side == 2 else None
        initial = int(rng.integers(0, 65536)) if side == 0 else 0
        if ragged:
            lens = _fuzz_lens(rng, n, lo)
            base = int(rng.integers(0, 16))
            offs = np.zeros(n + 1, np.uint64)
            offs[1:] = np.cumsum(lens)
            offs += base
            blob = _rand(rng, int(offs[-1]) + 16, ["rand", "rand", "rand", "zero", "ff"][it % 5])
            _fuzz_headers(rng, blob, offs[:-1], lens, mode)
            want = oracle_c.batch(blob, mode, offsets=offs, initial_arr=init, initial=initial, addrs=addrs)
            dshift = it % 4  # the data pointer itself at every alignment (no rng draw)
            d = _to(dev, np.concatenate([np.zeros(dshift, np.uint8), blob]))[dshift:]
            seen.add(batch.ragged_variant(mode, n, fill=fill))
            got = batch.checksum_ragged(d, _to(dev, offs.view(np.int64)), mode, initial=initial,
                                        initial_arr=None if init is None else _to(dev, init),
                                        addrs=None if addrs is None else _to(dev, addrs),
                                        fill=fill).cpu().numpy()
            starts = offs[:-1].astype(np.int64)
        else:
            length = int(_fuzz_lens(rng, 1, lo)[0])
            align = 0 if fill else int(rng.integers(0, 4))
            pad = int(rng.integers(0, 3)) * (4 if fill else int(rng.integers(1, 6)))
            stride = (length + 3) // 4 * 4 + pad if fill else length + pad
            blob = _rand(rng, align + (n - 1) * stride + length + 16, ["rand", "zero", "ff"][it % 3])
            starts = align + stride * np.arange(n, dtype=np.int64)
            _fuzz_headers(rng, blob, starts, np.full(n, length), mode)
            want = oracle_c.batch(blob[align:], mode, stride=stride, length=length, n=n,
                                  initial_arr=init, initial=initial, addrs=addrs)
            d = _to(dev, blob)
            seen.add(batch.variant(stride, length, mode, align, n=n))
            got = batch.checksum_uniform(d[align:], stride, length, n, mode, initial=initial,
                                         initial_arr=None if init is None else _to(dev, init),
                                         addrs=None if addrs is None else _to(dev, addrs),
                                         fill=fill).cpu().numpy()
        assert np.array_equal(got, want), (it, mode, ragged, n, side, fill, np.nonzero(got != want)[0][:8])
        if fill:
            h = d.cpu().numpy()
            f = _FIELD.get(mode, 10)  # IPv4: the header checksum field
            may = np.zeros(len(blob), bool)  # bytes the writer may change: the fields
            may[starts + f] = True
            may[starts + f + 1] = True
            assert np.array_equal(h[~may], blob[~may]), (it, mode, ragged, "bytes outside the fields changed")
            if mode in _FIELD:
                fields = (h[starts + f].astype(np.uint16) << 8) | h[starts + f + 1]
                assert np.array_equal(fields, want), (it, mode, ragged)
    assert {"k_tiny<4>", "k_small<16,6>", "k_hdr"} <= seen or len(seen) >= 6, seen


def test_host_fill_paths(dev, oracle_c):
    """Host-memory field writer (yu_csum_fill_host_*): each TX field is set to the
    oracle's value in the caller's buffer, nothing else changes, and the filled
    packets verify. Covers the direct (small) and pipelined (large) host paths,
    views that split the field, and IPv4 headers whose IHL leaves no room."""
    rng = np.random.default_rng(909)
    fld = {O.MODE_UDP: 6, O.MODE_TCP: 16, O.MODE_ICMP: 2, O.MODE_IPV4: 10}

    def check(before, after, starts, want, mode, may_skip=None):
        f = fld[mode]
        may = np.zeros(len(before), bool)
        may[starts + f] = True
        may[starts + f + 1] = True
        assert np.array_equal(after[~may], before[~may])
        got = (after[starts + f].astype(np.uint16) << 8) | after[starts + f + 1]
        keep = np.ones(len(starts), bool) if may_skip is None else ~may_skip
        assert np.array_equal(got[keep], want[keep])
        if may_skip is not None:  # no room for the field: left as it was
            assert np.array_equal(after[starts[may_skip] + f], before[starts[may_skip] + f])

    for n, L in ((300, 1500), (40_000, 1500), (5000, 72)):  # direct, pipelined, small
        for mode in (O.MODE_UDP, O.MODE_TCP, O.MODE_ICMP):
            host = _rand(rng, n * L)
            if mode == O.MODE_TCP:
                host[12::L] = 0x50
            addrs = _rand(rng, 8 * n)
            want = oracle_c.batch(host, mode, stride=L, length=L, n=n,
                                  addrs=addrs if mode in (1, 2) else None)
            buf = host.copy()
            out = batch.checksum_host_uniform(buf, L, L, n, mode, addrs=addrs if mode in (1, 2) else None,
                                              fill=True)
            assert np.array_equal(out, want)
            check(host, buf, L * np.arange(n), want, mode)
    # ragged IPv4 headers, some with IHL < 3 (field outside the header: not written)
    n = 2000
    lens = rng.integers(20, 1501, size=n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = _rand(rng, int(offs[-1]))
    starts = offs[:-1].astype(np.int64)
    ihl = rng.integers(0, 16, size=n)
    blob[starts] = (0x40 | ihl).astype(np.uint8)
    want = oracle_c.batch(blob, O.MODE_IPV4, offsets=offs)
    buf = blob.copy()
    out = batch.checksum_host_ragged(buf, offs, "ipv4", fill=True)
    assert np.array_equal(out, want)
    check(blob, buf, starts, want, O.MODE_IPV4, may_skip=np.minimum(ihl * 4, lens) < 12)
    v = batch.checksum_host_ragged(buf, offs, "verify_ipv4")
    assert np.isin(v[np.minimum(ihl * 4, lens) >= 12], (0, 0xFFFF)).all()
    # scatter-gather UDP datagrams split inside the 8-byte header (the field straddles)
    n = 500
    pk = [_rand(rng, int(rng.integers(8, 300))) for _ in range(n)]
    addrs = _rand(rng, 8 * n)
    flat = np.concatenate(pk)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in pk])
    want = oracle_c.batch(flat, O.MODE_UDP, offsets=offs, addrs=addrs)
    views = [[p[:7], p[7:]] for p in [p.copy() for p in pk]]
    out = batch.checksum_host_iov(views, "udp", addrs=addrs, fill=True)
    assert np.array_equal(out, want)
    after = np.concatenate([np.concatenate(v) for v in views])
    check(flat, after, offs[:-1].astype(np.int64), want, O.MODE_UDP)
    with pytest.raises(TypeError):
        batch.checksum_host_iov([[bytes(8)]], "udp", fill=True)


def test_uniform_large_dense_batches_take_k_seg(dev, oracle_c):
    """Dense uniform packets in a large batch that go to k_seg (above 3 KiB, 129..704
    bytes, or not 4-aligned): parity for TCP / UDP / RAW / VERIFY_UDP."""
    rng = np.random.default_rng(31)
    cases = ((4100, O.MODE_TCP, 70_000, "k_seg<8,tx>"), (9001, O.MODE_RAW, 65_536, "k_seg<8>"),
             (300, O.MODE_TCP, 70_000, "k_seg<4,tx>"), (66, O.MODE_UDP, 70_000, "k_seg<4,tx>"),
             (500, O.MODE_VERIFY_UDP, 65_536, "k_seg<8>"))
    for L, mode, n, want_kernel in cases:
        assert FORCED or batch.variant(L, L, mode, 0, n=n) == want_kernel
        host = _rand(rng, n * L)
        if mode == O.MODE_TCP:
            host[12::L] = 0x50
        addrs = _rand(rng, 8 * n) if mode in (O.MODE_TCP, O.MODE_UDP, O.MODE_VERIFY_UDP) else None
        init = rng.integers(0, 65536, size=n, dtype=np.uint16) if mode == O.MODE_RAW else None
        got = batch.checksum_uniform(_to(dev, host), L, L, n, mode,
                                     addrs=None if addrs is None else _to(dev, addrs),
                                     initial_arr=None if init is None else _to(dev, init)).cpu().numpy()
        want = oracle_c.batch(host, mode, stride=L, length=L, n=n, addrs=addrs, initial_arr=init, threads=8)
        assert np.array_equal(got, want), (L, mode)


@pytest.mark.parametrize("mode", [O.MODE_RAW, O.MODE_UDP, O.MODE_VERIFY_TCP, O.MODE_VERIFY_RX])
def test_ragged_batch_size_cutovers(dev, oracle_c, mode):
    """The same kind of burst at each ragged cut-over: a wave per packet (<= 4096),
    16-packet k_seg chunks (< 65536) and 64-packet ones, all bit-exact."""
    import rxgen
    for npk, want in ((4096, "k_loop"), (4097, "c16"), (65535, "c16"), (65536, "k_seg")):
        name = batch.ragged_variant(mode, npk)
        assert FORCED or name.startswith(want) or want in name, (npk, name)
        if npk == 65536 and not FORCED:
            assert "c16" not in name
        rng = np.random.default_rng(npk + mode)
        if mode == O.MODE_VERIFY_RX:
            blob, offs = rxgen.rx_batch(rng, npk, lo=0, hi=300)
        else:
            lens = rng.integers(20 if mode == O.MODE_VERIFY_TCP else 8, 400, size=npk)
            blob, offs = _ragged(rng, lens, base_off=1)
            if mode == O.MODE_VERIFY_TCP:
                blob[offs[:-1].astype(np.int64) + 12] = 0x50
        addrs = _rand(rng, 8 * npk) if mode in (O.MODE_UDP, O.MODE_VERIFY_TCP) else None
        got = batch.checksum_ragged(_to(dev, blob), _to(dev, offs.view(np.int64)), mode,
                                    addrs=None if addrs is None else _to(dev, addrs)).cpu().numpy()
        want_v = oracle_c.batch(blob, mode, offsets=offs, addrs=addrs, threads=8)
        assert np.array_equal(got, want_v), (mode, npk, np.nonzero(got != want_v)[0][:8])

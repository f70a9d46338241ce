"""Out-of-contract device ragged batches (include/yucsum.h, "Out of contract").

The device ragged calls never read their offsets back on the host, so a batch may
hold packets whose offsets decrease or whose length passes the mode's limit. The
reference's SetChecksum can only write its own two bytes (header/udp.go:60-62,
header/tcp.go:156-158, header/ipv4.go:165-167, header/icmpv4.go:46-48); the
in-place writers here promise the same for every in-contract packet: no byte
outside the checksum fields of in-contract packets is ever written, an
out-of-contract packet gets an unspecified result and no store, and the k_seg
kernels that take c consecutive packets at a time (16..64) also leave the other
packets of that group unwritten, with unspecified results. Every other packet's
result and field are exact.

Corruptions (seeded, applied to clean batches whose oracle values are known):
  hi32  offsets[k] += 2^32: packet k-1 is 2^32 bytes too long and packet k has a
        negative length, while every low dword is unchanged (what a 32-bit view of
        the offsets cannot see);
  long  packet k spans more than 65535 bytes, the packets it swallows are empty;
  down  offsets[k] moved 2 bytes before offsets[k-1] (packet k-1 negative,
        packet k starts inside packet k-2's tail);
  past  packet k moved past offsets[n] (a well-sized packet outside what the call
        may touch, data[0, offsets[n]); its neighbours' lengths go wrong with it).
The device buffer has 4 KiB of padding past offsets[n], so a store that escaped
the batch would land in it (and be seen) rather than outside the allocation.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from yustack_amd import batch

pytestmark = pytest.mark.gpu

_FIELD = {O.MODE_UDP: 6, O.MODE_TCP: 16, O.MODE_ICMP: 2}
_LO = {O.MODE_UDP: 8, O.MODE_TCP: 20, O.MODE_ICMP: 4, O.MODE_IPV4: 20, O.MODE_RAW: 0,
       O.MODE_VERIFY_RX: 0, O.MODE_TX_DATAGRAM: 0}
_NAME = {O.MODE_UDP: "udp", O.MODE_TCP: "tcp", O.MODE_ICMP: "icmp", O.MODE_IPV4: "ipv4",
         O.MODE_RAW: "raw", O.MODE_VERIFY_RX: "verify_rx", O.MODE_TX_DATAGRAM: "tx_datagram"}


def _to(dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _group(name: str) -> int:
    """Packets per group whose fields a bad packet takes with it: the writing k_seg
    kinds (tx, txw, dg) check whole chunks, k_hdr whole 64-packet steps (one buffer
    descriptor from lane 0's packet); per-packet kernels and the read-only k_seg kinds
    only the packet itself."""
    if name == "k_hdr":
        return 64
    if not name.startswith("k_seg<") or not any(t in name for t in (",tx", ",dg")):
        return 1
    for part in name[6:-1].split(","):
        if part.startswith("c") and part[1:].isdigit():
            return int(part[1:])
    return 64


def _clean_batch(rng, mode, n):
    if mode == O.MODE_TX_DATAGRAM or mode == O.MODE_VERIFY_RX:
        import rxgen
        return rxgen.tx_batch(rng, n, lo=0, hi=200, bad=0.1)
    lo = _LO[mode]
    lens = rng.integers(max(lo, 1), 201, size=n)
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)
    s = offs[:-1].astype(np.int64)
    if mode == O.MODE_TCP:
        blob[s + 12] = 0x50
    if mode == O.MODE_IPV4:
        ihl = rng.integers(5, 16, size=n)
        blob[s] = 0x40 | np.where(ihl * 4 <= lens, ihl, 5)
    return blob, offs


def _corrupt(rng, offs, kinds, sites):
    """Corrupted copy of offs (uint64) at the given packet indices, one kind each."""
    o = offs.copy()
    for kind, k in zip(kinds, sites):
        if kind == "hi32":
            o[k] += np.uint64(1 << 32)
        elif kind == "long":  # packet k swallows its successors until it passes 65535 bytes
            m = k + 1
            while int(offs[m]) - int(offs[k]) <= 70000:
                m += 1
            o[k + 1:m] = offs[m]
        elif kind == "past":
            o[k], o[k + 1] = offs[-1] + np.uint64(1000), offs[-1] + np.uint64(1100)
        elif kind == "rand":  # anywhere from just past the batch to 2^40 bytes further
            o[k] = offs[-1] + np.uint64(int(rng.integers(1, 1 << 40)))
        else:  # down
            o[k] = offs[k - 1] - np.uint64(2)
    return o


def _fields(mode, blob, s, e, vals):
    """(byte index, value) of the field bytes packet [s, e) stores when its field is
    defined, as the writers decide (include/yucsum.h)."""
    ln = e - s
    if mode in _FIELD:
        f = _FIELD[mode]
        return [(s + f, vals[0] >> 8), (s + f + 1, vals[0] & 0xFF)] if ln >= f + 2 else []
    if mode == O.MODE_IPV4:
        hl = (int(blob[s]) & 15) * 4 if ln >= 1 else 0
        return [(s + 10, vals[0] >> 8), (s + 11, vals[0] & 0xFF)] if min(ln, hl) >= 12 else []
    # TX_DATAGRAM: both fields where defined (tests/test_gpu_parity.py _tx_expected)
    if ln < 20:
        return []
    pk = blob[s:e]
    hl, tl = (int(pk[0]) & 15) * 4, (int(pk[2]) << 8) | int(pk[3])
    if hl < 20 or hl > tl or tl > ln:
        return []
    out = [(s + 10, vals[0] >> 8), (s + 11, vals[0] & 0xFF)]
    fo, mn = {17: (6, 8), 6: (16, 20), 1: (2, 4)}.get(int(pk[9]), (0, 0))
    if fo and tl - hl >= mn:
        out += [(s + hl + fo, vals[1] >> 8), (s + hl + fo + 1, vals[1] & 0xFF)]
    return out


def _run(dev, oracle_c, mode, n, kind, fill, seed, nsites=None):
    """kind: one corruption for every site, or a list (site i takes kinds[i])."""
    rng = np.random.default_rng(seed)
    blob, offs = _clean_batch(rng, mode, n)
    k_out = 2 if mode == O.MODE_TX_DATAGRAM else 1
    addrs = rng.integers(0, 256, size=8 * n, dtype=np.uint8) if mode in (O.MODE_UDP, O.MODE_TCP) else None
    want = oracle_c.batch(blob, mode, offsets=offs, addrs=addrs).reshape(n, k_out)
    # corruption sites, away from the ends. The read-only kinds bound a chunk's span
    # only, so their sites stay off chunk edges (k = 5 mod 16: no chunk of 16..64
    # packets starts there); `down` needs packet k-2 long enough that its field is not
    # among the moved packet k's first bytes (that packet reads them while they are
    # written). The writing kinds also get k = 3840, a chunk edge for every chunk size
    # (16, 40, 48, 64), where a chunk's first offset is the corrupt one.
    lens = np.diff(offs.astype(np.int64))
    nsites = nsites or (1 if n <= 4096 else 3)
    kinds = [kind] * nsites if isinstance(kind, str) else list(kind)
    cand = np.arange(8, n - 1000)
    if not fill:
        cand = cand[cand % 16 == 5]
    sites = []
    if fill and 3840 < n - 1000 and (kinds[0] != "down" or lens[3838] >= 16):
        sites = [3840]
    for _ in range(20000):  # >= 1000 packets apart (a long packet swallows <= ~900)
        if len(sites) == nsites:
            break
        k = int(rng.choice(cand))
        if kinds[len(sites)] == "down" and lens[k - 2] < 16:
            continue
        if all(abs(k - x) >= 1000 for x in sites):
            sites.append(k)
    nsites = len(sites)  # (random placement may fit fewer than asked)
    kinds = kinds[:nsites]
    order = np.argsort(sites)
    sites, kinds = [sites[i] for i in order], [kinds[i] for i in order]
    bad_offs = _corrupt(rng, offs, kinds, sites)
    name = batch.ragged_variant(_NAME[mode], n, fill=fill)
    c = _group(name)
    s_all, e_all = bad_offs[:-1].astype(np.int64), bad_offs[1:].astype(np.int64)
    ln = e_all - s_all  # (int64: negative for decreasing offsets, ~2^32 for hi32)
    in_c = (ln >= 0) & (ln <= (0xFFFF0000 if mode == O.MODE_RAW else 65535)) & (e_all <= int(bad_offs[-1]))
    if c > 1:
        g_bad = np.zeros((n + c - 1) // c, bool)
        np.logical_or.at(g_bad, np.arange(n) // c, ~in_c)
        clean = in_c & ~g_bad[np.arange(n) // c]
    else:
        clean = in_c
    same = (s_all == offs[:-1].astype(np.int64)) & (e_all == offs[1:].astype(np.int64))
    # (a RAW packet past 65535 bytes is in contract: `long` then only moves packets)
    assert ((~in_c).sum() >= nsites or (mode == O.MODE_RAW and "long" in kinds)) and clean.mean() > 0.7, (
        name, (~in_c).sum(), clean.mean())

    # expected results of the clean packets: the clean batch's, or (moved packets) the
    # oracle on the packet alone
    exp_val = want.copy()
    check = clean.copy()
    for i in np.nonzero(clean & ~same)[0]:
        if ln[i] == 0:
            check[i] = False  # an empty packet swallowed by a long one: no field, result not compared
            continue
        a = None if addrs is None else addrs[8 * i:8 * i + 8]
        exp_val[i] = oracle_c.batch(blob, mode, offsets=np.array([s_all[i], e_all[i]], np.uint64), addrs=a)
    pad = rng.integers(0, 256, size=4096, dtype=np.uint8)
    d = _to(dev, np.concatenate([blob, pad]))
    got = batch.checksum_ragged(d, _to(dev, bad_offs.view(np.int64)), _NAME[mode],
                                addrs=None if addrs is None else _to(dev, addrs),
                                fill=fill, validate=False).cpu().numpy().reshape(n, k_out)
    torch.cuda.synchronize()
    badv = np.nonzero(check & (got != exp_val).any(axis=1))[0]
    assert badv.size == 0, (name, kinds, sites, badv[:10])
    if not fill:
        return name, c
    # every byte outside the clean packets' defined fields is unchanged
    exp = np.concatenate([blob, pad])
    owner = {}
    for i in np.nonzero(clean)[0]:
        for pos, v in _fields(mode, blob, int(s_all[i]), int(e_all[i]), [int(x) for x in exp_val[i]]):
            assert pos not in owner, ("test layout: overlapping fields", owner[pos], i)
            owner[pos] = i
            exp[pos] = v
    filled = d.cpu().numpy()
    diff = np.nonzero(filled != exp)[0]
    assert diff.size == 0, (name, kinds, sites, diff[:10], [owner.get(int(x)) for x in diff[:10]])
    return name, c


# (mode, n): bursts (a wave per packet), 16-packet chunks, the large-batch chunks
_FILL_CASES = [(O.MODE_UDP, 3000), (O.MODE_UDP, 5000), (O.MODE_UDP, 70000), (O.MODE_TCP, 70000),
               (O.MODE_ICMP, 5000), (O.MODE_TX_DATAGRAM, 3000), (O.MODE_TX_DATAGRAM, 5000),
               (O.MODE_TX_DATAGRAM, 70000), (O.MODE_IPV4, 5000)]


@pytest.mark.parametrize("kind", ["hi32", "long", "down", "past"])
@pytest.mark.parametrize("mode,n", _FILL_CASES)
def test_fill_out_of_contract_writes_only_clean_fields(dev, oracle_c, mode, n, kind):
    """In place on ragged batches with out-of-contract packets: every clean packet's
    result and field equal the oracle's, and no other byte changes: no field of an
    out-of-contract packet, nor of the k_seg group holding one, and nothing outside
    fields (include/yucsum.h). `down` moves a TCP segment's or a
    datagram's start, whose contracts (DataOffset, IHL) then make its value
    unspecified: those modes take hi32 and long only."""
    if kind == "down" and mode in (O.MODE_TCP, O.MODE_TX_DATAGRAM):
        pytest.skip("a moved start leaves the mode's own contract")
    name, c = _run(dev, oracle_c, mode, n, kind, True, 7100 + 17 * mode + n + len(kind))
    print(f"{_NAME[mode]} n={n} {kind}: {name}, group {c}")


@pytest.mark.parametrize("kind", ["hi32", "long", "down", "past"])
@pytest.mark.parametrize("mode,n", [(O.MODE_RAW, 5000), (O.MODE_RAW, 70000), (O.MODE_UDP, 70000),
                                    (O.MODE_VERIFY_RX, 70000), (O.MODE_RAW, 3000)])
def test_results_next_to_out_of_contract_packets(dev, oracle_c, mode, n, kind):
    """Result arrays only: the read-only k_seg kinds (RAW, VERIFY_RX) keep every
    in-contract packet exact next to an out-of-contract one, and bound the work of a
    chunk whose offsets claim 4 GiB (no hang); the TX kind (UDP results) leaves its
    group unspecified and every other packet exact."""
    if kind == "down" and mode == O.MODE_VERIFY_RX:
        pytest.skip("a moved start leaves the datagram contract")
    name, c = _run(dev, oracle_c, mode, n, kind, False, 7300 + 17 * mode + n + len(kind))
    print(f"{_NAME[mode]} n={n} {kind}: {name}, group {c}")


def test_out_of_contract_fuzz(dev, oracle_c):
    """Seeded: 16 batches (YU_CONTRACT_FUZZ_ITERS) of 1100 to 80000 packets, every
    mode that has a ragged kernel (and its in-place form where it has one), 1 to 4
    sites each with a random
    corruption among hi32 / long / down / past / rand (rand: offsets[k] anywhere from
    just past the batch to 2^40 bytes beyond). Same checks as above: clean packets
    exact, no byte outside their fields changed, nothing written into the padding."""
    import os
    rng = np.random.default_rng(int(os.environ.get("YU_CONTRACT_FUZZ_SEED", "7500")))
    iters = int(os.environ.get("YU_CONTRACT_FUZZ_ITERS", "16"))
    modes = [O.MODE_RAW, O.MODE_UDP, O.MODE_TCP, O.MODE_ICMP, O.MODE_IPV4, O.MODE_VERIFY_RX,
             O.MODE_TX_DATAGRAM]
    seen = set()
    for it in range(iters):
        mode = modes[int(rng.integers(0, len(modes)))]
        fill = mode not in (O.MODE_RAW, O.MODE_VERIFY_RX) and bool(rng.integers(0, 2))
        n = int(rng.choice([1100, 3000, 4096, 4097, 9000, 30000, 65536, 80000]))
        # (sites >= 1000 packets apart in [8, n - 1000))
        nsites = int(rng.integers(1, min(4, 1 + (n - 1008) // 1000) + 1))
        allowed = ["hi32", "past", "rand"] + (["long"] if n >= 2100 else [])
        if mode not in (O.MODE_TCP, O.MODE_TX_DATAGRAM, O.MODE_VERIFY_RX):
            allowed.append("down")
        kinds = [allowed[int(rng.integers(0, len(allowed)))] for _ in range(nsites)]
        name, c = _run(dev, oracle_c, mode, n, kinds, fill, int(rng.integers(0, 1 << 30)), nsites=nsites)
        seen.add(name)
        print(f"{it}: {_NAME[mode]} n={n} fill={fill} {kinds}: {name}, group {c}")
    forced = os.environ.get("YU_TUNING") == "1" and bool(os.environ.get("YU_RAGGED"))
    assert forced or len(seen) >= 6, seen  # (a forced ragged kernel narrows the choice)

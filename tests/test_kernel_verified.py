"""The oracle on datagrams the Linux kernel verified or built
(tests/golden/kernel_verified.npz, tests/golden/make_kernel_verified.py): TX_DATAGRAM
gives exactly the fields the kernel accepted, and VERIFY_RX passes the kernel's own
datagrams. The HIP path runs the same fixture in
tests/test_gpu_parity.py::test_kernel_verified_datagrams_on_gpu."""
import os

import numpy as np

from oracle import oracle as O

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "kernel_verified.npz")
RX_OK = 0x2 | 0x4  # YU_RX_IP_OK | YU_RX_L4_OK


def load():
    f = np.load(FIX)  # arrays only (allow_pickle stays off)
    return f["sent_blob"], f["sent_offs"], f["kernel_blob"], f["kernel_offs"]


def stored_fields(blob, offs):
    """The IPv4 and transport fields each datagram carries, and the blob with both zeroed."""
    z = blob.copy()
    want = []
    for s in offs[:-1].astype(np.int64):
        hl = int(blob[s] & 0xF) * 4
        fo = s + hl + {6: 16, 17: 6, 1: 2}[int(blob[s + 9])]
        want += [int(blob[s + 10]) << 8 | int(blob[s + 11]), int(blob[fo]) << 8 | int(blob[fo + 1])]
        z[s + 10:s + 12] = 0
        z[fo:fo + 2] = 0
    return z, np.array(want, np.uint16)


def test_fixture_shape():
    sb, so, kb, ko = load()
    assert len(so) - 1 >= 40 and len(ko) - 1 >= 40
    assert so[-1] == sb.size and ko[-1] == kb.size
    assert {int(kb[s + 9]) for s in ko[:-1].astype(np.int64)} == {1, 6, 17}


def test_oracle_tx_datagram_reproduces_kernel_accepted_fields():
    sb, so, _, _ = load()
    z, want = stored_fields(sb, so)
    for blob in (sb, z):  # the fields are left out of the sum, whatever they hold
        assert np.array_equal(O.C().batch(blob, O.MODE_TX_DATAGRAM, offsets=so), want)


def test_oracle_verify_rx_passes_kernel_datagrams():
    sb, so, kb, ko = load()
    for blob, offs in ((kb, ko), (sb, so)):
        got = O.C().batch(blob, O.MODE_VERIFY_RX, offsets=offs)
        assert np.all(got & RX_OK == RX_OK), got


def mode_cases():
    """Every batch mode on the fixture's datagrams, pooled from both sets: (mode,
    ragged blob, offsets, {src,dst} records or None, check). The transport modes take
    each datagram's segment (TCP / UDP / ICMP) and its addresses, the IPv4 modes its
    header. The TX modes see the field zeroed (Encode leaves it 0) and must give the
    stored value; the VERIFY modes see it as sent and must sum to 0 or 0xFFFF
    (checker/checker.go:32-35,80-92)."""
    sb, so, kb, ko = load()
    dg = [b[s:e] for b, o in ((sb, so), (kb, ko)) for s, e in zip(o[:-1].astype(np.int64), o[1:].astype(np.int64))]

    def pack(parts):
        offs = np.zeros(len(parts) + 1, np.uint64)
        offs[1:] = np.cumsum([len(x) for x in parts])
        return np.concatenate(parts + [np.zeros(16, np.uint8)]), offs

    cases = []
    for proto, tx, verify, fo in ((6, O.MODE_TCP, O.MODE_VERIFY_TCP, 16), (17, O.MODE_UDP, O.MODE_VERIFY_UDP, 6),
                                  (1, O.MODE_ICMP, None, 2)):
        segs, zsegs, addrs, fields = [], [], [], []
        for d in dg:
            if int(d[9]) != proto:
                continue
            hl, tl = int(d[0] & 0xF) * 4, int(d[2]) << 8 | int(d[3])
            seg = d[hl:tl].copy()
            fields.append(int(seg[fo]) << 8 | int(seg[fo + 1]))
            segs.append(seg.copy())
            seg[fo:fo + 2] = 0
            zsegs.append(seg)
            addrs.append(d[12:20])
        want = np.array(fields, np.uint16)
        ad = np.concatenate(addrs) if proto != 1 else None
        cases.append((tx, *pack(zsegs), ad, lambda got, want=want: np.array_equal(got, want)))
        if verify is not None:
            cases.append((verify, *pack(segs), ad, lambda got: np.all((got == 0) | (got == 0xFFFF))))
    hdrs, zhdrs, fields = [], [], []
    for d in dg:
        h = d[:int(d[0] & 0xF) * 4].copy()
        fields.append(int(h[10]) << 8 | int(h[11]))
        hdrs.append(h.copy())
        h[10:12] = 0
        zhdrs.append(h)
    want = np.array(fields, np.uint16)
    cases.append((O.MODE_IPV4, *pack(zhdrs), None, lambda got, want=want: np.array_equal(got, want)))
    cases.append((O.MODE_VERIFY_IPV4, *pack(hdrs), None, lambda got: np.all((got == 0) | (got == 0xFFFF))))
    return cases


def test_oracle_every_mode_on_kernel_datagrams():
    cases = mode_cases()
    assert {c[0] for c in cases} == {O.MODE_TCP, O.MODE_VERIFY_TCP, O.MODE_UDP, O.MODE_VERIFY_UDP,
                                     O.MODE_ICMP, O.MODE_IPV4, O.MODE_VERIFY_IPV4}
    for mode, blob, offs, addrs, check in cases:
        assert check(O.C().batch(blob, mode, offsets=offs, addrs=addrs)), mode

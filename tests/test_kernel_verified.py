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

"""Mirror of yustack's ``checksum`` package (reference: checksum/checksum.go).

The three package functions keep the reference's names, argument meaning and
(total, never-failing) error behaviour, and call the C ABI's scalar entry points —
the same ones a cgo shim binds:

=============================  ======================================  ============================
reference                      here                                    C ABI
=============================  ======================================  ============================
``Checksum(buf, initial)``     :func:`Checksum`                        ``yu_checksum``
``PseudoHeaderChecksum(...)``  :func:`PseudoHeaderChecksum`            ``yu_pseudo_header_checksum``
``ChecksumCombine(a, b)``      :func:`ChecksumCombine`                 ``yu_checksum_combine``
=============================  ======================================  ============================

Go ``string`` addresses (``types.Address``) map to Python ``bytes``/``str`` (a str is
taken byte-for-byte, latin-1, as Go's ``[]byte(string)`` does).

The batched GPU path — the reason this package exists — is in :mod:`yustack_amd.batch`.
"""
from __future__ import annotations

from ._lib import lib


def _bytes(x) -> bytes:
    if isinstance(x, str):
        return x.encode("latin-1")
    return bytes(x)


def Checksum(buf, initial: int) -> int:  # noqa: N802 - reference name
    """checksum/checksum.go:4-18 — uncomplemented 16-bit one's-complement sum."""
    b = _bytes(buf)
    return lib().yu_checksum(b, len(b), initial & 0xFFFF)


def PseudoHeaderChecksum(protocol: int, srcAddr, dstAddr) -> int:  # noqa: N802,N803
    """checksum/checksum.go:24-28 — pseudo-header partial sum (length excluded)."""
    s, d = _bytes(srcAddr), _bytes(dstAddr)
    return lib().yu_pseudo_header_checksum(protocol & 0xFFFFFFFF, s, len(s), d, len(d))


def ChecksumCombine(a: int, b: int) -> int:  # noqa: N802
    """checksum/checksum.go:32-35 — end-around-carry add of two uint16."""
    return lib().yu_checksum_combine(a & 0xFFFF, b & 0xFFFF)


# snake_case aliases
checksum = Checksum
pseudo_header_checksum = PseudoHeaderChecksum
checksum_combine = ChecksumCombine

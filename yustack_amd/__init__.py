"""yustack_amd — MI355X-native batched Internet-checksum engine for yustack.

Drop-in for the reference's ``checksum`` package (checksum/checksum.go): the scalar
Go-signature functions live in :mod:`yustack_amd.checksum`, the GPU hot path in
:mod:`yustack_amd.batch`, both over the C ABI of include/yucsum.h
(``yustack_amd/libyucsum.so``).
"""
from .checksum import Checksum, ChecksumCombine, PseudoHeaderChecksum  # noqa: F401

__all__ = ["Checksum", "ChecksumCombine", "PseudoHeaderChecksum"]
__version__ = "0.1.0"

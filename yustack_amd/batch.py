"""Batched Internet checksum on MI355X — the hot path.

Thin Python front end over the C ABI's batched entry points
(``yu_csum_batch_uniform`` / ``yu_csum_batch_ragged`` / ``yu_csum_fill_*`` /
``yu_csum_batch_host_uniform``, include/yucsum.h). PyTorch is used only for device
memory and streams: the arithmetic happens in the hand-written gfx950 kernels of
``csrc/yucsum_kernels.hip``. There is no CPU fallback — without a HIP device every
entry point raises :class:`yustack_amd._lib.YuError`.

Modes (each reproduces one reference composition, see include/yucsum.h):

=============  =========================================================================
RAW            ``Checksum(pkt, initial)``                     checksum/checksum.go:4-18
UDP            field value of sendUDP                          transport/udp/endpoint.go:164-187
TCP            field value of sendTCP                          transport/tcp/connect.go:556-586
IPV4           field value of ipv4 WritePacket                 network/ipv4/ipv4.go:80-97
ICMP           field value of sendICMPv4                       network/ipv4/icmp.go:36-45
VERIFY_IPV4    checker.IPv4 sum (valid iff 0 or 0xFFFF)        checker/checker.go:25-40
VERIFY_TCP     checker.TCP sum                                 checker/checker.go:71-99
VERIFY_UDP     the checker.TCP formula for UDP
VERIFY_RX      whole received IPv4 packets: IsValid + checker.IPv4 + checker.TCP's
               test, inputs read from each packet; out = YU_RX_* bits
                                                               checker/checker.go:25-99
TX_DATAGRAM    whole outgoing IPv4 datagrams: both fields (IPv4 header and its
               sender's transport field), inputs read from each datagram; TWO
               results per packet, out[2i] / out[2i+1]     network/ipv4/ipv4.go:80-97
=============  =========================================================================
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import check, lib

RAW, UDP, TCP, IPV4, ICMP, VERIFY_IPV4, VERIFY_TCP, VERIFY_UDP, VERIFY_RX, TX_DATAGRAM = range(10)
MODES = {"raw": RAW, "udp": UDP, "tcp": TCP, "ipv4": IPV4, "icmp": ICMP,
         "verify_ipv4": VERIFY_IPV4, "verify_tcp": VERIFY_TCP, "verify_udp": VERIFY_UDP,
         "verify_rx": VERIFY_RX, "tx_datagram": TX_DATAGRAM}
# VERIFY_RX result bits (include/yucsum.h YU_RX_*)
RX_IP_OK, RX_L4, RX_L4_OK, RX_INVALID = 1, 2, 4, 8
TX_MODES = (UDP, TCP, IPV4, ICMP, TX_DATAGRAM)
MAX_TRANSPORT_LEN = 65535
MAX_RAW_LEN = 0xFFFF0000  # include/yucsum.h YU_MAX_RAW_LEN


def _mode(m) -> int:
    m = MODES[m] if isinstance(m, str) else int(m)
    if not 0 <= m < len(MODES):
        raise ValueError(f"bad mode {m}")
    return m


def outputs(mode) -> int:
    """Results per packet (include/yucsum.h YU_MODE_OUTPUTS): 2 for TX_DATAGRAM."""
    return 2 if _mode(mode) == TX_DATAGRAM else 1


def _dev_u8(t: torch.Tensor, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a CUDA (HIP) tensor")
    if t.dtype != torch.uint8 or not t.is_contiguous():
        raise TypeError(f"{name} must be a contiguous uint8 tensor")
    return t


def _opt(t, dtype, numel, device, name):
    if t is None:
        return None
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.device != device:
        raise TypeError(f"{name} must be a CUDA tensor on {device}")
    if t.dtype != dtype or not t.is_contiguous() or t.numel() < numel:
        raise TypeError(f"{name} must be a contiguous {dtype} tensor with >= {numel} elements")
    return t


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(device, stream):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return s.cuda_stream


def checksum_uniform(data: torch.Tensor, stride: int, length: int, n: int, mode="raw", *,
                     initial: int = 0, initial_arr: torch.Tensor | None = None,
                     addrs: torch.Tensor | None = None, out: torch.Tensor | None = None,
                     stream: torch.cuda.Stream | None = None, fill: bool = False) -> torch.Tensor:
    """Per-packet sums of a uniform-stride device batch: packet i is
    ``data[i*stride : i*stride+length]``. Returns a uint16 tensor of n results (2n for TX_DATAGRAM)
    (allocated unless ``out`` is given). ``fill=True`` additionally stores each TX
    result big-endian into the packet's checksum field (in place)."""
    m = _mode(mode)
    _dev_u8(data, "data")
    if n < 0 or stride < 0 or not 0 <= length < 2 ** 32:
        raise ValueError("bad geometry")
    if n and (n - 1) * stride + length > data.numel():
        raise ValueError(f"batch needs {(n - 1) * stride + length} bytes, data has {data.numel()}")
    dev = data.device
    initial_arr = _opt(initial_arr, torch.uint16, n, dev, "initial_arr")
    addrs = _opt(addrs, torch.uint8, 8 * n, dev, "addrs")
    k = outputs(m)
    if out is None:
        out = torch.empty(max(n * k, 1), dtype=torch.uint16, device=dev)[:n * k]
    else:
        _opt(out, torch.uint16, n * k, dev, "out")
    with torch.cuda.device(dev):
        f = lib().yu_csum_fill_uniform if fill else lib().yu_csum_batch_uniform
        rc = f(data.data_ptr(), stride, length, n, m, _ptr(initial_arr), initial & 0xFFFF,
               _ptr(addrs), out.data_ptr() if n else None, _stream(dev, stream))
    check(rc, "yu_csum_fill_uniform" if fill else "yu_csum_batch_uniform")
    return out


def checksum_ragged(data: torch.Tensor, offsets: torch.Tensor, mode="raw", *, initial: int = 0,
                    initial_arr: torch.Tensor | None = None, addrs: torch.Tensor | None = None,
                    out: torch.Tensor | None = None, stream: torch.cuda.Stream | None = None,
                    fill: bool = False, validate: bool = True) -> torch.Tensor:
    """Per-packet sums of a ragged device batch: packet i is
    ``data[offsets[i] : offsets[i+1]]`` (offsets: n+1 non-decreasing int64/uint64).
    ``validate`` checks the offsets against ``data`` on the device before launching
    (one small synchronisation); pass False only for offsets validated earlier."""
    m = _mode(mode)
    _dev_u8(data, "data")
    if not isinstance(offsets, torch.Tensor) or not offsets.is_cuda or offsets.device != data.device:
        raise TypeError("offsets must be a CUDA tensor on data's device")
    if offsets.dtype not in (torch.int64, torch.uint64) or not offsets.is_contiguous() or offsets.dim() != 1:
        raise TypeError("offsets must be a contiguous 1-D int64/uint64 tensor")
    n = offsets.numel() - 1
    if n < 0:
        raise ValueError("offsets must hold n+1 entries")
    if validate and n > 0:
        o = offsets.view(torch.int64)
        ok = bool(((o[1:] >= o[:-1]).all() & (o[0] >= 0) & (o[-1] <= data.numel())).item())
        if not ok:
            raise ValueError("offsets are not non-decreasing within data")
        cap = MAX_TRANSPORT_LEN if m != RAW else MAX_RAW_LEN
        if bool(((o[1:] - o[:-1]) > cap).any().item()):
            raise ValueError("transport/IPv4/ICMP packets must be <= 65535 bytes" if m != RAW
                             else f"RAW packets must be <= {MAX_RAW_LEN} bytes")
    dev = data.device
    initial_arr = _opt(initial_arr, torch.uint16, n, dev, "initial_arr")
    addrs = _opt(addrs, torch.uint8, 8 * n, dev, "addrs")
    k = outputs(m)
    if out is None:
        out = torch.empty(max(n * k, 1), dtype=torch.uint16, device=dev)[:n * k]
    else:
        _opt(out, torch.uint16, n * k, dev, "out")
    with torch.cuda.device(dev):
        f = lib().yu_csum_fill_ragged if fill else lib().yu_csum_batch_ragged
        rc = f(data.data_ptr(), offsets.data_ptr(), n, m, _ptr(initial_arr), initial & 0xFFFF,
               _ptr(addrs), out.data_ptr() if n else None, _stream(dev, stream))
    check(rc, "yu_csum_fill_ragged" if fill else "yu_csum_batch_ragged")
    return out


def _host_data(data, fill: bool):
    """Pointer and size of a host byte buffer; with ``fill`` the fields are written
    into it, so it must be the caller's own writable contiguous uint8 memory."""
    if isinstance(data, torch.Tensor):
        if data.is_cuda or data.dtype != torch.uint8 or not data.is_contiguous():
            raise TypeError("data must be a contiguous uint8 CPU tensor")
        return data, data.data_ptr(), data.numel()
    if fill:
        if not (isinstance(data, np.ndarray) and data.dtype == np.uint8 and data.flags.c_contiguous
                and data.flags.writeable):
            raise TypeError("fill=True needs a writable C-contiguous uint8 numpy array")
    else:
        data = np.ascontiguousarray(data, dtype=np.uint8)
    return data, data.ctypes.data, data.size


def _fill_name(name: str, fill: bool, device) -> str:
    if not fill:
        return name
    if isinstance(device, (list, tuple)):
        raise ValueError("fill=True takes one device")
    return name.replace("_batch_", "_fill_")


def checksum_host_uniform(data: np.ndarray, stride: int, length: int, n: int, mode="raw", *,
                          initial: int = 0, initial_arr: np.ndarray | None = None,
                          addrs: np.ndarray | None = None, out: np.ndarray | None = None,
                          device: int | list[int] = 0, fill: bool = False) -> np.ndarray:
    """Host-memory batch in, host-memory results out (pinned staging + pipelined
    H2D/kernel/D2H inside the library). ``data`` may be a numpy array or a pinned
    torch CPU tensor (then the copy engine reads it directly). ``device`` may be a
    list of device indices: one shard per GPU, all at once. ``fill=True`` (TX modes)
    also stores each result into the packet's checksum field in ``data``
    (yu_csum_fill_host_uniform)."""
    m = _mode(mode)
    data, dptr, dlen = _host_data(data, fill)
    if n and (n - 1) * stride + length > dlen:
        raise ValueError("data too small for the batch geometry")
    ia = None if initial_arr is None else np.ascontiguousarray(initial_arr, dtype=np.uint16)
    ad = None if addrs is None else np.ascontiguousarray(addrs, dtype=np.uint8)
    if ia is not None and ia.size < n or ad is not None and ad.size < 8 * n:
        raise ValueError("side arrays too small")
    k = outputs(m)
    if out is None:
        out = np.empty(n * k, dtype=np.uint16)
    if isinstance(out, torch.Tensor):
        if out.element_size() != 2 or out.is_cuda or not out.is_contiguous() or out.numel() < n * k:
            raise ValueError("out must be a contiguous 16-bit CPU tensor of >= n results")
        optr = out.data_ptr()
    else:
        if out.dtype.itemsize != 2 or out.size < n * k or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous 16-bit array of >= n results")
        optr = out.ctypes.data
    args = (dptr, stride, length, n, m, None if ia is None else ia.ctypes.data, initial & 0xFFFF,
            None if ad is None else ad.ctypes.data, optr)
    _host_call(_fill_name("yu_csum_batch_host_uniform", fill, device), args, device)
    return out


def _host_call(name: str, args: tuple, device) -> None:
    """``device`` an int: the single-GPU host call. A sequence of ints: the
    ``_multi`` variant, the batch split into one shard per listed device
    (include/yucsum.h)."""
    import ctypes
    if isinstance(device, (list, tuple)):
        devs = (ctypes.c_int * max(1, len(device)))(*[int(d) for d in device])
        rc = getattr(lib(), name + "_multi")(*args, devs, len(device))
        check(rc, name + "_multi")
    else:
        check(getattr(lib(), name)(*args, int(device)), name)


def _host_side(n, initial_arr, addrs, out, k=1):
    ia = None if initial_arr is None else np.ascontiguousarray(initial_arr, dtype=np.uint16)
    ad = None if addrs is None else np.ascontiguousarray(addrs, dtype=np.uint8)
    if ia is not None and ia.size < n or ad is not None and ad.size < 8 * n:
        raise ValueError("side arrays too small")
    if out is None:
        out = np.empty(n * k, dtype=np.uint16)
    elif out.dtype != np.uint16 or out.size < n * k or not out.flags.c_contiguous:
        raise ValueError("out must be a contiguous uint16 array of >= n results")
    return ia, ad, out


def checksum_host_ragged(data, offsets, mode="raw", *, initial: int = 0, initial_arr=None,
                         addrs=None, out: np.ndarray | None = None,
                         device: int | list[int] = 0, fill: bool = False) -> np.ndarray:
    """Ragged host batch (packet i = data[offsets[i]:offsets[i+1]], e.g. a tun read
    burst) through the pinned, pipelined host path (yu_csum_batch_host_ragged).
    ``fill=True``: also the fields, in place (yu_csum_fill_host_ragged)."""
    m = _mode(mode)
    data, dptr, dlen = _host_data(data, fill)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    n = offs.size - 1
    if n < 0:
        raise ValueError("offsets must hold n+1 entries")
    if n and int(offs[-1]) > dlen:
        raise ValueError("offsets run past data")
    ia, ad, out = _host_side(n, initial_arr, addrs, out, outputs(m))
    args = (dptr, offs.ctypes.data, n, m, None if ia is None else ia.ctypes.data, initial & 0xFFFF,
            None if ad is None else ad.ctypes.data, out.ctypes.data)
    _host_call(_fill_name("yu_csum_batch_host_ragged", fill, device), args, device)
    return out


def checksum_host_iov(packets, mode="raw", *, initial: int = 0, initial_arr=None, addrs=None,
                      out: np.ndarray | None = None,
                      device: int | list[int] = 0, fill: bool = False) -> np.ndarray:
    """Scatter-gather host packets: ``packets[i]`` is a list of views (numpy uint8
    arrays / bytes) whose concatenation is packet i, as tundev's readv fills them
    (link/tundev/tundev.go:116-125). Gathered into pinned staging by the library.
    ``fill=True``: the fields are written through the views, which must then be
    writable contiguous uint8 numpy arrays or bytearrays (yu_csum_fill_host_iov)."""
    from ._lib import YuIovec
    m = _mode(mode)
    n = len(packets)
    keep, views = [], []
    first = np.zeros(n + 1, np.uint64)
    for i, pk in enumerate(packets):
        for v in pk:
            if fill:
                a = np.frombuffer(v, np.uint8) if isinstance(v, bytearray) else v
                if not (isinstance(a, np.ndarray) and a.dtype == np.uint8 and a.flags.c_contiguous
                        and a.flags.writeable):
                    raise TypeError("fill=True needs writable contiguous uint8 views")
            else:
                a = np.frombuffer(v, np.uint8) if isinstance(v, (bytes, bytearray)) else \
                    np.ascontiguousarray(v, dtype=np.uint8)
            keep.append(a)
            views.append((a.ctypes.data if a.size else None, a.size))
        first[i + 1] = len(views)
    iov = (YuIovec * max(1, len(views)))(*[YuIovec(b, l) for b, l in views])
    ia, ad, out = _host_side(n, initial_arr, addrs, out, outputs(m))
    args = (ctypes_addr(iov), first.ctypes.data, n, m, None if ia is None else ia.ctypes.data,
            initial & 0xFFFF, None if ad is None else ad.ctypes.data, out.ctypes.data)
    _host_call(_fill_name("yu_csum_batch_host_iov", fill, device), args, device)
    del keep
    return out


def ctypes_addr(obj) -> int:
    import ctypes
    return ctypes.addressof(obj)


def verified(sums: torch.Tensor) -> torch.Tensor:
    """checker semantics: a VERIFY_* sum is valid iff it is 0x0000 or 0xFFFF."""
    s = sums.view(torch.int16)
    return (s == 0) | (s == -1)


def rx_accepted(flags: torch.Tensor) -> torch.Tensor:
    """VERIFY_RX: the packet is well formed, its header checksum verifies and, when
    it carries TCP/UDP/ICMP, so does the transport checksum."""
    f = flags.to(torch.int32)
    ok_ip = (f & (RX_IP_OK | RX_INVALID)) == RX_IP_OK
    ok_l4 = ((f & RX_L4) == 0) | ((f & RX_L4_OK) != 0)
    return ok_ip & ok_l4


def ragged_variant(mode="raw", n: int = 1 << 20, fill: bool = False) -> str:
    """Name of the kernel the ragged path launches for this mode and batch size
    (bursts of up to 4096 packets take a wave per packet); ``fill``: the in-place
    form (yu_csum_fill_ragged)."""
    f = lib().yu_ragged_fill_variant_n if fill else lib().yu_ragged_variant_n
    return f(_mode(mode), n).decode()


def variant(stride: int, length: int, mode="raw", align16: int = 0, n: int = 2) -> str:
    """Name of the kernel the uniform path launches for this geometry (and batch
    size: dense packets above 3 KiB go to k_seg only in large batches)."""
    return lib().yu_uniform_variant_n(stride, length, n, _mode(mode), align16).decode()

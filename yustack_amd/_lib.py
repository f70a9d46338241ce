"""Loader for the in-tree C-ABI library ``yustack_amd/libyucsum.so`` (include/yucsum.h).

There is no fallback: if the library is missing or cannot be loaded, importing
anything that needs it raises, and the batched (GPU) entry points return a negative
status that :func:`check` turns into an exception when no HIP device is usable.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libyucsum.so")

# Exported symbols declared in include/yucsum.h (checked by tests/test_abi.py).
EXPORTS = (
    "yu_checksum", "yu_checksum_combine", "yu_pseudo_header_checksum",
    "yu_csum_batch_uniform", "yu_csum_batch_ragged",
    "yu_csum_fill_uniform", "yu_csum_fill_ragged",
    "yu_csum_batch_host_uniform", "yu_csum_batch_host_ragged", "yu_csum_batch_host_iov",
    "yu_csum_batch_host_uniform_multi", "yu_csum_batch_host_ragged_multi",
    "yu_csum_batch_host_iov_multi",
    "yu_csum_fill_host_uniform", "yu_csum_fill_host_ragged", "yu_csum_fill_host_iov",
    "yu_abi_version", "yu_strerror", "yu_device_count", "yu_uniform_variant", "yu_uniform_variant_n",
    "yu_ragged_variant", "yu_ragged_variant_n", "yu_ragged_fill_variant_n",
    "yu_host_contexts", "yu_host_staging_bytes", "yu_host_staging_trim", "yu_hip_runtime_path",
)

# Host-path staging bounds (include/yucsum.h): per context, between calls.
HOST_SLICE_BYTES, HOST_SLICE_PACKETS = 32 << 20, 1 << 18
HOST_CONTEXT_PINNED_MAX = 3 * (HOST_SLICE_BYTES + 26 * HOST_SLICE_PACKETS + 72)
HOST_CONTEXT_DEVICE_MAX = 3 * (HOST_SLICE_BYTES + 22 * HOST_SLICE_PACKETS + 8)
HOST_BURST_CONTEXT_PINNED_MAX = (4 << 20) + 26 * HOST_SLICE_PACKETS + 72
HOST_BURST_CONTEXT_DEVICE_MAX = (4 << 20) + 22 * HOST_SLICE_PACKETS + 8

YU_OK, YU_EINVAL, YU_ENODEV, YU_ENOMEM, YU_EHIP_BASE = 0, -22, -19, -12, -1000


class YuIovec(ctypes.Structure):
    """struct yu_iovec (include/yucsum.h): one view of a scatter-gather packet."""
    _fields_ = [("base", ctypes.c_void_p), ("len", ctypes.c_uint64)]


class YuError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what} failed: status {status} ({strerror(status)})")


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not built — run `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C yustack_amd/csrc`")
    # One process, two HIP runtimes: PyTorch-ROCm bundles its own libamdhip64 (no
    # SONAME), the library binds /opt/rocm's. Measured on the GPU box
    # (tools/load_order_probe.py): with torch's loaded first both see the device in
    # either order of first use; with this library loaded first, whichever runtime
    # initialises second sees no device. So torch, when installed, is loaded first
    # (a torch that fails to import for any reason is skipped: the library itself
    # does not need it), and the binding is then checked (check_runtime).
    try:
        import torch  # noqa: F401
    except Exception:  # noqa: BLE001 — any broken torch install: load without it
        pass
    L = ctypes.CDLL(LIB_PATH)
    c = ctypes
    L.yu_hip_runtime_path.restype = c.c_char_p
    L.yu_hip_runtime_path.argtypes = []
    check_runtime(L)
    vp, u8, u16, u32, u64, sz, i32 = (c.c_void_p, c.c_uint8, c.c_uint16, c.c_uint32,
                                      c.c_uint64, c.c_size_t, c.c_int)
    L.yu_checksum.restype = u16
    L.yu_checksum.argtypes = [vp, sz, u16]
    L.yu_checksum_combine.restype = u16
    L.yu_checksum_combine.argtypes = [u16, u16]
    L.yu_pseudo_header_checksum.restype = u16
    L.yu_pseudo_header_checksum.argtypes = [u32, vp, sz, vp, sz]
    for name in ("yu_csum_batch_uniform", "yu_csum_fill_uniform"):
        f = getattr(L, name)
        f.restype = i32
        f.argtypes = [vp, u64, u32, u64, i32, vp, u16, vp, vp, vp]
    for name in ("yu_csum_batch_ragged", "yu_csum_fill_ragged"):
        f = getattr(L, name)
        f.restype = i32
        f.argtypes = [vp, vp, u64, i32, vp, u16, vp, vp, vp]
    L.yu_csum_batch_host_uniform.restype = i32
    L.yu_csum_batch_host_uniform.argtypes = [vp, u64, u32, u64, i32, vp, u16, vp, vp, i32]
    L.yu_csum_batch_host_ragged.restype = i32
    L.yu_csum_batch_host_ragged.argtypes = [vp, vp, u64, i32, vp, u16, vp, vp, i32]
    L.yu_csum_batch_host_iov.restype = i32
    L.yu_csum_batch_host_iov.argtypes = [vp, vp, u64, i32, vp, u16, vp, vp, i32]
    L.yu_csum_fill_host_uniform.restype = i32
    L.yu_csum_fill_host_uniform.argtypes = [vp, u64, u32, u64, i32, vp, u16, vp, vp, i32]
    L.yu_csum_fill_host_ragged.restype = i32
    L.yu_csum_fill_host_ragged.argtypes = [vp, vp, u64, i32, vp, u16, vp, vp, i32]
    L.yu_csum_fill_host_iov.restype = i32
    L.yu_csum_fill_host_iov.argtypes = [vp, vp, u64, i32, vp, u16, vp, vp, i32]
    L.yu_csum_batch_host_uniform_multi.restype = i32
    L.yu_csum_batch_host_uniform_multi.argtypes = [vp, u64, u32, u64, i32, vp, u16, vp, vp, vp, i32]
    L.yu_csum_batch_host_ragged_multi.restype = i32
    L.yu_csum_batch_host_ragged_multi.argtypes = [vp, vp, u64, i32, vp, u16, vp, vp, vp, i32]
    L.yu_csum_batch_host_iov_multi.restype = i32
    L.yu_csum_batch_host_iov_multi.argtypes = [vp, vp, u64, i32, vp, u16, vp, vp, vp, i32]
    L.yu_abi_version.restype = i32
    L.yu_abi_version.argtypes = []
    L.yu_strerror.restype = c.c_char_p
    L.yu_strerror.argtypes = [i32]
    L.yu_device_count.restype = i32
    L.yu_device_count.argtypes = []
    L.yu_uniform_variant.restype = c.c_char_p
    L.yu_uniform_variant.argtypes = [u64, u32, i32, u64]
    L.yu_uniform_variant_n.restype = c.c_char_p
    L.yu_uniform_variant_n.argtypes = [u64, u32, u64, i32, u64]
    L.yu_ragged_variant.restype = c.c_char_p
    L.yu_ragged_variant.argtypes = [i32]
    L.yu_ragged_variant_n.restype = c.c_char_p
    L.yu_ragged_variant_n.argtypes = [i32, u64]
    L.yu_ragged_fill_variant_n.restype = c.c_char_p
    L.yu_ragged_fill_variant_n.argtypes = [i32, u64]
    L.yu_host_contexts.restype = i32
    L.yu_host_contexts.argtypes = []
    L.yu_host_staging_bytes.restype = u64
    L.yu_host_staging_bytes.argtypes = [i32, vp]
    L.yu_host_staging_trim.restype = i32
    L.yu_host_staging_trim.argtypes = [i32]
    del u8
    _lib = L
    return L


def torch_hip_runtime() -> str | None:
    """Path of the HIP runtime PyTorch-ROCm bundles (torch/lib/libamdhip64*), when
    torch is imported and that file is mapped into this process; else None (no
    torch, or a torch that uses the system runtime like this library)."""
    import sys
    torch = sys.modules.get("torch")
    if torch is None or not getattr(torch, "__file__", None):
        return None
    tlib = os.path.join(os.path.dirname(os.path.realpath(torch.__file__)), "lib") + os.sep
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.split(maxsplit=5)[-1].strip()
                if path.startswith(tlib) and os.path.basename(path).startswith("libamdhip64"):
                    return path
    except OSError:  # pragma: no cover - /proc is always there on Linux
        return None
    return None


def check_runtime(L) -> None:
    """One HIP runtime per process: when torch's bundled runtime is
    loaded, the library's HIP calls must be bound to it. They are not when the
    library was loaded (e.g. by ctypes) before torch was imported; every HIP call of
    the library would then run on a second runtime, and whichever of the two
    initialises second sees no device (profiles/r05/load_order_r05.log). Raises
    ImportError naming the fix instead of failing later as "no device"."""
    theirs = torch_hip_runtime()
    if theirs is None:
        return
    raw = L.yu_hip_runtime_path()
    ours = raw.decode() if raw else None
    if ours is None or os.path.realpath(ours) != os.path.realpath(theirs):
        raise ImportError(
            f"{LIB_PATH} is bound to the HIP runtime {ours}, but torch uses {theirs}: two HIP "
            "runtimes in one process (the one initialised second sees no device). The library "
            "was loaded before torch; import torch (or yustack_amd) before loading "
            "libyucsum.so by any other means.")


def strerror(status: int) -> str:
    try:
        return lib().yu_strerror(status).decode()
    except Exception:  # pragma: no cover - only when the library itself is unusable
        return "unknown"


def check(status: int, what: str) -> None:
    if status != YU_OK:
        raise YuError(status, what)


def host_staging(device: int = 0) -> tuple[int, int]:
    """(pinned host bytes, device bytes) the host-path staging of `device` holds now
    (yu_host_staging_bytes); both 0 before its first host call."""
    d = ctypes.c_uint64(0)
    pinned = lib().yu_host_staging_bytes(device, ctypes.byref(d))
    return int(pinned), int(d.value)

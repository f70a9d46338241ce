"""Multi-GPU partitioning of a packet batch.

Packets are independent (every result depends on one packet's bytes only), so a
batch shards across the GPUs of a node with no data-path collective: contiguous
packet ranges, one rank per GPU. Uniform batches split evenly by packet count;
ragged batches split on packet boundaries balanced by bytes (a prefix-sum search),
since 64..9000-byte packets make equal counts very unequal in work. The only
communication is control-plane timing (:func:`gather_over_ranks`, one all_gather of
each rank's wall and kernel time) that bench.py uses to report the slowest rank and
the per-GPU rates.
"""
from __future__ import annotations

import numpy as np


def shard_uniform(n: int, world: int, rank: int) -> tuple[int, int]:
    """(first, count) of rank's contiguous share of n packets (even split, the
    first n % world ranks take one extra)."""
    if world < 1 or not 0 <= rank < world or n < 0:
        raise ValueError("bad shard request")
    per, rem = divmod(n, world)
    first = rank * per + min(rank, rem)
    return first, per + (1 if rank < rem else 0)


def shard_ragged(offsets: np.ndarray, world: int, rank: int) -> tuple[int, int]:
    """(first, count) of rank's packets for a ragged batch with n+1 offsets: cut
    points are the packet boundaries closest to equal byte shares."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad shard request")
    off = np.asarray(offsets, dtype=np.int64)
    n = len(off) - 1
    if n <= 0:
        return 0, 0
    total = off[-1] - off[0]
    targets = off[0] + (total * np.arange(world + 1)) // world
    cuts = np.searchsorted(off, targets, side="left")
    cuts[0], cuts[-1] = 0, n
    cuts = np.minimum(np.maximum.accumulate(cuts), n)
    return int(cuts[rank]), int(cuts[rank + 1] - cuts[rank])


def max_over_ranks(value: float, device=None) -> float:
    """Max of a float over all ranks of the default process group (identity when
    torch.distributed is not initialised). Uses the group's backend: RCCL on GPU
    ranks, gloo on CPU ranks."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(values, device=None) -> list[list[float]]:
    """Every rank's list of floats (same length on all ranks), in rank order: one
    all_gather of a small float64 tensor over the default group (RCCL when
    ``device`` is a GPU, gloo for CPU tensors). ``[values]`` when torch.distributed
    is not initialised. bench.py uses it for the per-GPU figures and the slowest
    rank's wall time; it never carries packet data."""
    import torch
    import torch.distributed as dist
    vals = [float(v) for v in values]
    if not (dist.is_available() and dist.is_initialized()):
        return [vals]
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]

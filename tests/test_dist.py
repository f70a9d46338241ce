"""Multi-rank plumbing on CPU (gloo, world_size 2): the shard arithmetic of
yustack_amd.shard and the timing collectives bench.py uses (gather_over_ranks,
max_over_ranks). The shards here run the oracle, so this checks the split, not the
product: the HIP path on shards is tests/test_gpu_dist.py. Packets are independent,
so the shards' results concatenated equal the whole batch's — no data collective."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from yustack_amd.shard import gather_over_ranks, max_over_ranks, shard_ragged, shard_uniform


def test_shard_uniform_covers_exactly():
    for n in (0, 1, 7, 8, 1 << 20, 8 << 20, 1000003):
        for world in (1, 2, 3, 4, 8):
            spans = [shard_uniform(n, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (a, c), (b, _) in zip(spans, spans[1:]):
                assert a + c == b
            assert sum(c for _, c in spans) == n
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1


def test_shard_ragged_byte_balanced():
    rng = np.random.default_rng(4)
    lens = rng.integers(64, 9001, size=100000)
    offs = np.zeros(len(lens) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    for world in (1, 2, 4, 8):
        spans = [shard_ragged(offs, world, r) for r in range(world)]
        assert sum(c for _, c in spans) == len(lens)
        bytes_ = [offs[f + c] - offs[f] for f, c in spans]
        assert max(bytes_) - min(bytes_) <= 2 * 9000  # within one or two packets of even
    assert shard_ragged(np.array([0]), 4, 2) == (0, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from oracle import oracle as O
        rng = np.random.default_rng(11)
        n, L = 4096, 1500
        host = rng.integers(0, 256, size=n * L, dtype=np.uint8)
        host.reshape(n, L)[:, 12] = 0x50
        addrs = rng.integers(0, 256, size=8 * n, dtype=np.uint8)
        first, cnt = shard_uniform(n, world, rank)
        part = O.C().batch(host[first * L:(first + cnt) * L], O.MODE_TCP, stride=L, length=L, n=cnt,
                           addrs=addrs[8 * first: 8 * (first + cnt)])
        parts = [None] * world
        dist.all_gather_object(parts, part.tolist())  # test-only gather of results
        t = max_over_ranks(0.5 + rank)
        per = gather_over_ranks([rank, cnt])
        if rank == 0:
            full = O.C().batch(host, O.MODE_TCP, stride=L, length=L, n=n, addrs=addrs)
            ok = sum(parts, []) == full.tolist() and per == [[0.0, n / 2], [1.0, n / 2]]
            q.put((ok, t, torch.__version__ is not None))
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_shard_and_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        ok, t, _ = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert ok
    assert t == 1.5
    assert all(p.exitcode == 0 for p in procs)


def test_max_over_ranks_without_group():
    assert not dist.is_initialized()
    assert max_over_ranks(3.25) == 3.25


if __name__ == "__main__":
    pytest.main([__file__])

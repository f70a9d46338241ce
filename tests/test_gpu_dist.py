"""Multi-rank product path on one MI355X: ranks share cuda:0 over gloo,
each runs the HIP path (batch.checksum_uniform / checksum_ragged through the C ABI)
on its own shard (yustack_amd.shard), and rank 0 checks that the shards' results,
concatenated, equal the oracle's over the whole batch. Shards are re-based to start
at byte 0 on their rank, as a real split hands them over, so alignments change.
Plus bench.py --gpus 2 self-launching two ranks on the one card."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches():
    """Seeded on every rank alike: a config-3-shaped uniform TCP batch, a
    config-4-shaped ragged RAW batch and a config-6-shaped VERIFY_RX batch (sizes
    cut so the oracle finishes in seconds; each rank's shard still crosses the
    k_small run and 16-packet k_seg cut-overs)."""
    rng = np.random.default_rng(2024)
    n3, L = 200003, 1500
    b3 = rng.integers(0, 256, size=n3 * L, dtype=np.uint8)
    b3.reshape(n3, L)[:, 12] = 0x50
    b3.reshape(n3, L)[:, 16:18] = 0
    a3 = rng.integers(0, 256, size=8 * n3, dtype=np.uint8)
    n4 = 100001
    l4 = rng.integers(64, 9001, size=n4)
    o4 = np.zeros(n4 + 1, np.int64)
    o4[1:] = np.cumsum(l4)
    b4 = rng.integers(0, 256, size=int(o4[-1]), dtype=np.uint8)
    i4 = rng.integers(0, 65536, size=n4, dtype=np.uint16)
    n6 = 150001
    l6 = rng.integers(40, 1501, size=n6)
    o6 = np.zeros(n6 + 1, np.int64)
    o6[1:] = np.cumsum(l6)
    b6 = rng.integers(0, 256, size=int(o6[-1]), dtype=np.uint8)
    s6 = o6[:-1]
    b6[s6], b6[s6 + 2], b6[s6 + 3], b6[s6 + 9] = 0x45, l6 >> 8, l6 & 0xFF, 6
    return (n3, L, b3, a3), (o4, b4, i4), (o6, b6)


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from yustack_amd import batch
    from yustack_amd.shard import gather_over_ranks, shard_ragged, shard_uniform
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        (n3, L, b3, a3), (o4, b4, i4), (o6, b6) = _batches()
        mine = {}
        f, c = shard_uniform(n3, world, rank)
        d = torch.from_numpy(b3[f * L:(f + c) * L].copy()).to(dev)
        a = torch.from_numpy(a3[8 * f:8 * (f + c)].copy()).to(dev)
        mine["tcp"] = batch.checksum_uniform(d, L, L, c, "tcp", addrs=a).cpu().numpy().tolist()
        mine["tcp_kernel"] = batch.variant(L, L, "tcp", d.data_ptr() & 15, n=c)
        for name, (o, b, ia, mode) in (("raw", (o4, b4, i4, "raw")), ("rx", (o6, b6, None, "verify_rx"))):
            f, c = shard_ragged(o, world, rank)
            lo, hi = int(o[f]), int(o[f + c])
            d = torch.from_numpy(b[lo:hi].copy()).to(dev)
            offs = torch.from_numpy(o[f:f + c + 1] - lo).to(dev)
            ini = None if ia is None else torch.from_numpy(ia[f:f + c].copy()).to(dev)
            mine[name] = batch.checksum_ragged(d, offs, mode, initial_arr=ini).cpu().numpy().tolist()
            mine[name + "_kernel"] = batch.ragged_variant(mode, c)
        torch.cuda.synchronize()
        parts = [None] * world
        dist.all_gather_object(parts, mine)  # test-only gather of the results
        per = gather_over_ranks([rank, 2.0 * rank])
        if rank == 0:
            from oracle import oracle as O
            C = O.C()
            ok = {}
            want = C.batch(b3, O.MODE_TCP, stride=L, length=L, n=n3, addrs=a3, threads=8)
            ok["tcp"] = sum((p["tcp"] for p in parts), []) == want.tolist()
            want = C.batch(b4, O.MODE_RAW, offsets=o4.view(np.uint64), initial_arr=i4, threads=8)
            ok["raw"] = sum((p["raw"] for p in parts), []) == want.tolist()
            want = C.batch(b6, O.MODE_VERIFY_RX, offsets=o6.view(np.uint64), threads=8)
            ok["rx"] = sum((p["rx"] for p in parts), []) == want.tolist()
            q.put((ok, [[p[k] for k in ("tcp_kernel", "raw_kernel", "rx_kernel")] for p in parts], per))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shards_on_hip_path_concatenate_to_oracle(dev, world):
    """world 8 is the driver's SCALE shape (config 5: eight shards), here with the
    eight ranks sharing cuda:0."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        ok, kernels, per = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert ok == {"tcp": True, "raw": True, "rx": True}, (ok, kernels)
    assert per == [[r, 2.0 * r] for r in range(world)]
    assert all(p.exitcode == 0 for p in procs)
    # every rank ran the device kernels, not a host path
    assert all(k[0].startswith("k_") for k in kernels)


def test_bench_self_launch_two_ranks_on_one_card(dev):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "YU_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "10",
                        "--warmup", "2", "--no-extra", "--no-e2e", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and len(line["per_gpu"]) == 2
    assert [p["rank"] for p in line["per_gpu"]] == [0, 1]
    assert all(p["GiB_s"] > 0 and p["kernel_avg_us"] > 0 for p in line["per_gpu"])
    assert line["config"]["backend"] == "gloo" and "SHARE" in line["config"]["parallelism"]
    assert line["config"]["kernel"] == "k_small<16,6>"


@pytest.mark.parametrize("config", [9, 10, 12, 13])
def test_bench_fill_configs_check_against_oracle(dev, config):
    """The in-place configs' own line with the CPU baseline on: the workload first
    checks the writer kernel against the read-only one (Workload.check_fill), then the
    cpu_baseline leg reads each stored field back (ragged: at offsets[i] + field, both
    fields of a TX_DATAGRAM) and compares the whole timed batch with the oracle, the
    side records (config 13's addresses) included."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "YU_BENCH_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", str(config), "--steps", "5",
                        "--warmup", "2", "--no-extra", "--no-e2e", "--cpu-budget", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["parity_full_batch_vs_oracle"] is True, line
    assert line["cpu_baseline"]["value"] > 0


def _bench_line(n, timeout):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "YU_BENCH_BACKEND")}
    import time
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "20",
                        "--warmup", "5", "--no-extra", "--no-e2e", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=timeout)
    wall = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), wall


def test_bench_self_launch_eight_ranks_on_one_card(dev):
    """The driver's SCALE shape at N=8 (`bench.py --gpus 8`, no outer launcher),
    rehearsed with the eight ranks sharing the one card over gloo: one line, eight
    per_gpu entries, well inside a driver timeout."""
    line, wall = _bench_line(8, 500)
    print(f"bench --gpus 8 on one card: {wall:.1f} s, value {line['value']} GiB/s")
    assert line["n_gpus"] == 8 and len(line["per_gpu"]) == 8
    assert [p["rank"] for p in line["per_gpu"]] == list(range(8))
    assert all(p["GiB_s"] > 0 and p["kernel_avg_us"] > 0 and p["device"] == 0 for p in line["per_gpu"])
    assert line["config"]["backend"] == "gloo" and "SHARE" in line["config"]["parallelism"]
    assert line["config"]["kernel"] == "k_small<16,6>"
    assert wall < 300


def test_host_multi_child_on_one_card(dev):
    """bench.host_multi_isolated, the form the line takes the host-memory rate over
    several GPUs in (a child process, so a fault there cannot cost the line): two
    shards both on device 0, bit-exact against the device path; a device that does
    not exist comes back as an error entry."""
    import bench
    r = bench.host_multi_isolated(3, [0, 0])
    assert r.get("pinned_2gpu_matches") is True and r["pinned_2gpu_GiB_s"] > 0, r
    r = bench.host_multi_isolated(3, [0, 64])
    assert "pinned_2gpu_error" in r and "pinned_2gpu_matches" not in r, r


def test_launcher_device_count_matches_hip(dev):
    """bench._device_count (KFD topology + render nodes, no HIP) against
    torch.cuda.device_count() in a fresh process, with and without visibility lists:
    HIP and CUDA lists set together (HIP's wins), empty strings (no list at the HIP
    level), an index past the card count, and the ROCr-level list. Every case is
    run and printed before any assertion, so one run records the runtime's whole
    behaviour."""
    import bench
    code = "import torch; print(torch.cuda.device_count())"
    vis = ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
    base = {k: v for k, v in os.environ.items() if k not in vis}
    cases = ({}, {"HIP_VISIBLE_DEVICES": "0"}, {"HIP_VISIBLE_DEVICES": ""},
             {"CUDA_VISIBLE_DEVICES": ""}, {"CUDA_VISIBLE_DEVICES": "0"},
             {"HIP_VISIBLE_DEVICES": "0", "CUDA_VISIBLE_DEVICES": "7"},
             {"HIP_VISIBLE_DEVICES": "7", "CUDA_VISIBLE_DEVICES": "0"},
             {"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "0"},
             {"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "7"},
             {"ROCR_VISIBLE_DEVICES": "0"}, {"ROCR_VISIBLE_DEVICES": ""})
    rows = []
    for extra in cases:
        env = dict(base, **extra)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        rows.append((extra, bench._device_count(env), int(r.stdout.strip().splitlines()[-1])))
    for extra, mine, hip in rows:
        print(f"device count {extra}: launcher {mine}, HIP {hip}")
    assert all(mine == hip for _, mine, hip in rows), rows


def _rccl_rank(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from yustack_amd.shard import gather_over_ranks, max_over_ranks
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        per = gather_over_ranks([1.5, 2.5, 3.0], device=dev)
        mx = max_over_ranks(4.25, device=dev)
        q.put((per, mx, dist.get_backend()))
    finally:
        dist.destroy_process_group()


def test_rccl_timing_collectives_one_rank(dev):
    """The RCCL ("nccl") group bench.py builds when every rank has its own GPU, at
    world size 1 (the box has one card; RCCL refuses two ranks on one device):
    the per-GPU gather and the max over ranks run on device tensors."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), q))
    p.start()
    try:
        per, mx, backend = q.get(timeout=120)
    finally:
        p.join(timeout=60)
    assert per == [[1.5, 2.5, 3.0]] and mx == 4.25 and backend == "nccl"
    assert p.exitcode == 0

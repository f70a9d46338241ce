"""bench.py's --gpus N launch on CPU: argument resolution (pure) and the self-launch
of N rank processes that rendezvous over gloo (``--launch-check``: no GPU work).
The timed path itself is GPU-only (tests/test_gpu_dist.py runs it on one card)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (stdlib-only at import: the launcher touches no GPU)


def test_bench_import_is_stdlib_only():
    assert bench.np is None and bench.torch is None and bench.batch is None


def test_single_process_default():
    p = bench.resolve_launch(1, {}, 1)
    assert p["role"] == "single" and p["world"] == 1 and p["device"] == 0 and p["backend"] == "nccl"


def test_gpus_n_without_launcher_spawns():
    p = bench.resolve_launch(8, {}, 8)
    assert p["role"] == "spawn" and p["world"] == 8 and p["backend"] == "nccl" and not p["shared"]
    p = bench.resolve_launch(2, {}, 1)  # one card: ranks share it over gloo
    assert p["role"] == "spawn" and p["backend"] == "gloo" and p["shared"]


def test_rank_under_torchrun():
    env = {"WORLD_SIZE": "4", "RANK": "3", "LOCAL_RANK": "3"}
    p = bench.resolve_launch(4, env, 8)
    assert (p["role"], p["world"], p["rank"], p["device"], p["backend"]) == ("rank", 4, 3, 3, "nccl")
    p = bench.resolve_launch(4, env, 2)
    assert p["device"] == 1 and p["backend"] == "gloo" and p["shared"]
    p = bench.resolve_launch(1, {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, 1)
    assert p["role"] == "single"


def test_gpus_disagreeing_with_world_size_fails_loudly():
    with pytest.raises(SystemExit, match="disagrees"):
        bench.resolve_launch(8, {"WORLD_SIZE": "2", "RANK": "0"}, 8)
    with pytest.raises(SystemExit):
        bench.resolve_launch(0, {}, 1)
    with pytest.raises(SystemExit, match="YU_BENCH_BACKEND"):
        bench.resolve_launch(2, {"YU_BENCH_BACKEND": "mpi"}, 2)


def test_backend_override():
    assert bench.resolve_launch(2, {"YU_BENCH_BACKEND": "gloo"}, 8)["backend"] == "gloo"


def test_backend_follows_ranks_per_node():
    # 2 nodes x 8 GPUs under torchrun: each node's 8 ranks have a GPU each -> RCCL
    env = {"WORLD_SIZE": "16", "RANK": "11", "LOCAL_RANK": "3", "LOCAL_WORLD_SIZE": "8"}
    p = bench.resolve_launch(16, env, 8)
    assert (p["backend"], p["shared"], p["device"], p["per_node"]) == ("nccl", False, 3, 8)
    # the same on 4-GPU nodes: ranks share cards -> gloo rehearsal
    p = bench.resolve_launch(16, env, 4)
    assert p["backend"] == "gloo" and p["shared"]
    # no LOCAL_WORLD_SIZE from the launcher: the world is the node
    p = bench.resolve_launch(8, {"WORLD_SIZE": "8", "RANK": "0", "LOCAL_RANK": "0"}, 8)
    assert p["per_node"] == 8 and p["backend"] == "nccl"


def _fake_topology(tmp_path, gpus_minor, cpus=1, gfx="90500"):
    """A KFD topology tree: `cpus` CPU nodes, then one GPU node per render minor in
    gpus_minor; a render node file exists (and opens) only for minors >= 0."""
    nodes, dri = tmp_path / "nodes", tmp_path / "dri"
    nodes.mkdir()
    dri.mkdir()
    k = 0
    for _ in range(cpus):
        (nodes / str(k)).mkdir()
        (nodes / str(k) / "properties").write_text("cpu_cores_count 64\ngfx_target_version 0\n")
        k += 1
    for m in gpus_minor:
        (nodes / str(k)).mkdir()
        minor = abs(m)
        (nodes / str(k) / "properties").write_text(
            f"simd_count 1024\ngfx_target_version {gfx}\ndrm_render_minor {minor}\n")
        if m >= 0:
            (dri / f"renderD{minor}").write_bytes(b"")
        k += 1
    return str(nodes), str(dri)


def test_device_count_reads_kfd_topology_without_hip(tmp_path):
    # 3 GPU nodes, of which the process can open two render nodes (the third is not
    # passed into this container); CPU nodes never count
    nodes, dri = _fake_topology(tmp_path, [128, 136, -144], cpus=2)
    assert bench._device_count({}, nodes, dri) == 2
    assert bench._device_count({"HIP_VISIBLE_DEVICES": "1"}, nodes, dri) == 1
    assert bench._device_count({"ROCR_VISIBLE_DEVICES": "0,1", "CUDA_VISIBLE_DEVICES": "0"}, nodes, dri) == 1
    # one HIP-level list: HIP_VISIBLE_DEVICES when set (empty: no device), else
    # CUDA_VISIBLE_DEVICES; an empty ROCR_VISIBLE_DEVICES is no list (as measured on
    # the MI355X box, tests/test_gpu_dist.py::test_launcher_device_count_matches_hip)
    assert bench._device_count({"HIP_VISIBLE_DEVICES": ""}, nodes, dri) == 0
    assert bench._device_count({"HIP_VISIBLE_DEVICES": "", "CUDA_VISIBLE_DEVICES": "1"}, nodes, dri) == 0
    assert bench._device_count({"HIP_VISIBLE_DEVICES": "0,1", "CUDA_VISIBLE_DEVICES": "0"}, nodes, dri) == 2
    assert bench._device_count({"HIP_VISIBLE_DEVICES": "1", "CUDA_VISIBLE_DEVICES": "7"}, nodes, dri) == 1
    assert bench._device_count({"HIP_VISIBLE_DEVICES": "7", "CUDA_VISIBLE_DEVICES": "0"}, nodes, dri) == 0
    assert bench._device_count({"CUDA_VISIBLE_DEVICES": ""}, nodes, dri) == 0
    assert bench._device_count({"ROCR_VISIBLE_DEVICES": ""}, nodes, dri) == 2
    assert bench._device_count({"HIP_VISIBLE_DEVICES": "0,5,1"}, nodes, dri) == 1  # stops at the bad index
    assert bench._device_count({"ROCR_VISIBLE_DEVICES": "GPU-1234abcd"}, nodes, dri) == 1
    assert bench._device_count({}, str(tmp_path / "absent"), dri) == 0
    # the counting loaded nothing (the launcher imports the standard library only)
    assert bench.torch is None


def test_device_count_eight_gpu_node(tmp_path):
    nodes, dri = _fake_topology(tmp_path, [128 + 8 * i for i in range(8)], cpus=2)
    assert bench._device_count({}, nodes, dri) == 8
    assert bench.resolve_launch(8, {}, bench._device_count({}, nodes, dri))["backend"] == "nccl"


def _run(args, env=None, timeout=240):
    e = dict(os.environ, **(env or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "YU_BENCH_BACKEND"):
        if env is None or k not in env:
            e.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_self_launch_starts_n_ranks(n):
    r = _run(["--gpus", str(n), "--launch-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    lc = json.loads(lines[0])["launch_check"]
    assert lc["world"] == n
    assert [x["rank"] for x in lc["ranks"]] == list(range(n))
    assert [x["local"] for x in lc["ranks"]] == list(range(n))
    assert len({x["pid"] for x in lc["ranks"]}) == n
    assert all(x["backend"] == "gloo" and x["shared"] for x in lc["ranks"])  # no GPU in this container


def test_mismatch_exits_nonzero():
    r = _run(["--gpus", "4", "--launch-check"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "disagrees" in r.stderr


def test_failing_rank_fails_the_launch():
    # no GPU here: every rank fails at its device; the launcher must not report success
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-extra", "--no-e2e", "--no-cpu-baseline"])
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    return True


def _spawn(args, env):
    e = dict(os.environ, **env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "YU_BENCH_BACKEND"):
        e.pop(k, None)
    return subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=e,
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def _rank_pids(p, n, timeout=60):
    """The launcher logs each rank's pid as it starts it. Read the raw pipe: a
    buffered readline after select() can leave a second line in the buffer, which
    select() then never reports."""
    import select
    import time
    fd = p.stderr.fileno()
    pids, buf, end = {}, b"", time.monotonic() + timeout
    while len(pids) < n and time.monotonic() < end:
        r, _, _ = select.select([fd], [], [], 1.0)
        if r:
            chunk = os.read(fd, 65536)
            if not chunk:
                break
            buf += chunk
            *lines, buf = buf.split(b"\n")
            for ln in lines:
                ln = ln.decode(errors="replace")
                if ln.startswith("bench: rank ") and " pid " in ln:
                    w = ln.split()
                    pids[int(w[2])] = int(w[4])
    assert len(pids) == n, pids
    return list(pids.values())


def test_signal_to_launcher_stops_its_ranks():
    import signal
    p = _spawn(["--gpus", "2", "--launch-check"], {"YU_BENCH_LAUNCH_SLEEP": "120"})
    pids = _rank_pids(p, 2)
    assert all(_alive(x) for x in pids)
    p.send_signal(signal.SIGTERM)
    rc = p.wait(30)
    assert rc == 128 + signal.SIGTERM, (rc, p.stderr.read()[:3000])
    assert not any(_alive(x) for x in pids)  # stopped and reaped by the launcher


def test_rank_ignoring_sigterm_is_killed_after_grace():
    # rank 1 fails; rank 0 ignores the SIGTERM that follows and must get SIGKILL
    p = _spawn(["--gpus", "2", "--launch-check"],
               {"YU_BENCH_LAUNCH_FAIL_RANK": "1", "YU_BENCH_LAUNCH_DEAF_RANK": "0",
                "YU_BENCH_LAUNCH_SLEEP": "120", "YU_BENCH_STOP_GRACE": "1"})
    pids = _rank_pids(p, 2)
    assert p.wait(60) == 3  # the first failure's status
    assert not any(_alive(x) for x in pids)


def test_host_multi_child_failure_is_reported_not_fatal():
    """The multi-GPU host measurement runs in a child (`--host-multi`): a child that
    cannot run (here: no GPU) or outlives its limit leaves an error entry, and the
    caller — the bench line — carries on."""
    r = bench.host_multi_isolated(3, [0, 1], timeout=300)
    assert list(r) == ["pinned_2gpu_error"] and "child exited" in r["pinned_2gpu_error"], r
    r = bench.host_multi_isolated(3, [0, 1], timeout=0.05)
    assert r == {"pinned_2gpu_error": "child killed after 0 s"}, r

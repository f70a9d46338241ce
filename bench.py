#!/usr/bin/env python3
"""Benchmark: device-resident batched Internet checksum on MI355X (BASELINE.json metric).

A "step" = one launch of the hot path over one batch. Headline workload (N=1) is
BASELINE config 3 — 1M x 1500-byte TCP segments including the pseudo-header, the
configuration the north-star target (>=70 % of HBM peak) is quoted on; with
--gpus N every rank processes its own 1M-segment shard (config 5 = 8 x config 3,
weak scaling, no data-path collective — packets are independent).

Launch: under torch.distributed.run (WORLD_SIZE set) this process is one rank and
--gpus must equal WORLD_SIZE. Without a launcher, --gpus N > 1 makes this process a
launcher that starts N rank processes itself (RCCL when every rank has its own GPU,
gloo when ranks share fewer, stated in config.parallelism). `per_gpu` lists each
rank's GiB/s and kernel time; `value` = all ranks' bytes / the slowest rank's wall.

value      = algorithmic bytes of all ranks / max-over-ranks wall time, in GiB/s
             (payload + per-packet side arrays + uint16 results)
roofline   = the dominant (only) kernel's algorithmic bytes / its average launch
             duration from HIP events on its stream, vs 8.0 TB/s HBM peak
cpu_baseline = the C restatement of checksum.go (oracle/, "port", reference-faithful
             -O2 -fno-tree-vectorize) on host cores over a bounded sample of the
             same batch (rank 0, N=1 only); the same leg checks the GPU results
             of the timed batch bit-for-bit against it.

Run: python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3] [--launch-check]
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# numpy / torch / the package are imported by the rank processes only (_imports):
# the --gpus N launcher must start its N ranks before anything can touch the GPU.
np = torch = batch = None

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
N_PKT = 1 << 20
ROTATE_MIN_BYTES = 2 << 30  # rotate batches so each step streams from HBM, not the 256 MiB MALL


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Workload:
    """One BASELINE config, materialised on the device with R rotating copies."""

    def __init__(self, cfg: int, dev: torch.device, seed: int):
        self.cfg = cfg
        self.dev = dev
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        n = N_PKT
        self.n = n
        self.offsets = None
        self.initial_arr = None
        self.addrs = None
        # 9 / 10: configs 3 / 8 through the in-place field writer (SetChecksum on
        # the device): the field is stored, no uint16 array;
        # 12 / 13: the ragged in-place writers (a tun TX burst, both fields of whole
        # datagrams; small UDP datagrams back to back)
        self.fill = cfg in (9, 10, 12, 13)
        base = {9: 3, 10: 8}.get(cfg, cfg)
        if base == 2:  # 1M x 64-B UDP payloads: A1 over the payload, pseudo-header partial as initial
            self.mode, self.L = batch.RAW, 64
            nbytes = n * self.L
            self.side = 2 * n  # uint16 initial
            self.name = "config2: 1M x 64-B UDP payloads, Checksum(payload, pseudo) per packet"
        elif base == 8:  # config 2 as whole UDP datagrams: 8-B header + 64-B payload, sendUDP field
            self.mode, self.L = batch.UDP, 72
            nbytes = n * self.L
            self.side = 8 * n  # addrs
            self.name = "config2-udp: 1M x (8-B UDP header + 64-B payload), sendUDP field value"
        elif base == 3:  # 1M x 1500-B TCP segments, (src,dst) side array
            self.mode, self.L = batch.TCP, 1500
            nbytes = n * self.L
            self.side = 8 * n  # addrs
            self.name = "config3: 1M x 1500-B TCP segments incl. pseudo-header (sendTCP field value)"
        elif cfg in (4, 6, 7, 11, 12, 13):
            # 4: ragged 64..9000 B back-to-back, RAW with initial (BASELINE config 4)
            # 6: tun RX burst, 1M whole IPv4 datagrams U{40..1500} B, VERIFY_RX (§8f row 1)
            # 7: the same with small datagrams U{40..200} B (ACKs, DNS, VoIP)
            # 11: tun TX burst, 1M outgoing TCP/IPv4 datagrams U{40..1500} B, both
            #     checksum fields (TX_DATAGRAM, two results per datagram)
            # 12: config 11 written in place, the burst tundev writes
            #     (network/ipv4/ipv4.go:94 + transport/tcp/connect.go:583, then
            #     link/tundev/tundev.go:171-196): lengths rounded up to 4 B (the
            #     shape rounds 4-5 measure; the writer itself takes any alignment)
            # 13: 1M sendUDP datagrams U{40..200} B back to back, field in place
            #     (header/udp.go:60-62), 4-aligned like 12
            self.mode = {4: batch.RAW, 11: batch.TX_DATAGRAM, 12: batch.TX_DATAGRAM,
                         13: batch.UDP}.get(cfg, batch.VERIFY_RX)
            rng = np.random.default_rng(cfg)
            hi = {4: 9001, 6: 1501, 7: 201, 11: 1501, 12: 1501, 13: 201}[cfg]
            lo = 64 if cfg == 4 else 40
            self.shape = f"U{{{lo}..{hi - 1}}}" + (" rounded up to 4" if cfg in (12, 13) else "")
            lens = rng.integers(lo, hi, size=n)
            if cfg in (12, 13):
                lens = (lens + 3) & ~3
            offs = np.zeros(n + 1, dtype=np.int64)
            offs[1:] = np.cumsum(lens)
            nbytes = int(offs[-1])
            self.L = 0
            self.offsets = torch.from_numpy(offs).to(dev)
            self.lens = torch.from_numpy(lens).to(dev)
            self.side = 8 * (n + 1) + (2 * n if cfg == 4 else 0) + (8 * n if cfg == 13 else 0)
            self.name = {
                4: "config4: ragged 1M packets U{64..9000} B back-to-back (odd offsets)",
                11: "tun TX: 1M outgoing TCP/IPv4 datagrams U{40..1500} B back-to-back, IPv4 header and "
                    "TCP checksum fields (TX_DATAGRAM, 2 results per datagram)",
                12: "tun TX in place: 1M outgoing TCP/IPv4 datagrams U{40..1500} B (4-aligned) back-to-back, "
                    "both checksum fields stored into each datagram (yu_csum_fill_ragged, TX_DATAGRAM)",
                13: "ragged UDP in place: 1M sendUDP datagrams U{40..200} B (4-aligned) back-to-back, "
                    "field stored into each datagram (yu_csum_fill_ragged, UDP + pseudo-header)",
            }.get(cfg, f"tun RX: 1M received IPv4 datagrams U{{40..{hi - 1}}} B back-to-back, header + TCP "
                       "checksum verification (VERIFY_RX)")
        else:
            raise SystemExit(f"unknown config {cfg}")
        self.payload = nbytes
        self.R = max(1, -(-ROTATE_MIN_BYTES // nbytes))
        self.data = []
        for _ in range(self.R):
            d = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=dev, generator=g)
            if base == 3:  # 20-B header: DataOffset 5, checksum field 0 (Encode)
                v = d.view(n, self.L)
                v[:, 12] = 0x50
                v[:, 16:18] = 0
            if cfg in (6, 7, 11, 12):  # IPv4 header: IHL 5, TotalLength = packet length, protocol TCP
                s0 = self.offsets[:-1]
                d[s0] = 0x45
                d[s0 + 2] = (self.lens >> 8).to(torch.uint8)
                d[s0 + 3] = (self.lens & 0xFF).to(torch.uint8)
                d[s0 + 9] = 6
                if cfg in (11, 12):  # the TCP segment as sendTCP encodes it: DataOffset 5
                    d[s0 + 32] = 0x50
            self.data.append(d)
        if cfg == 2 or cfg == 4:
            self.initial_arr = torch.randint(0, 65536, (n,), dtype=torch.int32, device=dev,
                                             generator=g).to(torch.uint16)
        if self.fill and self.offsets is None:
            self.name += "; fused in-place field writer (yu_csum_fill_uniform, no uint16 array)"
        if base in (3, 8) or cfg == 13:
            self.addrs = torch.randint(0, 256, (8 * n,), dtype=torch.uint8, device=dev, generator=g)
        self.out = torch.empty(n * batch.outputs(self.mode), dtype=torch.uint16, device=dev)
        if self.offsets is not None:  # validate once; the timed launches skip the check
            batch.checksum_ragged(self.data[0], self.offsets, self.mode,
                                  initial_arr=self.initial_arr, addrs=self.addrs, out=self.out)
        if self.fill:
            self.check_fill()
        # algorithmic bytes per launch: payload + side arrays + uint16 out
        self.bytes = self.payload + self.side + 2 * n * batch.outputs(self.mode)

    def step(self, k: int) -> None:
        d = self.data[k % self.R]
        if self.fill:  # the fields go into the packets; no result array
            stream = torch.cuda.current_stream(self.dev).cuda_stream
            ad = None if self.addrs is None else self.addrs.data_ptr()
            if self.offsets is None:
                rc = batch.lib().yu_csum_fill_uniform(d.data_ptr(), self.L, self.L, self.n, self.mode, None, 0,
                                                      ad, None, stream)
            else:
                rc = batch.lib().yu_csum_fill_ragged(d.data_ptr(), self.offsets.data_ptr(), self.n, self.mode,
                                                     None, 0, ad, None, stream)
            batch.check(rc, "yu_csum_fill_uniform" if self.offsets is None else "yu_csum_fill_ragged")
        elif self.offsets is None:
            batch.checksum_uniform(d, self.L, self.L, self.n, self.mode, initial_arr=self.initial_arr,
                                   addrs=self.addrs, out=self.out)
        else:
            batch.checksum_ragged(d, self.offsets, self.mode, initial_arr=self.initial_arr,
                                  out=self.out, validate=False)

    def stored_fields(self, d: torch.Tensor) -> torch.Tensor:
        """The checksum fields the in-place writer stored into batch d (big-endian), as
        uint16 values in result order: the transport field per packet (uniform configs
        9 / 10 and ragged UDP config 13), or [IPv4 field, transport field] per datagram
        (TX_DATAGRAM config 12, IHL read from each header)."""
        if self.offsets is None:
            f = 16 if self.mode == batch.TCP else 6
            fb = d.view(self.n, self.L)[:, f:f + 2].to(torch.int32)
            return (fb[:, 0] << 8) | fb[:, 1]
        s0 = self.offsets[:-1]
        be16 = lambda at: (d[at].to(torch.int32) << 8) | d[at + 1].to(torch.int32)  # noqa: E731
        if self.mode == batch.TX_DATAGRAM:
            hl = (d[s0].to(torch.int64) & 0xF) * 4
            return torch.stack([be16(s0 + 10), be16(s0 + hl + 16)], dim=1).reshape(-1)
        return be16(s0 + 6)

    def check_fill(self) -> None:
        """The timed in-place launches are the writer's kernel (k_seg's TXW / DG forms,
        k_small / k_lane fill), not the read-only one the result-array calls run: run it
        once on a copy of batch 0 and require that the fields it stored, and the results
        it returned, equal the read-only kernel's values (self.out, from the same bytes)."""
        d = self.data[0].clone()
        got = torch.empty_like(self.out)
        if self.offsets is None:
            batch.checksum_uniform(d, self.L, self.L, self.n, self.mode, initial_arr=self.initial_arr,
                                   addrs=self.addrs, out=self.out)
            batch.checksum_uniform(d, self.L, self.L, self.n, self.mode, initial_arr=self.initial_arr,
                                   addrs=self.addrs, out=got, fill=True)
        else:
            batch.checksum_ragged(d, self.offsets, self.mode, initial_arr=self.initial_arr, addrs=self.addrs,
                                  out=got, fill=True, validate=False)
        want = self.out.to(torch.int32)
        if not (torch.equal(got.to(torch.int32), want) and torch.equal(self.stored_fields(d), want)):
            raise SystemExit(f"config {self.cfg}: the in-place writer disagrees with the read-only kernel")
        del d

    def kernel_name(self) -> str:
        if self.offsets is not None:
            return batch.ragged_variant(self.mode, self.n, fill=self.fill)
        return batch.variant(self.L, self.L, self.mode, self.data[0].data_ptr() & 15, n=self.n)


def timed(w: Workload, steps: int, warmup: int, dist: bool):
    for k in range(warmup):
        w.step(k)
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for k in range(steps):
        w.step(warmup + k)
    ev1.record()
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    kern = ev0.elapsed_time(ev1) / 1e3 / steps  # s per launch, HIP events on the kernel's stream
    return wall, kern


SIDE_CONFIGS = (2, 8, 3, 4, 6, 7, 9, 10, 11, 12, 13)  # every workload; all but --config are side lines
SIDE_LAUNCHES = 50  # launches per side-config graph, fixed whatever --steps says
SIDE_SETTLE = 2     # untimed replays first: upload, then ~50 launches of load to leave the clock ramp
SIDE_TIMED = 3      # timed replays; the per-launch figure is their median


def timed_graph(w: Workload, warmup: int):
    """A side config's launches captured in a HIP graph and replayed: a 15-30 us kernel
    is shorter than a Python-side launch, so eager launches would time the host, not
    the kernel. The launch count is fixed (SIDE_LAUNCHES), not tied to --steps: a
    fresh card needs ~17 ms of sustained load to leave its low-clock ramp (DESIGN.md
    §5), and 10 launches of a 15-us kernel never get there. Returns (wall s per
    replay, s per launch), both medians over SIDE_TIMED replays."""
    for k in range(warmup):
        w.step(k)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(SIDE_LAUNCHES):
            w.step(warmup + k)
    for _ in range(SIDE_SETTLE):
        g.replay()
    torch.cuda.synchronize()
    walls, kerns = [], []
    for _ in range(SIDE_TIMED):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        g.replay()
        ev1.record()
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        kerns.append(ev0.elapsed_time(ev1) / 1e3 / SIDE_LAUNCHES)
    del g
    return sorted(walls)[SIDE_TIMED // 2], sorted(kerns)[SIDE_TIMED // 2]


def cpu_baseline(w: Workload, threads: int, budget_s: float):
    """Oracle ("port") on host cores over a bounded sample; also full-batch parity."""
    from oracle import oracle as O  # cpu_baseline leg only (test infrastructure)
    C = O.C()
    host = w.data[0].cpu().numpy()
    ia = None if w.initial_arr is None else w.initial_arr.cpu().numpy()
    ad = None if w.addrs is None else w.addrs.cpu().numpy()
    offs = None if w.offsets is None else w.offsets.cpu().numpy().view(np.uint64)
    # full-size parity of the GPU path on data[0]
    w.step(0)
    torch.cuda.synchronize()
    if w.fill:  # the fields written in place (big-endian), against the oracle's values
        got = w.stored_fields(w.data[0]).cpu().numpy().astype(np.uint16)
    else:
        got = w.out.cpu().numpy()
    if offs is None:
        want = C.batch(host, w.mode, stride=w.L, length=w.L, n=w.n, initial_arr=ia, addrs=ad, threads=threads)
    else:
        want = C.batch(host, w.mode, offsets=offs, initial_arr=ia, addrs=ad, threads=threads)
    parity = bool(np.array_equal(got, want))

    def rate(nthreads, sample_pk):
        sample_pk = min(sample_pk, w.n)
        if offs is None:
            run = lambda: C.batch(host, w.mode, stride=w.L, length=w.L, n=sample_pk, initial_arr=ia,  # noqa: E731
                                  addrs=ad, threads=nthreads)
            b = sample_pk * w.L
        else:
            o = offs[:sample_pk + 1]
            run = lambda: C.batch(host, w.mode, offsets=o, initial_arr=ia, addrs=ad,  # noqa: E731
                                  threads=nthreads)
            b = int(o[-1] - o[0])
        b_alg = b + (w.side + 2 * w.n * batch.outputs(w.mode)) * sample_pk / w.n
        reps, t = 0, 0.0
        t0 = time.perf_counter()
        while t < budget_s / 2 or reps < 2:
            run()
            reps += 1
            t = time.perf_counter() - t0
        return reps * b_alg / t / GIB, sample_pk, reps, t
    r1, s1, n1, t1 = rate(1, 1 << 15)
    rT, sT, nT, tT = rate(threads, w.n)
    wall = t1 + tT
    opt = {}
    flags = open("/proc/cpuinfo").read() if os.path.exists("/proc/cpuinfo") else ""
    if " avx2" in flags:  # the -march=x86-64-v3 build needs AVX2
        C = O.C_opt()  # "optimised CPU" (SURVEY.md §8d): same restatement, vectorised
        o1 = rate(1, 1 << 15)
        oT = rate(threads, w.n)
        wall += o1[3] + oT[3]
        opt = {"optimised_value": round(oT[0], 3), "optimised_value_1core": round(o1[0], 3),
               "optimised_build": "oracle/csum_oracle.c -O3 -march=x86-64-v3 (vectorised)"}
    return parity, {
        "value": round(rT, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
        "sample": (f"oracle/csum_oracle.c (literal checksum.go + sendTCP/sendUDP composition, "
                   f"-O2 -fno-tree-vectorize), static even split over {threads} host threads: "
                   f"{nT} pass(es) over the first {sT} packets of the timed batch in {tT:.1f} s; "
                   f"1 thread: {r1:.3f} GiB/s, {n1} pass(es) over {s1} packets in {t1:.1f} s"),
        "value_1core": round(r1, 3),
        "cpu_work_s": round(t1 + tT * threads, 1),  # CPU-seconds of the port's two timings
        "timing_wall_s": round(wall, 1),  # wall time of every timed CPU leg (port and vectorised)
        "cpu_model": cpu_model(),
        "host_cpus_visible": os.cpu_count(),
        **opt,
    }


def end_to_end(w: Workload, reps: int = 3):
    """Host memory in, host results out (yu_csum_batch_host_uniform: pinned
    staging, H2D / kernel / D2H pipelined over 3 streams), config 3 shape. Reported
    in DESIGN.md, never as `value`. Pageable = numpy buffer (CPU memcpy into the
    library's pinned slots); pinned = page-locked torch tensor (DMA straight from it)."""
    if w.offsets is not None:
        return None
    host = w.data[0].cpu().numpy()
    addrs = None if w.addrs is None else w.addrs.cpu().numpy()
    init = None if w.initial_arr is None else w.initial_arr.cpu().numpy()
    pinned = torch.from_numpy(host).pin_memory()
    out = np.empty(w.n, np.uint16)
    res = {}
    for kind, src in (("pageable", host), ("pinned", pinned)):
        batch.checksum_host_uniform(src, w.L, w.L, w.n, w.mode, initial_arr=init, addrs=addrs, out=out,
                                    device=w.dev.index or 0)  # warm-up: staging allocation
        t0 = time.perf_counter()
        for _ in range(reps):
            batch.checksum_host_uniform(src, w.L, w.L, w.n, w.mode, initial_arr=init, addrs=addrs,
                                        out=out, device=w.dev.index or 0)
        dt = (time.perf_counter() - t0) / reps
        res[f"{kind}_GiB_s"] = round(w.bytes / dt / GIB, 2)
        res[f"{kind}_ms"] = round(dt * 1e3, 2)
    w.step(0)
    torch.cuda.synchronize()
    res["matches_device_path"] = bool(np.array_equal(out, w.out.cpu().numpy()))
    res["bytes"] = w.bytes
    # small tun-style bursts through the same host path: per-call latency (fixed
    # costs of the H2D / kernel / D2H round trip dominate here, not bandwidth)
    for bn in (64, 1024, 8192):
        src = pinned[: bn * w.L]
        o = np.empty(bn, np.uint16)
        ad = None if addrs is None else addrs[: 8 * bn]
        ia = None if init is None else init[:bn]
        for _ in range(10):
            batch.checksum_host_uniform(src, w.L, w.L, bn, w.mode, initial_arr=ia, addrs=ad, out=o)
        k = 300
        t0 = time.perf_counter()
        for _ in range(k):
            batch.checksum_host_uniform(src, w.L, w.L, bn, w.mode, initial_arr=ia, addrs=ad, out=o)
        res[f"burst{bn}_pinned_us_per_call"] = round((time.perf_counter() - t0) / k * 1e6, 1)
    # tun RX bursts: whole IPv4 datagrams U{40..1500} B back to back in pinned
    # memory, verified (VERIFY_RX) through the ragged host path
    rng = np.random.default_rng(5)
    for bn in (64, 1024):
        lens = rng.integers(40, 1501, size=bn)
        offs = np.zeros(bn + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        blob = torch.from_numpy(rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)).pin_memory()
        b, s0 = blob.numpy(), offs[:-1]
        b[s0], b[s0 + 2], b[s0 + 3], b[s0 + 9] = 0x45, lens >> 8, lens & 0xFF, 6
        o = np.empty(bn, np.uint16)
        for _ in range(10):
            batch.checksum_host_ragged(blob, offs, "verify_rx", out=o)
        k = 300
        t0 = time.perf_counter()
        for _ in range(k):
            batch.checksum_host_ragged(blob, offs, "verify_rx", out=o)
        res[f"rx_burst{bn}_pinned_us_per_call"] = round((time.perf_counter() - t0) / k * 1e6, 1)
    # tun TX bursts: whole outgoing TCP/IPv4 datagrams U{40..1500} B (IHL 5, DataOffset
    # 5) in pinned memory, both checksum fields written in place (TX_DATAGRAM fill)
    for bn in (64, 1024):
        lens = (rng.integers(40, 1501, size=bn) + 3) & ~3  # 4-aligned offsets (fill contract)
        offs = np.zeros(bn + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        blob = torch.from_numpy(rng.integers(0, 256, size=int(offs[-1]), dtype=np.uint8)).pin_memory()
        b, s0 = blob.numpy(), offs[:-1]
        b[s0], b[s0 + 2], b[s0 + 3], b[s0 + 9], b[s0 + 32] = 0x45, lens >> 8, lens & 0xFF, 6, 0x50
        for _ in range(10):
            batch.checksum_host_ragged(blob, offs, "tx_datagram", fill=True)
        k = 300
        t0 = time.perf_counter()
        for _ in range(k):
            batch.checksum_host_ragged(blob, offs, "tx_datagram", fill=True)
        res[f"tx_burst{bn}_pinned_us_per_call"] = round((time.perf_counter() - t0) / k * 1e6, 1)
    res["crossover"] = burst_crossover()
    ndev = torch.cuda.device_count()
    if ndev > 1:  # yu_csum_batch_host_uniform_multi: one shard per visible GPU, each on its own PCIe link
        res.update(host_multi_isolated(w.cfg, list(range(ndev))))
    return res


CROSSOVER_BURSTS = (1, 8, 64, 256, 1024, 4096, 16384)


def burst_crossover(L: int = 1500) -> dict:
    """When does batching pay for a caller holding host packets? The reference hands
    up one datagram per tundev dispatch (link/tundev/tundev.go:78-114) and sums it on
    the calling goroutine. Measured here, on one core of this host:
    * the product's own scalar drop-in, yu_checksum (the Go shim's Checksum for
      buffers >= 256 B), over one large buffer: its byte rate, and from it the cost of
      one L-byte packet (a C caller adds ~2 ns per call, a cgo caller ~100 ns);
    * the batched host path, yu_csum_batch_host_ragged (BatchHostRagged in Go), RAW
      mode (Checksum(pkt, initial) per packet) on bursts of L-byte packets packed back
      to back, per call, from pageable memory (a Go heap buffer) and from pinned,
      called straight through the C ABI (ctypes, pointers taken once: ~1 us of call
      overhead, close to a cgo caller's) and checked against the scalar drop-in;
    * the burst size above which one batched call beats that many scalar calls: the
      first measured burst where it does, and k* where the straight line through that
      burst's time and the one before it meets k * s, s being the scalar cost of one
      packet (None when no measured burst is faster).
    Bursts up to 4 MiB take the direct path (one launch reading host memory), larger
    ones the pipelined copies (include/yucsum.h)."""
    L_ = batch.lib()
    big = np.random.default_rng(3).integers(0, 256, size=256 << 20, dtype=np.uint8)
    p = big.ctypes.data
    L_.yu_checksum(p, big.size, 0)  # warm: page faults, caches
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t0 < 0.5:
        L_.yu_checksum(p, big.size, 0)
        reps += 1
    scalar_bps = reps * big.size / (time.perf_counter() - t0)
    s_us = L / scalar_bps * 1e6
    res = {"scalar_yu_checksum_GiB_s_1core": round(scalar_bps / GIB, 2),
           "scalar_us_per_packet": round(s_us, 4), "packet_bytes": L, "bursts": list(CROSSOVER_BURSTS)}
    rng = np.random.default_rng(11)
    nmax = max(CROSSOVER_BURSTS)
    blob_np = rng.integers(0, 256, size=nmax * L, dtype=np.uint8)
    blob_pin = torch.from_numpy(blob_np.copy()).pin_memory()
    init = rng.integers(0, 65536, size=nmax, dtype=np.uint16)
    for kind, blob in (("pageable", blob_np), ("pinned", blob_pin)):
        us = []
        src = blob.ctypes.data if kind == "pageable" else blob.data_ptr()
        for k in CROSSOVER_BURSTS:
            offs = np.arange(k + 1, dtype=np.uint64) * L
            o = np.empty(k, np.uint16)
            # straight through the C ABI with the pointers taken once, as a cgo or C++
            # caller makes the call (the Python wrapper's argument checks add ~4 us)
            args = (src, offs.ctypes.data, k, batch.MODES["raw"], init.ctypes.data, 0, None, o.ctypes.data, 0)
            for _ in range(10):
                rc = L_.yu_csum_batch_host_ragged(*args)
            if rc:
                raise RuntimeError(f"yu_csum_batch_host_ragged: {rc}")
            n = 300
            t0 = time.perf_counter()
            for _ in range(n):
                L_.yu_csum_batch_host_ragged(*args)
            us.append((time.perf_counter() - t0) / n * 1e6)
            if k == 64:  # the batched results equal the scalar drop-in's, packet by packet
                ok = all(int(o[i]) == L_.yu_checksum(src + i * L, L, int(init[i])) for i in range(k))
                res[f"{kind}_matches_scalar"] = ok
        res[f"host_ragged_{kind}_us_per_call"] = [round(u, 2) for u in us]
        cross = None
        for j, (k, u) in enumerate(zip(CROSSOVER_BURSTS, us)):
            if u < k * s_us:
                if j == 0:
                    cross = float(k)
                else:
                    k0, u0 = CROSSOVER_BURSTS[j - 1], us[j - 1]
                    slope = (u - u0) / (k - k0)
                    cross = (u0 - slope * k0) / (s_us - slope)
                res[f"first_burst_batched_wins_{kind}"] = k
                break
        res[f"crossover_packets_{kind}"] = None if cross is None else round(cross, 1)
    res["scalar_us_per_call_at_bursts"] = [round(k * s_us, 2) for k in CROSSOVER_BURSTS]
    return res


def host_multi(w: Workload, devs: list, pinned=None, want=None, reps: int = 3) -> dict:
    """Host memory in and out over several GPUs at once (yu_csum_batch_host_uniform_multi:
    the batch split into one contiguous shard per listed device, each through that
    device's own pinned pipeline and PCIe link). Reported beside the
    device-resident line, never as `value`; never fatal to the bench line."""
    res, nd = {}, len(devs)
    try:
        if pinned is None:
            pinned = w.data[0].cpu().pin_memory()
        addrs = None if w.addrs is None else w.addrs.cpu().numpy()
        init = None if w.initial_arr is None else w.initial_arr.cpu().numpy()
        out2 = np.empty(w.n, np.uint16)
        batch.checksum_host_uniform(pinned, w.L, w.L, w.n, w.mode, initial_arr=init, addrs=addrs,
                                    out=out2, device=devs)
        t0 = time.perf_counter()
        for _ in range(reps):
            batch.checksum_host_uniform(pinned, w.L, w.L, w.n, w.mode, initial_arr=init, addrs=addrs,
                                        out=out2, device=devs)
        dt = (time.perf_counter() - t0) / reps
        res[f"pinned_{nd}gpu_GiB_s"] = round(w.bytes / dt / GIB, 2)
        if want is None:
            w.step(0)
            torch.cuda.synchronize()
            want = w.out.cpu().numpy()
        res[f"pinned_{nd}gpu_matches"] = bool(np.array_equal(out2, want))
    except Exception as e:  # reported, never fatal to the bench line
        res[f"pinned_{nd}gpu_error"] = str(e)[:200]
    return res


# wall seconds for the --host-multi child (torch import, its own workload, 1 + reps passes)
HOST_MULTI_TIMEOUT_S = float(os.environ.get("YU_BENCH_HOST_MULTI_TIMEOUT", "180"))


def host_multi_isolated(config: int, devs: list, timeout: float = None) -> dict:
    """host_multi in a child process (`bench.py --host-multi 0,1,...`), so that the
    line survives whatever the multi-device host path does on a node it has not run
    on before: a crash or a hang there costs the child and is reported as
    pinned_<n>gpu_error, never the bench line. The child builds its own copy of the
    workload (same config and seed as rank 0) and checks its result against the
    device path itself. Started as a child (fork + exec of a fresh interpreter),
    never by replacing this process."""
    nd = len(devs)
    timeout = HOST_MULTI_TIMEOUT_S if timeout is None else timeout
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "ROLE_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--config", str(config),
           "--host-multi", ",".join(str(d) for d in devs)]
    try:
        p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    except OSError as e:
        return {f"pinned_{nd}gpu_error": f"child not started: {e}"[:200]}
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        p.communicate()
        return {f"pinned_{nd}gpu_error": f"child killed after {timeout:.0f} s"}
    for line in reversed(out.strip().splitlines()):
        if line.startswith("{"):
            try:
                return json.loads(line)
            except ValueError:
                break
    tail = (err.strip().splitlines() or [""])[-1]
    return {f"pinned_{nd}gpu_error": f"child exited {p.returncode}: {tail}"[:200]}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def pmc_traffic(cfg: int, kernel: str):
    """HBM bytes per launch of config `cfg` from rocprofv3 PMC passes of this same
    command (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from
    tools/profile.sh output: 2 x FETCH_SIZE + WRITE_SIZE, KiB -> bytes), if the
    record is for the kernel this run launches; else (None, None)."""
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        rec = json.load(open(tf)).get(f"config{cfg}")
        if rec and rec.get("kernel") == kernel:
            return rec["hbm_bytes_per_launch"], rec["source"]
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def _imports():
    global np, torch, batch
    import numpy
    import torch as _torch
    from yustack_amd import batch as _batch
    np, torch, batch = numpy, _torch, _batch


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
DRI_DIR = "/dev/dri"


def _visible_cut(n: int, value) -> int:
    """Devices left of n after a HIP_VISIBLE_DEVICES-style list: entries are taken in
    order up to the first that names no device (an index out of range, or junk),
    as HIP and ROCr apply them; a GPU-<uuid> entry counts as one device. An empty
    value hides every device."""
    if value is None:
        return n
    k = 0
    for tok in value.split(","):
        tok = tok.strip()
        if tok.startswith("GPU-") and len(tok) > 4:
            k += 1
        elif tok.isdigit() and int(tok) < n:
            k += 1
        else:
            break
    return min(n, k)


def _device_count(env=None, nodes: str = KFD_NODES, dri: str = DRI_DIR) -> int:
    """GPUs this process can use, counted without loading HIP, so that the --gpus N
    launcher starts its ranks before anything here has touched a GPU: the KFD topology
    nodes that are GPUs (gfx_target_version != 0) and whose render node this process
    can open — the enumeration the ROCm runtime does — then cut by
    ROCR_VISIBLE_DEVICES (the ROCr layer; an empty value is no list), then by ONE
    HIP-level list: HIP_VISIBLE_DEVICES when it is set, else CUDA_VISIBLE_DEVICES when
    that is; at this level an empty value hides every device. Measured on the MI355X
    box (profiles/r05/device_count_r05a.txt, tests/test_gpu_dist.py): HIP="" -> 0,
    CUDA="" -> 0, HIP=0 with CUDA=7 -> 1, HIP=7 with CUDA=0 -> 0, HIP="" with CUDA=0 ->
    0, ROCR="" -> 1 (of 1). Opening a render node is a plain DRM file open (no KFD
    queue, no HIP). tests/test_bench_launch.py checks the parsing on a fake topology."""
    env = os.environ if env is None else env
    n = 0
    try:
        names = sorted(os.listdir(nodes), key=lambda s: int(s) if s.isdigit() else -1)
    except OSError:
        names = []
    for name in names:
        props = {}
        try:
            with open(os.path.join(nodes, name, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    props[k] = v.strip()
        except OSError:
            continue
        if props.get("gfx_target_version", "0") in ("0", ""):
            continue  # a CPU node
        minor = props.get("drm_render_minor")
        if minor is None:
            continue
        try:
            fd = os.open(os.path.join(dri, f"renderD{int(minor)}"), os.O_RDWR | os.O_CLOEXEC)
        except (OSError, ValueError):
            continue  # not ours (not passed into this container, or no permission)
        os.close(fd)
        n += 1
    n = _visible_cut(n, env.get("ROCR_VISIBLE_DEVICES") or None)
    hip_list = env.get("HIP_VISIBLE_DEVICES")
    if hip_list is None:
        hip_list = env.get("CUDA_VISIBLE_DEVICES")
    return _visible_cut(n, hip_list)


def resolve_launch(gpus: int, env: dict, ndev: int) -> dict:
    """How this process takes part in a --gpus N run (pure; tests/test_bench_launch.py).

    * WORLD_SIZE set (torch.distributed.run started us): we are one rank of it; --gpus
      must equal WORLD_SIZE, or the line would claim GPUs it never used.
    * WORLD_SIZE unset, --gpus 1: the single-rank bench.
    * WORLD_SIZE unset, --gpus N > 1: this process is only a launcher; it starts N rank
      processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set) before anything here
      touches a GPU, and exits with their status.

    Backend: RCCL ("nccl") when every rank of this node has a GPU of its own (ndev >=
    LOCAL_WORLD_SIZE, the node's rank count; WORLD_SIZE when the launcher sets none);
    gloo when the node's ranks share fewer GPUs (a rehearsal on a smaller box: RCCL
    refuses two ranks on one device). YU_BENCH_BACKEND overrides. Rank r runs on
    device LOCAL_RANK % ndev."""
    if gpus < 1:
        raise SystemExit(f"--gpus must be >= 1 (got {gpus})")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        world = int(ws)
        if world != gpus:
            raise SystemExit(f"--gpus {gpus} disagrees with WORLD_SIZE={world} from the launcher: "
                             "pass --gpus equal to --nproc-per-node")
        role = "rank" if world > 1 else "single"
        rank, local = int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", env.get("RANK", "0")))
        per_node = int(env.get("LOCAL_WORLD_SIZE", world))
    else:
        world, rank, local = gpus, 0, 0
        role = "spawn" if gpus > 1 else "single"
        per_node = world
    backend = env.get("YU_BENCH_BACKEND") or ("nccl" if ndev >= per_node else "gloo")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"YU_BENCH_BACKEND must be nccl or gloo (got {backend})")
    shared = ndev < per_node
    return {"role": role, "world": world, "rank": rank, "local": local, "backend": backend,
            "ndev": ndev, "device": local % max(1, ndev), "shared": shared, "per_node": per_node}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# after SIGTERM, a rank that is still alive gets SIGKILL
STOP_GRACE_S = float(os.environ.get("YU_BENCH_STOP_GRACE", "10"))


def spawn_ranks(plan: dict, argv: list) -> int:
    """The --gpus N launcher: N child processes running this script as ranks 0..N-1
    on 127.0.0.1. Nothing in this process has touched a GPU. A rank that fails takes
    the others down (their exact PIDs: SIGTERM, then SIGKILL after STOP_GRACE_S), and
    the exit status is the first failure's. A SIGTERM / SIGINT to the launcher itself
    (a timeout, ^C) stops the ranks the same way before it exits, so no rank is left
    running on a GPU."""
    port = _free_port()
    procs = []
    stop_at = [None]  # when the ranks were told to stop

    def stop_all():
        if stop_at[0] is None:
            stop_at[0] = time.monotonic()
            for q in procs:
                if q.poll() is None:
                    q.terminate()

    # The handler only records the signal and sends SIGTERM to the ranks; the loop
    # below reaps them (SIGKILL after STOP_GRACE_S) and returns 128 + signum. Waiting
    # inside the handler could block on a Popen lock the interrupted loop holds, and
    # printing could re-enter sys.stderr's buffer while the loop is writing a log line
    # (a RuntimeError that used to end the launcher and orphan its ranks), so the
    # handler writes its note with one unbuffered os.write.
    got = [0]

    def on_signal(signum, _frame):
        if not got[0]:
            got[0] = signum
            try:
                os.write(2, f"bench: launcher got signal {signum}; stopping the ranks\n".encode())
            except OSError:
                pass
        stop_all()

    prev = {sig: signal.signal(sig, on_signal) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(plan["world"]):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(plan["world"]),
                       LOCAL_WORLD_SIZE=str(plan["world"]), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       YU_BENCH_BACKEND=plan["backend"])
            procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env))
            log(f"bench: rank {r} pid {procs[-1].pid}")
        rc = 0
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    log(f"bench: rank pid {p.pid} exited with {c}; stopping the other ranks")
                    stop_all()
            if stop_at[0] is not None and time.monotonic() - stop_at[0] > STOP_GRACE_S:
                for q in live:
                    q.kill()
            time.sleep(0.05)
        return 128 + got[0] if got[0] else rc
    finally:
        for sig, h in prev.items():
            signal.signal(sig, h)


def launch_check(plan: dict) -> None:
    """--launch-check: rendezvous and gather each rank's placement, with no GPU work
    (gloo, whatever the plan's backend), then rank 0 prints it. For CPU tests of the
    launcher and for checking a node's launch before the real run."""
    import torch.distributed as dist
    world = plan["world"]
    # test hooks (tests/test_bench_launch.py): a rank that fails, one that ignores
    # SIGTERM, and ranks that are slow to start
    if os.environ.get("YU_BENCH_LAUNCH_FAIL_RANK") == str(plan["rank"]):
        sys.exit(3)
    if os.environ.get("YU_BENCH_LAUNCH_DEAF_RANK") == str(plan["rank"]):
        signal.signal(signal.SIGTERM, signal.SIG_IGN)
    if os.environ.get("YU_BENCH_LAUNCH_SLEEP"):
        time.sleep(float(os.environ["YU_BENCH_LAUNCH_SLEEP"]))
    if world > 1:
        dist.init_process_group("gloo", rank=plan["rank"], world_size=world)
    me = {"rank": plan["rank"], "local": plan["local"], "device": plan["device"], "pid": os.getpid(),
          "backend": plan["backend"], "shared": plan["shared"]}
    ranks = [None] * world
    if world > 1:
        dist.all_gather_object(ranks, me)
        dist.destroy_process_group()
    else:
        ranks = [me]
    if plan["rank"] == 0:
        print(json.dumps({"launch_check": {"world": world, "ndev": plan["ndev"], "ranks": ranks}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=SIDE_CONFIGS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the side-config measurements")
    ap.add_argument("--cpu-budget", type=float, default=6.0, help="wall seconds for the CPU baseline")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory end-to-end measurement")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks, rendezvous, print their placement; no GPU work")
    ap.add_argument("--host-multi", metavar="DEVS", default=None,
                    help="(child of the bench) host memory over the listed GPUs, e.g. 0,1,2,3; "
                         "prints one JSON object")
    args = ap.parse_args()

    if args.host_multi is not None:
        _imports()
        devs = [int(d) for d in args.host_multi.split(",") if d.strip()]
        torch.cuda.set_device(devs[0])
        w = Workload(args.config, torch.device("cuda", devs[0]), seed=1000)
        print(json.dumps(host_multi(w, devs)), flush=True)
        return

    plan = resolve_launch(args.gpus, os.environ, _device_count())
    if plan["role"] == "spawn":
        sys.exit(spawn_ranks(plan, sys.argv[1:]))
    if args.launch_check:
        launch_check(plan)
        return
    rank_main(args, plan)


def rank_main(args, plan: dict) -> None:
    """One rank (or the single process): its own 1M-packet shard of the workload on its
    own device, timed between barriers; rank 0 prints the line."""
    _imports()
    from yustack_amd.shard import gather_over_ranks
    world, rank, backend = plan["world"], plan["rank"], plan["backend"]
    dist = world > 1
    dev = torch.device("cuda", plan["device"])
    torch.cuda.set_device(dev)
    if dist:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group("gloo")

    w = Workload(args.config, dev, seed=1000 + rank)
    wall, kern = timed(w, args.steps, args.warmup, dist)
    # the only collective: each rank's (wall, kernel time, bytes), for the slowest
    # rank's wall time and the per-GPU figures
    per = gather_over_ranks([wall, kern, float(w.bytes), float(plan["device"])],
                            device=dev if dist and backend == "nccl" else None)
    wall_max = max(p[0] for p in per)
    ms_per_step = wall_max / args.steps * 1e3
    value = sum(p[2] for p in per) * args.steps / wall_max / GIB
    achieved = w.bytes / kern / 1e9  # GB/s (decimal, like the peak)

    traffic, traffic_src = pmc_traffic(args.config, w.kernel_name())

    if backend == "nccl" or not dist:
        par = f"shard{world} (independent packets, no collective; one rank per GPU)"
    else:
        par = (f"shard{world} over gloo, {world} ranks on {plan['ndev']} GPU(s)"
               + (" — ranks SHARE a card: a launch rehearsal, not a scaling figure" if plan["shared"] else ""))
    res = {
        "metric": "GiB/s device-resident Internet checksum, batched packets, 1/2/4/8 MI355X",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded torch.randint bytes on device; TCP header DataOffset 5, field 0)",
        "config": {
            "workload": w.name + (f"; config5 shape: {world} x 1M packets, one shard per rank" if dist else ""),
            "packets_per_gpu": w.n,
            "packet_bytes": w.L if w.L else w.shape,
            "mode": {0: "raw", 1: "udp", 2: "tcp", 8: "verify_rx", 9: "tx_datagram"}.get(w.mode, str(w.mode)),
            "algorithmic_bytes_per_step_per_gpu": w.bytes,
            "rotating_batches": w.R,
            "kernel": w.kernel_name(),
            "parallelism": par,
            "backend": "rccl" if dist and backend == "nccl" else (backend if dist else "none"),
        },
        "per_gpu": [{"rank": r, "device": int(p[3]), "GiB_s": round(p[2] * args.steps / p[0] / GIB, 2),
                     "kernel_avg_us": round(p[1] * 1e6, 2),
                     "roofline_frac": round(p[2] / p[1] / 1e9 / HBM_PEAK_GBS, 4)}
                    for r, p in enumerate(per)],
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes": w.bytes,
            "kernel_avg_us": round(kern * 1e6, 2),
        },
    }

    if rank == 0 and world == 1 and not args.no_extra:
        extra = {}
        for c in SIDE_CONFIGS:
            if c == args.config:
                continue
            wc = Workload(c, dev, seed=77 + c)
            wl, kc = timed_graph(wc, args.warmup)
            extra[f"config{c}"] = {
                "GiB_s": round(wc.bytes * SIDE_LAUNCHES / wl / GIB, 2),
                "kernel_avg_us": round(kc * 1e6, 2),
                "roofline_frac": round(wc.bytes / kc / 1e9 / HBM_PEAK_GBS, 4),
                "kernel": wc.kernel_name(),
                "timing": (f"{SIDE_LAUNCHES} launches captured in one HIP graph; {SIDE_SETTLE} untimed "
                           f"replays, median of {SIDE_TIMED} timed replays"),
            }
            tr, _ = pmc_traffic(c, wc.kernel_name())
            if tr:  # bytes the kernel physically moves (PMC): the in-place writers write whole ranges
                extra[f"config{c}"]["traffic_bytes"] = tr
                extra[f"config{c}"]["traffic_frac"] = round(tr / kc / 1e9 / HBM_PEAK_GBS, 4)
            del wc
            torch.cuda.empty_cache()
        res["other_configs"] = extra

    if rank == 0 and world == 1 and not args.no_e2e:
        res["end_to_end_host_memory"] = end_to_end(w)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        parity, cb = cpu_baseline(w, host_threads(), args.cpu_budget)
        res["cpu_baseline"] = cb
        res["parity_full_batch_vs_oracle"] = parity
    else:
        res["cpu_baseline"] = None

    if dist:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if rank == 0 and dist and not args.no_e2e and plan["ndev"] >= world:
        # Host memory over all the job's GPUs at once (rank 0). Taken after the group
        # is torn down: a rank waiting in an RCCL barrier meanwhile would keep a
        # collective kernel spinning on its GPU. The other ranks have left the timed
        # work and hold no kernels; they exit while this runs.
        res["end_to_end_host_memory"] = host_multi_isolated(args.config, list(range(world)))
        res["end_to_end_host_memory"]["measured"] = ("a child of rank 0 after destroy_process_group; "
                                                     "other ranks idle")
    if rank == 0:
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

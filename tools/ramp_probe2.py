"""Config 3 launch ramp after an idle gap (measurement only): does the slow
stretch of a fresh process (launches ~10-40) come back after the GPU idles?"""
import sys, time
sys.path.insert(0, ".")
import torch
import bench

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
w = bench.Workload(3, dev, seed=1000)
torch.cuda.synchronize()


def burst(n, k0):
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for k, (a, b) in enumerate(evs):
        a.record()
        w.step(k0 + k)
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in evs]


def show(tag, ts):
    win = [sum(ts[i:i + 10]) / 10 for i in range(0, len(ts), 10)]
    print(tag, " ".join(f"{x:6.1f}" for x in win))


show("fresh      ", burst(120, 0))
time.sleep(0.5)
show("after 0.5 s", burst(120, 0))
time.sleep(3.0)
show("after 3 s  ", burst(120, 0))
# same buffer only (no rotation): TLB reach vs clocks
ts = []
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(120)]
for a, b in evs:
    a.record()
    w.step(0)
    b.record()
torch.cuda.synchronize()
show("one buffer ", [a.elapsed_time(b) * 1e3 for a, b in evs])

"""Per-launch kernel time of config 3 for the first launches of a fresh process
(measurement only): does the bench's short default warm-up leave a ramp?"""
import sys, time
sys.path.insert(0, ".")
import torch
import bench

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
w = bench.Workload(3, dev, seed=1000)
torch.cuda.synchronize()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
for k, (a, b) in enumerate(evs):
    a.record()
    w.step(k)
    b.record()
torch.cuda.synchronize()
ts = [a.elapsed_time(b) * 1e3 for a, b in evs]
for i in range(0, 200, 10):
    print(f"launch {i:3d}-{i+9:3d}: " + " ".join(f"{t:6.1f}" for t in ts[i:i + 10]))
print("mean 5..25", sum(ts[5:25]) / 20, "mean 100..200", sum(ts[100:]) / 100)

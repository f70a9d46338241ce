"""Host cost of one Python-side batch call (measurement only): wall time of 1000
back-to-back calls on a one-packet batch, the GPU work being negligible."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from yustack_amd import batch

dev = torch.device("cuda:0")
d = torch.zeros(4096, dtype=torch.uint8, device=dev)
o = torch.tensor([0, 1500], dtype=torch.int64, device=dev)
out = torch.empty(2, dtype=torch.uint16, device=dev)
for mode in ("verify_rx", "tx_datagram"):
    for _ in range(100):
        batch.checksum_ragged(d, o, mode, out=out, validate=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(1000):
        batch.checksum_ragged(d, o, mode, out=out, validate=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{mode}: host {1e6 * (t1 - t0) / 1000:.1f} us/call, with drain {1e6 * (t2 - t0) / 1000:.1f} us/call")

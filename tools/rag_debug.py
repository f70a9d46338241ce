"""Debug helper (not product): runs a ragged RAW batch through the C ABI and
prints the packets whose checksum differs from the C oracle, with their
position in the step / phase layout k_rag uses."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from oracle import oracle as O  # noqa: E402
from yustack_amd import batch  # noqa: E402


def run(n, lo, hi, seed=4):
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, size=n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    d = torch.randint(0, 256, (int(offs[-1]),), dtype=torch.uint8, device=dev, generator=g)
    init = rng.integers(0, 65536, size=n, dtype=np.uint16)
    got = batch.checksum_ragged(d, torch.from_numpy(offs.view(np.int64)).to(dev), "raw",
                                initial_arr=torch.from_numpy(init).to(dev)).cpu().numpy()
    want = O.C().batch(d.cpu().numpy(), O.MODE_RAW, offsets=offs, initial_arr=init, threads=16)
    bad = np.nonzero(got != want)[0]
    print(f"n={n} U[{lo},{hi}] total={int(offs[-1])} bad={len(bad)}", flush=True)
    for i in bad[:20]:
        print(f"  p={i} len={lens[i]} off={int(offs[i])} off&3={int(offs[i]) & 3} step_pos={i % 4} "
              f"got={got[i]:#06x} want={want[i]:#06x}", flush=True)
    if len(bad):
        print("  len histogram of bad:", np.histogram(lens[bad], bins=[0, 1536, 4096, 9001])[0])
        print("  first/last bad:", bad[0], bad[-1], "offsets>4GiB:", int((offs[bad] >= (1 << 32)).sum()),
              "offsets>2GiB:", int((offs[bad] >= (1 << 31)).sum()))


if __name__ == "__main__":
    for spec in sys.argv[1:]:
        n, lo, hi = (int(x) for x in spec.split(","))
        run(n, lo, hi)

"""Time the fused DACE/DMCount loss (forward+grad, one launch) for 16 crops at several point counts.

python tools/loss_probe.py   (GPU)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ebc_amd import synthetic as syn  # noqa: E402
from ebc_amd.losses import DACELoss  # noqa: E402

BINS = [(0.0, 0.0), (1.0, 1.0), (2.0, 2.0), (3.0, 3.0), (4.0, float("inf"))]


def run(counts, reps=10, seed=3):
    B = len(counts)
    _, pts, dens = syn.synthetic_crops(B, 224, seed=seed, counts=counts)
    g = torch.Generator().manual_seed(seed)
    pc = torch.randn(B, 5, 28, 28, generator=g).cuda().requires_grad_()
    pd = (torch.rand(B, 1, 28, 28, generator=g) * 2).cuda().requires_grad_()
    td = torch.from_numpy(dens).cuda()
    tp = [torch.from_numpy(p).cuda() for p in pts]
    crit = DACELoss(BINS, 8, weight_count_loss=1.0, count_loss="dmcount", input_size=224)
    for _ in range(3):
        loss, _ = crit(pc, pd, td, tp)
        loss.backward()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        loss, _ = crit(pc, pd, td, tp)
        loss.backward()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    for n in (0, 20, 100, 300, 600, 1000, 2000):
        print(f"16 crops x {n:5d} points: {run([n] * 16) * 1e3:8.1f} us (loss fwd+bwd, host-side packing included)")
    g = np.random.default_rng(0)
    for s in range(3):
        counts = np.clip(np.floor(g.lognormal(np.log(20.0), 1.2, 16)), 0, 2048).astype(int).tolist()
        print(f"bench-like counts max {max(counts):5d} sum {sum(counts):6d}: {run(counts, seed=s) * 1e3:8.1f} us")


if __name__ == "__main__":
    main()

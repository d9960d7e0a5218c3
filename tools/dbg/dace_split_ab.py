"""DACE loss launch timing by kernel trace, per call: `python tools/dbg/dace_split_ab.py run` runs the fused loss on
fixed point-count configurations and on the bench's own 16-crop batches (bench.py make_batch seeds 1000..1024);
`python tools/dbg/dace_split_ab.py parse <results.db>` prints, per configuration, the median span of one call's
dace_loss_kernel launches (the light and heavy kernels may overlap on two streams: first start to last end).
Under rocprofv3 --kernel-trace; EBC_LIB_PATH selects the library build."""
import os
import sqlite3
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import numpy as np  # noqa: E402

BINS = [(0.0, 0.0), (1.0, 1.0), (2.0, 2.0), (3.0, 3.0), (4.0, float("inf"))]
FIXED = [("16x20", [20] * 16), ("16x64", [64] * 16), ("16x100", [100] * 16), ("16x150", [150] * 16),
         ("16x200", [200] * 16), ("16x256", [256] * 16), ("16x300", [300] * 16), ("15x20+1x400", [400] + [20] * 15)]
NBENCH = 25
WARM, REPS = 3, 10


def configs():
    from ebc_amd import synthetic as syn
    out = [(name, counts, None) for name, counts in FIXED]
    for s in range(NBENCH):
        _, pts, dens = syn.synthetic_crops(16, 224, seed=1000 + s)
        out.append((f"bench{s}", [len(p) for p in pts], (pts, dens)))
    return out


def run():
    import torch
    from ebc_amd import synthetic as syn
    from ebc_amd.losses import DACELoss
    crit = DACELoss(BINS, 8, weight_count_loss=1.0, count_loss="dmcount", input_size=224)
    for name, counts, data in configs():
        B = len(counts)
        if data is None:
            _, pts, dens = syn.synthetic_crops(B, 224, seed=3, counts=counts)
        else:
            pts, dens = data
        g = torch.Generator().manual_seed(3)
        pc = torch.randn(B, 5, 28, 28, generator=g).cuda().requires_grad_()
        pd = (torch.rand(B, 1, 28, 28, generator=g) * 2).cuda().requires_grad_()
        td = torch.from_numpy(dens).cuda()
        tp = [torch.from_numpy(p).cuda() for p in pts]
        for _ in range(WARM + REPS):
            loss, _ = crit(pc, pd, td, tp)
        torch.cuda.synchronize()


def parse(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, start, end from kernels where name like '%dace_%' order by start").fetchall()
    spans, cur = [], []
    for name, s, e in rows:
        if "dace_finalize_kernel" in name:
            spans.append((max(x[1] for x in cur) - min(x[0] for x in cur)) / 1e3 if cur else 0.0)
            cur = []
        else:
            cur.append((s, e))
    cfg = configs()
    per = WARM + REPS
    assert len(spans) == per * len(cfg), (len(spans), per * len(cfg))
    tot = []
    for k, (name, counts, _) in enumerate(cfg):
        x = np.array(spans[k * per + WARM:(k + 1) * per])
        if name.startswith("bench"):
            tot.append(np.median(x))
        print(f"{name:12s} max n {max(counts):5d}: median {np.median(x):8.1f} us  min {x.min():8.1f}")
    print(f"bench batches: mean of medians {np.mean(tot):8.1f} us")


if __name__ == "__main__":
    run() if sys.argv[1] == "run" else parse(sys.argv[2])

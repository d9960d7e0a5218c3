"""Loss-kernel A/B timing: `python tools/loss_ab.py run` launches the fused DACE loss for a fixed list of
point-count configurations (WARM + REPS launches each) under rocprofv3 --kernel-trace; `python
tools/loss_ab.py parse <results.db>` prints the median dace_loss_kernel duration per configuration."""
import os
import sqlite3
import sys

import numpy as np

CONFIGS = [("16x0", [0] * 16), ("16x20", [20] * 16), ("16x100", [100] * 16), ("16x150", [150] * 16), ("16x200", [200] * 16), ("16x300", [300] * 16),
           ("16x600", [600] * 16), ("16x1000", [1000] * 16)]
g = np.random.default_rng(0)
for s in range(3):
    CONFIGS.append((f"bench{s}", np.clip(np.floor(g.lognormal(np.log(20.0), 1.2, 16)), 0, 2048).astype(int).tolist()))
WARM, REPS = 3, 20


def run():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
    from loss_probe import run as probe
    for name, counts in CONFIGS:
        probe(counts, reps=REPS)        # 3 warm-up launches inside + REPS timed


def parse(db):
    con = sqlite3.connect(db)
    d = [r[0] for r in con.execute("select duration from kernels where name like '%dace_loss_kernel%' order by start")]
    per = WARM + REPS
    assert len(d) == per * len(CONFIGS), (len(d), per * len(CONFIGS))
    for k, (name, counts) in enumerate(CONFIGS):
        x = np.array(d[k * per + WARM:(k + 1) * per]) / 1e3
        print(f"{name:10s} max n {max(counts):5d}: median {np.median(x):8.1f} us  min {x.min():8.1f}")


if __name__ == "__main__":
    run() if sys.argv[1] == "run" else parse(sys.argv[2])

"""Loss-kernel A/B across library builds in ONE process per build, interleaved by running this script once per
build per round (tools/dbg/loss_lib_ab.sh): fused DACE loss fwd+grad per 16-crop configuration, CUDA-event timed."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from loss_probe import run as probe

CONFIGS = [("16x20", [20] * 16), ("16x150", [150] * 16), ("16x300", [300] * 16)]
g = np.random.default_rng(0)
for s in range(4):
    CONFIGS.append((f"bench{s}", np.clip(np.floor(g.lognormal(np.log(20.0), 1.2, 16)), 0, 2048).astype(int).tolist()))
lib = os.path.basename(os.path.dirname(os.environ.get("EBC_LIB_PATH", "tree/x")))
for name, counts in CONFIGS:
    ms = probe(counts, reps=20)
    print(f"{lib:10s} {name:8s} max n {max(counts):5d}: {ms * 1e3:8.1f} us (loss fwd+bwd per call)")

"""Per-phase shader clocks of the fused DACE loss (lab build with -DEBC_DACE_PROF, EBC_LIB_PATH=.../libebc_hip.so):
prints, per crop of the last launch, the crop body's phase spans and the Sinkhorn per-iteration phase costs (core-clock
ticks of s_memtime, thread 0 of the crop's workgroup).  python tools/dbg/dace_prof.py   (GPU)"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from loss_probe import run as probe  # noqa: E402
from ebc_amd import _lib  # noqa: E402

CONFIGS = [("16x20", [20] * 16), ("16x150", [150] * 16), ("16x300", [300] * 16)]
g = np.random.default_rng(0)
for s in range(4):
    CONFIGS.append((f"bench{s}", np.clip(np.floor(g.lognormal(np.log(20.0), 1.2, 16)), 0, 2048).astype(int).tolist()))

lib = _lib.load()
rd = lib.ebc_dace_prof_read
rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
for name, counts in CONFIGS:
    ms = probe(counts, reps=10)
    buf = np.zeros((64, 64), dtype=np.uint64)
    assert rd(buf.ctypes.data, buf.nbytes) == 0
    B = len(counts)
    p = buf[:B].astype(np.int64)
    tot = p[:, 7] - p[:, 0]
    print(f"{name}: {ms * 1e3:.1f} us per call; counts {counts}")
    print("  crop     n LPB  it |   total   load     ce     dm  setup   loop   post   grad | A/it  B/it  err/it")
    for b in np.argsort(-tot)[:6]:
        r = p[b]
        it = max(int(r[11]) - 1, 1)
        sp = lambda a, c: int(r[c] - r[a]) if r[c] and r[a] else -1  # noqa: E731
        print(f"  {b:4d} {int(r[12]):5d} {int(r[13]):3d} {it:3d} | {tot[b]:7d} {sp(0, 1):6d} {sp(1, 2):6d} {sp(2, 3):6d} "
              f"{sp(3, 4):6d} {sp(4, 5):6d} {sp(5, 6):6d} {sp(6, 7):6d} | {r[8] // it:5d} {r[9] // it:5d} {r[10] // it:5d}")
        print(f"        setup: windows {sp(3, 48)} prefix {sp(48, 49)} scatter {sp(49, 50)} init {sp(50, 4)};"
              f" per-wave work A/it {[int(x) // it for x in r[16:32]]}")
        print(f"        per-wave work B/it {[int(x) // it for x in r[32:48]]}")

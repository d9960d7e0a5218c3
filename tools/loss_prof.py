"""One loss launch per point count with EBC_DACE_PROF=1 (per-phase shader cycles on stderr)."""
import os
import sys

os.environ["EBC_DACE_PROF"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
from loss_probe import run  # noqa: E402

NS = tuple(int(x) for x in sys.argv[1:]) or (20, 300, 1000, 2000)
for n in NS:
    print(f"--- n={n}", file=sys.stderr, flush=True)
    run([n] * 2, reps=1)

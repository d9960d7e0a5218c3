"""Host-side enqueue time of the bench step vs its device time: is the step launch-bound?

Runs bench.setup's step closure; times each step's Python/launch work with perf_counter and no sync, then
the same K steps' wall time between synchronizes.  python tools/host_time.py [--model clip_vit_b_16] [--steps K]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="clip_vit_b_16")
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    args = bench.parse(["--model", a.model, "--steps", str(a.steps), "--warmup", "5", "--no-cpu-baseline", "--no-probe"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    step = bench.setup(args, 0, 1, 0, dev)
    for i in range(5):
        step(i)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        h0 = time.perf_counter()
        step(5 + i)
        host.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    host.sort()
    print(f"{a.model}: wall {wall / a.steps * 1e3:.3f} ms/step, host enqueue median {host[len(host) // 2] * 1e3:.3f} "
          f"ms/step (min {host[0] * 1e3:.3f}, max {host[-1] * 1e3:.3f})")


if __name__ == "__main__":
    main()

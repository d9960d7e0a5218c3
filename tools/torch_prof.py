"""torch.profiler attribution of one bench.py train step: which aten ops / C-ABI calls launch what.

usage: python tools/torch_prof.py [--steps 3] [--top 40]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda:0")
    step = bench.setup(args, 0, 1, 0, dev)
    for i in range(4):
        step(i)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        for i in range(a.steps):
            step(10 + i)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=a.top,
                                                             max_name_column_width=60, max_shapes_column_width=70))
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25, max_name_column_width=60))
    # every copy / fill / cast with its shapes (where the glue time goes)
    rows = [e for e in prof.key_averages(group_by_input_shape=True)
            if any(k in e.key for k in ("copy", "fill", "zero", "_to_copy", "clone", "cat", "stack", "flip", "Memcpy", "Memset"))]
    rows.sort(key=lambda e: -e.device_time_total)
    print("\n== copy/fill ops by call stack")
    for e in sorted(prof.key_averages(group_by_stack_n=6), key=lambda e: -e.device_time_total):
        if not any(k in e.key for k in ("copy_", "fill_", "_to_copy", "clone", "cat")) or e.device_time_total <= 0:
            continue
        print(f"{e.device_time_total:10.1f} us  n={e.count:4d}  {e.key}")
        for fr in (e.stack or [])[:6]:
            print("        ", fr)
    print("\n== glue ops (per profiled window of %d steps)" % a.steps)
    for e in rows[:40]:
        print(f"{e.device_time_total:10.1f} us  n={e.count:4d}  {e.key[:40]:40s} {str(e.input_shapes)[:150]}")


if __name__ == "__main__":
    main()

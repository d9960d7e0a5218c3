"""Host enqueue time of the bench step (lab): how long the Python / ctypes side takes to issue one train step, against
the GPU's own time per step (HIP events), to see whether the host keeps the GPU's queue fed.
    python tools/lab/host_time.py [--steps 30] [--crops-per-gpu 16]"""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import bench  # noqa: E402


def main():
    args = bench.parse(sys.argv[1:])
    device = torch.device("cuda:0")
    torch.cuda.set_device(0)
    step = bench.setup(args, 0, 1, 0, device)
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    host = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i].record(st)
        a = time.perf_counter()
        step(args.warmup + i)
        host.append((time.perf_counter() - a) * 1e3)
    ev[-1].record(st)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    gpu = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    host.sort()
    gpu_s = sorted(gpu)
    print(f"host enqueue ms/step: median {host[len(host) // 2]:.3f}  min {host[0]:.3f}  max {host[-1]:.3f}")
    print(f"gpu ms/step (events): median {gpu_s[len(gpu_s) // 2]:.3f}  mean {sum(gpu) / len(gpu):.3f}")
    print(f"all steps enqueued after {t_enq * 1e3:.1f} ms, drained after {t_all * 1e3:.1f} ms ({args.steps} steps)")
    print("per-step gpu ms in order:", " ".join(f"{g:.2f}" for g in gpu))


if __name__ == "__main__":
    main()

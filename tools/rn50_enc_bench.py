"""Time the clip_resnet50 encoder (ModifiedResNet, trainable, PyTorch-ROCm / MIOpen) forward + backward at the
config-2 shape (8 crops of 448, bf16 autocast) in several memory-format / MIOpen-search variants.

    python tools/rn50_enc_bench.py [--iters 10]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

from ebc_amd.resnet import ModifiedResNet  # noqa: E402


def run(fmt, bench, iters, B=8, size=448):
    torch.backends.cudnn.benchmark = bench
    torch.manual_seed(0)
    enc = ModifiedResNet(reduction=8).cuda().train()
    x = torch.randn(B, 3, size, size, device="cuda")
    if fmt == "cl":
        enc = enc.to(memory_format=torch.channels_last)
        x = x.contiguous(memory_format=torch.channels_last)

    def step():
        enc.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = enc(x)
        y.float().sum().backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / iters * 1e3
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for _ in range(2):
            enc(x)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            enc(x)
        torch.cuda.synchronize()
    fms = (time.perf_counter() - t0) / iters * 1e3
    print(f"format={fmt} benchmark={bench}: fwd+bwd {ms:.2f} ms  fwd {fms:.2f} ms", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="cl:0,nchw:0,cl:1,nchw:1")
    a = ap.parse_args()
    for v in a.variants.split(","):
        fmt, b = v.split(":")
        run(fmt, b == "1", a.iters)


if __name__ == "__main__":
    main()

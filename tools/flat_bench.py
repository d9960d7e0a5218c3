"""Isolated HIP-event timing of the clip_resnet50 flat BatchNorm kernels at the encoder's layer shapes
(8 crops of 448, bf16): achieved HBM rate of each (bytes = one read of every operand + one write)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

from ebc_amd import _lib  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    L = _lib.lib()
    dt, tdt = _lib.EBC_BF16, torch.bfloat16
    st = _lib.stream()
    for P, C in ((8 * 112 * 112, 256), (8 * 56 * 56, 512), (8 * 28 * 28, 1024), (8 * 28 * 28, 2048)):
        z = torch.randn(P, C, device="cuda").to(tdt)
        x = torch.randn(P, C, device="cuda").to(tdt)
        y = torch.empty_like(z)
        sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
        t1 = timeit(lambda: L.ebc_bn_add_relu_flat(dt, _lib.ptr(z), _lib.ptr(sc), _lib.ptr(sh), _lib.ptr(x), None, None,
                                                   _lib.ptr(y), P, C, st))
        t2 = timeit(lambda: L.ebc_bn_add_relu_flat(dt, _lib.ptr(z), _lib.ptr(sc), _lib.ptr(sh), _lib.ptr(x), _lib.ptr(sc),
                                                   _lib.ptr(sh), _lib.ptr(y), P, C, st))
        t3 = timeit(lambda: L.ebc_bn_relu(dt, _lib.ptr(z), _lib.ptr(sc), _lib.ptr(sh), _lib.ptr(y), P, C, st))
        t4 = timeit(lambda: y.copy_(z))
        n = P * C * 2
        print(f"P={P:6d} C={C:4d}: add_relu {t1*1e6:6.1f} us {3*n/t1/1e12:4.2f} TB/s | +ds-bn {t2*1e6:6.1f} us "
              f"{3*n/t2/1e12:4.2f} TB/s | bn_relu {t3*1e6:6.1f} us {2*n/t3/1e12:4.2f} TB/s | torch copy {t4*1e6:6.1f} us "
              f"{2*n/t4/1e12:4.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()

"""Decoder conv GEMMs alone (fwd+stats, dgrad, wgrad) at the bench shape, HIP-event timed.
EBC_CONV_CFG=<cfg> forces the tile config (gemm.hip)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

from ebc_amd import _lib  # noqa: E402


def timeit(fn, reps=20):
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
    B, H, C = int(os.environ.get("CB", 16)), int(os.environ.get("CH", 28)), int(os.environ.get("CC", 768))
    W = H
    dt = _lib.EBC_BF16 if os.environ.get("CDT") == "bf16" else _lib.EBC_F16
    tdt = torch.bfloat16 if dt == _lib.EBC_BF16 else torch.float16
    geo = (ctypes.c_long * 6)()
    _lib.check(L.ebc_dec_geometry(dt, B, H, W, C, geo), "geo")
    Q, Qs = geo[4], geo[5]
    x = (torch.randn(Q, C, device="cuda") * 0.5).to(tdt)
    wk = (torch.randn(C, 3, 3, C, device="cuda") / 80).to(tdt)
    out = torch.empty(B * H * W, C, device="cuda", dtype=tdt)
    colsum = torch.empty(2, C, device="cuda", dtype=torch.float64)
    ws = torch.zeros(L.ebc_dec_workspace_bytes(dt, B, H, W, C, C), device="cuda", dtype=torch.uint8)
    dzT = (torch.randn(C, Qs, device="cuda") * 0.1).to(tdt)
    xT3 = (torch.randn(3, C, Qs, device="cuda") * 0.5).to(tdt)
    dw = torch.empty(C, 3, 3, C, device="cuda")
    st = _lib.stream()
    f = 2.0 * B * H * W * C * C * 9
    t1 = timeit(lambda: L.ebc_conv3x3_fwd(dt, _lib.ptr(x), _lib.ptr(wk), _lib.ptr(out), _lib.ptr(colsum), None, None, _lib.ptr(ws),
                                          ws.numel(), B, H, W, C, C, st))
    t2 = timeit(lambda: L.ebc_conv3x3_fwd(dt, _lib.ptr(x), _lib.ptr(wk), _lib.ptr(out), None, None, None, _lib.ptr(ws),
                                          ws.numel(), B, H, W, C, C, st))
    t3 = timeit(lambda: L.ebc_conv3x3_wgrad(dt, _lib.ptr(dzT), _lib.ptr(xT3), _lib.ptr(dw), _lib.ptr(ws), ws.numel(),
                                            B, H, W, C, C, st))
    cfg = os.environ.get("EBC_CONV_CFG", "auto") + " tail=" + os.environ.get("EBC_CONV_TAIL", "1")
    print(f"B={B} H={H} C={C} cfg {cfg:>4}: fwd+stats {t1*1e6:7.1f} us {f/t1/1e12:6.0f} TF/s | fwd {t2*1e6:7.1f} us {f/t2/1e12:6.0f} TF/s"
          f" | wgrad {t3*1e6:7.1f} us {f/t3/1e12:6.0f} TF/s (algorithmic)")


if __name__ == "__main__":
    main()

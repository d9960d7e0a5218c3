"""Run ONE hot-path kernel class repeatedly, for rocprofv3 PMC passes and isolated A/B timing.

usage: python tools/kbench.py gemm M N K EPI [--reps R] [--dtype f16|bf16]   (EPI 0 store 1 gelu 2 resid 3 gelu')
       python tools/kbench.py multi gemm:M,N,K,EPI attn:B ... [--rounds R]   (several classes, interleaved rounds)
       python tools/kbench.py attn B [--reps R]                              (fwd + bwd at L = 229, 12 heads)
       python tools/kbench.py conv B [--reps R]                              (decoder 3x3 conv fwd + BN stats, 768 ch)
       python tools/kbench.py head B [--reps R]                              (similarity head fwd + bwd, f32 Z)
Prints the HIP-event average per launch.  Operands are random (DVFS: zero-filled data reads high).
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

from ebc_amd import _lib  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what")
    ap.add_argument("args", nargs="*")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--dtype", default="f16")
    a = ap.parse_args()
    if a.what == "multi":
        specs = [(x.split(":")[0], [int(v) for v in x.split(":")[1].split(",")]) for x in a.args]
    else:
        specs = [(a.what, [int(v) for v in a.args])]
    for r in range(a.rounds):
        for what, args in specs:
            run(what, args, a)


def run(what, args, a):
    L = _lib.lib()
    dt = {"f16": torch.float16, "bf16": torch.bfloat16}[a.dtype]
    code = _lib.dtype_code(dt)
    st = _lib.stream()
    if what == "gemm":
        M, N, K, epi = args
        A = torch.randn(M, K, device="cuda").to(dt)
        B = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        bias = torch.randn(N, device="cuda")
        aux = torch.randn(M, N, device="cuda").to(dt)
        C = torch.empty(M, N, device="cuda", dtype=torch.float32 if epi == 2 else dt)
        R = torch.randn(M, N, device="cuda")
        tile = (ctypes.c_int * 3)()
        cfg = L.ebc_gemm_tile_config(code, M, N, K, tile)
        wsb = L.ebc_gemm_workspace_bytes(code, M, N, K)
        ws = torch.zeros(max(wsb, 1), device="cuda", dtype=torch.uint8)
        us = timeit(lambda: _lib.check(L.ebc_gemm_ws(code, epi, 0, _lib.ptr(A), _lib.ptr(B), _lib.ptr(C), _lib.ptr(bias),
                                                     _lib.ptr(R), _lib.ptr(aux), M, N, K, _lib.ptr(ws) if wsb else None,
                                                     wsb, st), "gemm"), a.reps)
        f = 2.0 * M * N * K
        print(f"gemm M={M} N={N} K={K} epi={epi} cfg={cfg} tile={tuple(tile)}: {us:.2f} us  {f / us / 1e6:.1f} TF/s")
    elif what == "attn":
        (B,) = args
        Lq, H = 229, 12
        qkv = (torch.randn(B * Lq, 3 * H * 64, device="cuda") * 0.5).to(dt)
        out = torch.empty(B * Lq, H * 64, device="cuda", dtype=dt)
        lse = torch.empty(B, H, Lq, device="cuda")
        dout = (torch.randn(B * Lq, H * 64, device="cuda") * 0.1).to(dt)
        delta = torch.empty(B, H, Lq, device="cuda")
        dqkv = torch.empty_like(qkv)
        tf = timeit(lambda: L.ebc_attention_fwd(code, _lib.ptr(qkv), _lib.ptr(out), _lib.ptr(lse), B, Lq, H, st), a.reps)
        tb = timeit(lambda: L.ebc_attention_bwd(code, _lib.ptr(qkv), _lib.ptr(dout), _lib.ptr(out), _lib.ptr(lse),
                                                _lib.ptr(delta), _lib.ptr(dqkv), B, Lq, H, st), a.reps)
        f = 4.0 * B * H * Lq * Lq * 64
        print(f"attn B={B}: fwd {tf:.2f} us ({f / tf / 1e6:.0f} TF/s)  bwd {tb:.2f} us ({2 * f / tb / 1e6:.0f} TF/s)")
    elif what == "head":
        (B,) = args                                  # crops of 224 at reduction 8: 784 pixels each, embed 512, 5 bins
        HW, CH, NB = 784, 512, 5
        P = B * HW
        f32, f16 = _lib.dtype_code(torch.float32), _lib.dtype_code(torch.float16)
        Z = torch.randn(P, CH, device="cuda")
        text = torch.randn(NB, CH, device="cuda")
        ls = torch.full((1,), 4.6, device="cuda")
        anchors = torch.tensor([0.0, 1.0, 2.0, 3.0, 4.2], device="cuda")
        logits = torch.empty(B, NB, HW, device="cuda")
        expo = torch.empty(B, 1, HW, device="cuda")
        dl, de = torch.randn_like(logits), torch.randn_like(expo)
        dZ = torch.empty(P, CH, device="cuda", dtype=torch.float16)
        dbias, dscale = torch.zeros(CH, device="cuda"), torch.zeros(1, device="cuda")
        p = _lib.ptr
        tf = timeit(lambda: L.ebc_head_fwd(f32, p(Z), p(text), p(ls), p(anchors), p(logits), p(expo), P, HW, NB, CH, st), a.reps)
        ws = torch.empty(L.ebc_head_bwd_workspace_bytes(P, CH), device="cuda", dtype=torch.uint8)
        tb = timeit(lambda: L.ebc_head_bwd(f32, f16, p(Z), p(text), p(ls), p(anchors), p(dl), p(de), None, p(dZ), p(dbias),
                                           p(dscale), P, HW, NB, CH, p(ws), ws.numel(), st), a.reps)
        print(f"head B={B}: fwd {tf:.2f} us ({P * CH * 4 / tf / 1e3:.0f} GB/s)  bwd {tb:.2f} us ({P * CH * 6 / tb / 1e3:.0f} GB/s)")
    elif what == "conv":
        (B,) = args
        H = W = 28
        C = N = 768
        geo = (ctypes.c_long * 6)()
        _lib.check(L.ebc_dec_geometry(code, B, H, W, C, geo), "geo")
        xpad = torch.randn(geo[4], C, device="cuda").to(dt)
        wk = (torch.randn(N, 3, 3, C, device="cuda") / 80).to(dt)
        out = torch.empty(B * H * W, N, device="cuda", dtype=dt)
        colsum = torch.empty(2, N, device="cuda", dtype=torch.float64)
        ws = torch.zeros(L.ebc_dec_workspace_bytes(code, B, H, W, C, N), device="cuda", dtype=torch.uint8)
        us = timeit(lambda: L.ebc_conv3x3_fwd(code, _lib.ptr(xpad), _lib.ptr(wk), _lib.ptr(out), _lib.ptr(colsum), None,
                                              None, _lib.ptr(ws), ws.numel(), B, H, W, C, N, st), a.reps)
        f = 2.0 * B * H * W * N * 9 * C
        print(f"conv3x3 B={B}: {us:.2f} us  {f / us / 1e6:.1f} TF/s")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

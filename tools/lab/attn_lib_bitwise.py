"""Bitwise A/B of the attention kernels of two library builds (lab, not product): the default in-tree library against
another build (tools/build_old.sh attention <rev> <name> -> clip-ebc_amd/lib/<name>/libebc_hip.so), same inputs, same
stream.  Used for changes that must not move a bit (operand staging, store forms).
    python tools/lab/attn_lib_bitwise.py clip-ebc_amd/lib/old/libebc_hip.so"""
import ctypes
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
from ebc_amd import _lib  # noqa: E402

CODES = {torch.float16: 1, torch.bfloat16: 2}


def run(L_, dt, B, L, H=12, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed + B * 1000 + L)
    qkv = (torch.randn(B * L, 3 * H * 64, device="cuda", generator=g) * 1.5).to(dt)
    dout = torch.randn(B * L, H * 64, device="cuda", generator=g).to(dt)
    out = torch.empty(B * L, H * 64, device="cuda", dtype=dt)
    lse = torch.empty(B, H, L, device="cuda")
    delta = torch.empty(B, H, L, device="cuda")
    dqkv = torch.full_like(qkv, float("nan"))
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = L_.ebc_attention_fwd(CODES[dt], p(qkv), p(out), p(lse), B, L, H, st)
    rc |= L_.ebc_attention_bwd(CODES[dt], p(qkv), p(dout), p(out), p(lse), p(delta), p(dqkv), B, L, H, st)
    torch.cuda.synchronize()
    assert rc == 0, rc
    return out, lse, dqkv


def main():
    other = ctypes.CDLL(os.path.abspath(sys.argv[1]))
    mine = _lib.lib()
    bad = 0
    for dt in (torch.float16, torch.bfloat16):
        for B, L in ((16, 229), (32, 229), (3, 229), (2, 197), (1, 5), (2, 256), (22, 229), (1, 100)):
            a, b = run(mine, dt, B, L), run(other, dt, B, L)
            same = [torch.equal(x.view(torch.int16) if x.dtype != torch.float32 else x.view(torch.int32),
                                y.view(torch.int16) if y.dtype != torch.float32 else y.view(torch.int32)) for x, y in zip(a, b)]
            fin = bool(torch.isfinite(a[2]).all())
            print(f"{str(dt):15s} B {B:2d} L {L:3d}  out / lse / dqkv bitwise {same}  dqkv finite {fin}", flush=True)
            bad += (not all(same)) or (not fin)
    print("ALL BITWISE" if bad == 0 else f"{bad} CASES DIFFER")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

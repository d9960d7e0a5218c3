"""Debug: attention forward/backward per (crop, head) independent of the batch and repeatable, f32 / f16 (r04)."""
import sys
import torch
sys.path.insert(0, "clip-ebc_amd")
from ebc_amd import _lib
L = _lib.lib()
H, Lq = 12, 229
for dname, dt in (("f32", torch.float32), ("f16", torch.float16)):
    g = torch.Generator(device="cuda").manual_seed(3)
    qkv = (torch.randn(3 * Lq, 3 * H * 64, device="cuda", generator=g) * 1.5).to(dt)
    dout = torch.randn(3 * Lq, H * 64, device="cuda", generator=g).to(dt)
    def fwd(x, B):
        out = torch.empty(B * Lq, H * 64, device="cuda", dtype=dt)
        lse = torch.empty(B, H, Lq, device="cuda")
        _lib.check(L.ebc_attention_fwd(_lib.dtype_code(dt), _lib.ptr(x), _lib.ptr(out), _lib.ptr(lse), B, Lq, H,
                                       _lib.stream()), "fwd")
        return out, lse
    def bwd(x, do, out, lse, B):
        delta = torch.empty(B, H, Lq, device="cuda")
        d = torch.empty_like(x)
        _lib.check(L.ebc_attention_bwd(_lib.dtype_code(dt), _lib.ptr(x), _lib.ptr(do), _lib.ptr(out), _lib.ptr(lse),
                                       _lib.ptr(delta), _lib.ptr(d), B, Lq, H, _lib.stream()), "bwd")
        return d
    o3, l3 = fwd(qkv, 3)
    o3b, l3b = fwd(qkv, 3)
    o1, l1 = fwd(qkv[2 * Lq:].contiguous(), 1)
    d3 = bwd(qkv, dout, o3, l3, 3)
    d1 = bwd(qkv[2 * Lq:].contiguous(), dout[2 * Lq:].contiguous(), o1, l1, 1)
    print(dname, "fwd repeat bitwise", torch.equal(o3, o3b), torch.equal(l3, l3b),
          "| crop 2 alone vs in batch of 3: out", torch.equal(o3[2 * Lq:], o1), "lse", torch.equal(l3[2], l1[0]),
          "max|d|", float((o3[2 * Lq:].float() - o1.float()).abs().max()),
          "| bwd", torch.equal(d3[2 * Lq:], d1), float((d3[2 * Lq:].float() - d1.float()).abs().max()))

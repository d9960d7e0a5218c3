"""Debug helper: where the chunked attention forward differs from fp64 torch (rows / heads / columns)."""
import sys
import torch
sys.path.insert(0, "clip-ebc_amd")
from ebc_amd import _lib

for dname, dt in (("f16", torch.float16),):
    for B, L in ((1, 257),):
        H = 12
        g = torch.Generator(device="cuda").manual_seed(7)
        qkv = (torch.randn(B * L, 3 * H * 64, device="cuda", generator=g) * 1.5).to(dt)
        out = torch.full((B * L, H * 64), 77.0, device="cuda", dtype=dt)
        lse = torch.full((B, H, L), 77.0, device="cuda")
        _lib.check(_lib.lib().ebc_attention_fwd(_lib.dtype_code(dt), _lib.ptr(qkv), _lib.ptr(out), _lib.ptr(lse), B, L, H,
                                                _lib.stream()), "attn")
        torch.cuda.synchronize()
        q, k, v = qkv.double().view(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
        s = (q @ k.transpose(-1, -2)) / 8.0
        ref_l = torch.logsumexp(s, -1)
        ob = out.double().view(B * L, H, 64)
        nanm = torch.isnan(ob)
        print("nan columns (head 0, any row):", nanm[:, 0].any(0).nonzero().flatten().tolist())
        print("nan rows (head 0):", nanm[:, 0].any(1).nonzero().flatten().tolist()[:40])
        print("nan count per row (head 0) first 20:", nanm[:20, 0].sum(1).tolist())
        d = (lse.double() - ref_l)[0, 0]
        print("lse diff head 0 rows 0..20:", [round(x, 4) for x in d[:20].tolist()])
        print("lse diff head 0 rows 240..257:", [round(x, 4) for x in d[240:].tolist()])
        print("row 0 head 0 got:", [round(x, 3) for x in ob[0, 0].tolist()])

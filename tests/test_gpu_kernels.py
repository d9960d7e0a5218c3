"""GPU numerics of the encoder building blocks (LayerNorm, attention, head) vs plain torch fp64/fp32."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import ANCHORS_NWPU, golden, rel_l2, rel_max
from ebc_amd import _lib
from oracle import ref
from ebc_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}
TOL = {"f32": 1e-5, "f16": 2e-3, "bf16": 1.6e-2}


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
def test_layernorm_fwd_bwd(dname):
    dt = DT[dname]
    M, D = 1000, 768
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(M, D, device="cuda", generator=g) * 3 + 1
    gam = torch.randn(D, device="cuda", generator=g) * 0.1 + 1
    bet = torch.randn(D, device="cuda", generator=g) * 0.1
    out = torch.empty(M, D, device="cuda", dtype=dt)
    mean = torch.empty(M, device="cuda"); rstd = torch.empty(M, device="cuda")
    L = _lib.lib()
    _lib.check(L.ebc_layernorm_fwd(_lib.dtype_code(dt), _lib.ptr(x), 0, 0, 0, _lib.ptr(gam), _lib.ptr(bet), _lib.ptr(out),
                                   None, _lib.ptr(mean), _lib.ptr(rstd), M, D, _lib.stream()), "ln")
    xr = x.double().requires_grad_(True)
    y = F.layer_norm(xr, (D,), gam.double(), bet.double(), 1e-5)
    assert _rel(out, y) < TOL[dname]
    dy = torch.randn(M, D, device="cuda", generator=g).to(dt)
    dx_in = torch.randn(M, D, device="cuda", generator=g)
    dx = torch.empty(M, D, device="cuda")
    dxt = torch.empty(M, D, device="cuda", dtype=dt)
    _lib.check(L.ebc_layernorm_bwd(_lib.dtype_code(dt), 0, _lib.ptr(dy), _lib.ptr(x), 0, 0, 0, _lib.ptr(mean), _lib.ptr(rstd),
                                   _lib.ptr(gam), _lib.ptr(dx_in), _lib.ptr(dx), _lib.ptr(dxt), M, D, _lib.stream()), "lnb")
    (gx,) = torch.autograd.grad(y, xr, dy.double())
    assert _rel(dx, gx + dx_in.double()) < 1e-5
    assert _rel(dxt, gx + dx_in.double()) < TOL[dname] + 1e-5


@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("B,L", [(3, 229), (2, 197), (1, 5), (2, 256), (2, 257), (1, 300), (2, 513), (1, 817),
                                 (22, 229)])
def test_attention_fwd_bwd(dname, B, L):
    """L > 256: K / V (Q / dO) streamed through LDS in 256-row chunks, online softmax in the forward (817 = 448x448
    inputs with 32 prompts, the reference trainer's default input_size).  22 crops x 12 heads = 264 (crop, head) units,
    more than the 256 CUs: the forward's 8-wave workgroups of 128 queries (the 32-crop step's instance)."""
    dt = DT[dname]
    H = 12
    g = torch.Generator(device="cuda").manual_seed(B * 1000 + L)
    qkv = (torch.randn(B * L, 3 * H * 64, device="cuda", generator=g) * 1.5).to(dt)
    out = torch.empty(B * L, H * 64, device="cuda", dtype=dt)
    lse = torch.empty(B, H, L, device="cuda")
    Lb = _lib.lib()
    _lib.check(Lb.ebc_attention_fwd(_lib.dtype_code(dt), _lib.ptr(qkv), _lib.ptr(out), _lib.ptr(lse), B, L, H, _lib.stream()), "attn")
    q, k, v = qkv.double().view(B, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    q.requires_grad_(True); k.requires_grad_(True); v.requires_grad_(True)
    s = (q @ k.transpose(-1, -2)) / 8.0
    o = (s.softmax(-1) @ v)
    o_flat = o.permute(0, 2, 1, 3).reshape(B * L, H * 64)
    assert _rel(out, o_flat) < TOL[dname]
    assert _rel(lse, torch.logsumexp(s, -1)) < 1e-5
    # every row on its own (a wrong running maximum in one query lane overflows that row's exp sum: r03's long-kernel
    # failure was NaN rows), not only the whole tensor's norm
    ref_lse = torch.logsumexp(s, -1)
    assert bool(torch.isfinite(out).all()) and bool(torch.isfinite(lse).all())
    assert float(((lse.double() - ref_lse).abs() / (1.0 + ref_lse.abs())).max()) < 1e-5
    row_err = (out.double() - o_flat).norm(dim=1) / o_flat.norm(dim=1)
    assert float(row_err.max()) < 8 * TOL[dname], float(row_err.max())
    dout = torch.randn(B * L, H * 64, device="cuda", generator=g).to(dt)
    delta = torch.empty(B, H, L, device="cuda")
    dqkv = torch.empty_like(qkv)
    _lib.check(Lb.ebc_attention_bwd(_lib.dtype_code(dt), _lib.ptr(qkv), _lib.ptr(dout), _lib.ptr(out), _lib.ptr(lse),
                                    _lib.ptr(delta), _lib.ptr(dqkv), B, L, H, _lib.stream()), "attn_bwd")
    gq, gk, gv = torch.autograd.grad(o_flat, (q, k, v), dout.double())
    ref_d = torch.stack([gq, gk, gv], 0).permute(1, 3, 0, 2, 4).reshape(B * L, 3 * H * 64)
    tol = TOL[dname] * (3 if dt != torch.float32 else 1)
    d3 = dqkv.view(B * L, 3, H * 64)
    r3 = ref_d.view(B * L, 3, H * 64)
    for i in range(3):
        assert _rel(d3[:, i], r3[:, i]) < tol, i


@pytest.mark.parametrize("dname", ["f32", "f16"])
def test_attention_batch_invariance(dname):
    """One crop's attention output / lse / gradient must not depend on the batch it is in: alone (the 16-wave
    forward: 12 units <= 256 CUs) and as crop 21 of 22 (264 units: the 8-wave forward of 128-query workgroups,
    attn_fwd_waves), and bitwise repeatable.  The DDP / SyncBN test compares ranks of 2 and 1 crops with one
    process on 3, and the 32-crop ranks of the multi-GPU bench with 16-crop single-GPU runs."""
    dt = DT[dname]
    H, Lq, B = 12, 229, 22
    Lb = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(11)
    qkv = (torch.randn(B * Lq, 3 * H * 64, device="cuda", generator=g) * 1.5).to(dt)
    dout = torch.randn(B * Lq, H * 64, device="cuda", generator=g).to(dt)

    def run(x, do, n):
        out = torch.empty(n * Lq, H * 64, device="cuda", dtype=dt)
        lse = torch.empty(n, H, Lq, device="cuda")
        _lib.check(Lb.ebc_attention_fwd(_lib.dtype_code(dt), _lib.ptr(x), _lib.ptr(out), _lib.ptr(lse), n, Lq, H,
                                        _lib.stream()), "fwd")
        delta = torch.empty(n, H, Lq, device="cuda")
        d = torch.empty_like(x)
        _lib.check(Lb.ebc_attention_bwd(_lib.dtype_code(dt), _lib.ptr(x), _lib.ptr(do), _lib.ptr(out), _lib.ptr(lse),
                                        _lib.ptr(delta), _lib.ptr(d), n, Lq, H, _lib.stream()), "bwd")
        return out, lse, d
    ob, lb, db = run(qkv, dout, B)
    ob2, lb2, db2 = run(qkv, dout, B)
    assert torch.equal(ob, ob2) and torch.equal(lb, lb2) and torch.equal(db, db2)
    c = B - 1
    sl = slice(c * Lq, (c + 1) * Lq)
    o1, l1, d1 = run(qkv[sl].contiguous(), dout[sl].contiguous(), 1)
    assert torch.equal(ob[sl], o1), float((ob[sl].float() - o1.float()).abs().max())
    assert torch.equal(lb[c], l1[0])
    assert torch.equal(db[sl], d1)


@pytest.mark.parametrize("embed,NB", [(512, 5), (512, 16), (1024, 5), (1024, 12), (1024, 16)])
@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
def test_head_bwd_dz_dtypes(dname, embed, NB):
    """dZ is written in the caller's dtype (fp16/bf16 under autocast), checked against autograd; both CLIP joint
    widths (ViT-B/16 512, ResNet-50 1024) up to 16 bins (embed 1024 with 12+ bins needs > 64 KiB of LDS); the
    d bias / d logit_scale column sums are per-block partials reduced in block order: bitwise equal across runs."""
    dt = DT[dname]
    P, HW = 2 * 784, 784
    g = torch.Generator(device="cuda").manual_seed(3)
    Z = torch.randn(P, embed, device="cuda", generator=g)
    text = torch.randn(NB, embed, device="cuda", generator=g)
    ls = torch.tensor([2.3], device="cuda")
    anchors = torch.arange(NB, device="cuda", dtype=torch.float32) * 0.9
    dl = torch.randn(2, NB, 28, 28, device="cuda", generator=g)
    de = torch.randn(2, 1, 28, 28, device="cuda", generator=g)
    dZ = torch.full((P + 64, embed), 7.0, device="cuda", dtype=dt)      # guard rows must survive
    ws = torch.empty(_lib.lib().ebc_head_bwd_workspace_bytes(P, embed), device="cuda", dtype=torch.uint8)
    runs = []
    for _ in range(2):
        dbias = torch.empty(embed, device="cuda"); dsc = torch.empty(1, device="cuda")
        _lib.check(_lib.lib().ebc_head_bwd(_lib.EBC_F32, _lib.dtype_code(dt), _lib.ptr(Z), _lib.ptr(text), _lib.ptr(ls),
                                           _lib.ptr(anchors), _lib.ptr(dl), _lib.ptr(de), None, _lib.ptr(dZ),
                                           _lib.ptr(dbias), _lib.ptr(dsc), P, HW, NB, embed, _lib.ptr(ws), ws.numel(),
                                           _lib.stream()), "head_bwd")
        runs.append((dbias, dsc))
    assert torch.equal(runs[0][0], runs[1][0]) and torch.equal(runs[0][1], runs[1][1])
    Zr = Z.double().requires_grad_(True)
    lsr = ls.double().requires_grad_(True)
    zn = torch.nn.functional.normalize(Zr, dim=-1)
    tn = torch.nn.functional.normalize(text.double(), dim=-1)
    logits = (lsr.exp() * zn @ tn.t()).view(2, HW, NB).permute(0, 2, 1).reshape(2, NB, 28, 28)
    exp = (logits.softmax(1) * anchors.double().view(1, -1, 1, 1)).sum(1, keepdim=True)
    gz, gls = torch.autograd.grad((logits * dl.double()).sum() + (exp * de.double()).sum(), (Zr, lsr))
    assert _rel(dZ[:P], gz) < TOL[dname] + 1e-5
    assert bool((dZ[P:] == 7.0).all())
    assert _rel(dbias, gz.sum(0)) < 1e-4
    assert abs(float(dsc) - float(gls)) < 1e-4 * abs(float(gls))


def test_head_matches_reference_fixture():
    """F2: projection + similarity head fwd/bwd (fp32) against the reference's own outputs."""
    from ebc_amd.model import _HeadFn
    d = golden("f2_head.npz")
    g = np.random.Generator(np.random.PCG64(int(d["seed"])))
    X = np.maximum(g.standard_normal((2, 768, 28, 28)), 0).astype(np.float32)
    R1 = torch.from_numpy(g.standard_normal((2, 5, 28, 28)).astype(np.float32)).cuda()
    R2 = torch.from_numpy(g.standard_normal((2, 1, 28, 28)).astype(np.float32)).cuda()
    sd = syn.trainable_state(0, layers=1)
    W = torch.tensor(sd["projection.weight"], device="cuda", requires_grad=True)
    b = torch.tensor(sd["projection.bias"], device="cuda", requires_grad=True)
    ls = torch.tensor(sd["logit_scale"], device="cuda", requires_grad=True)
    x = torch.tensor(X, device="cuda", requires_grad=True)
    text = torch.from_numpy(d["text_features"]).cuda()
    anchors = torch.tensor(ANCHORS_NWPU, device="cuda")
    logits, exp = _HeadFn.apply(x, W, b, ls, text, anchors, torch.float32)
    ((logits * R1).sum() + (exp * R2).sum()).backward()
    # the fp32 1x1 projection has K = 768 in a different summation order than MKL
    assert rel_max(logits.detach().cpu().numpy(), d["logits"]) < 1e-4
    assert rel_max(exp.detach().cpu().numpy(), d["exp"]) < 1e-5
    assert (logits.detach().cpu().numpy().argmax(1) == d["logits"].argmax(1)).all()
    assert rel_l2(x.grad.cpu().numpy()[:, ::7, ::3, ::3], d["grad_x_sub"]) < 1e-4
    assert rel_l2(W.grad.cpu().numpy()[::3, ::3], d["grad_proj_w_sub"]) < 1e-4
    assert rel_l2(b.grad.cpu().numpy(), d["grad_proj_b"]) < 1e-4
    assert abs(float(ls.grad) - float(d["grad_logit_scale"])) < 1e-4 * abs(float(d["grad_logit_scale"]))

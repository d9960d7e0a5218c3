"""Parity of the kernel instances that only the BENCHMARKED shapes dispatch.

The GEMM / implicit-GEMM tile configuration depends on the product's shape (gemm.hip pick_cfg /
conv_cfg), so the small shapes of the other tests never run the tiles the bench's 16- and 32-crop steps
and the 140-tile eval batch use.  Each test here first asserts WHICH configuration the shape dispatches
(ebc_gemm_tile_config / ebc_conv_tile_config, the same selection the launch makes) and then checks the
result against torch float64:
  * MLP c_fc + QuickGELU / GELU' and QKV at 16 crops (M = 3664): 256x192 (cfg 3), 192x192 (cfg 4)
  * the N = 768 products at 16 crops (128x96 with 4 loader waves: 4-stage ring for K >= 2304, cfg 16, 3-stage
    for K = 768, cfg 15) and at 32 crops (M = 7328: 2-stage 128x96, cfg 5), STORE and the f32 residual epilogue
  * the 1x1 projection at 16 crops (M = 12544, 128x128, cfg 1) and its dX (128x64, cfg 2)
  * the eval batch (140 tiles, M = 32060): 256x256 (cfg 7) and 256x192 (cfg 3)
  * the decoder BasicBlock at 16 crops (M = 12544: 256x192 implicit GEMM with the BN-statistics,
    store and ReLU-masked gradient-add epilogues, stream-K weight gradient; 32 crops: stream-K convs) in fp16 and bf16:
    forward, every gradient, batch and running statistics
  * a whole 12-layer fp16 training step at 16 and 32 crops against the CPU oracle.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import ANCHORS_NWPU, BINS, golden, rel_l2
from ebc_amd import _lib
from oracle import ref
from ebc_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DT = {"f16": torch.float16, "bf16": torch.bfloat16}
TOL = {"f16": 2e-3, "bf16": 1.6e-2}


def gemm_cfg(dt, M, N, K):
    out = (ctypes.c_int * 3)()
    cfg = _lib.lib().ebc_gemm_tile_config(_lib.dtype_code(dt), M, N, K, out)
    return cfg, tuple(out)


def conv_cfg(dt, mode, M, N, K):
    out = (ctypes.c_int * 3)()
    cfg = _lib.lib().ebc_conv_tile_config(_lib.dtype_code(dt), mode, M, N, K, out)
    return cfg, tuple(out)


def _gemm(dt, epi, out_f32, A, B, bias=None, resid=None, aux=None, C=None):
    M, K = A.shape
    N = B.shape[0]
    if C is None:
        od = torch.float32 if (out_f32 or epi == 2) else dt
        C = torch.empty(M, N, device=A.device, dtype=od)
    _lib.check(_lib.lib().ebc_gemm(_lib.dtype_code(dt), epi, int(out_f32), _lib.ptr(A), _lib.ptr(B), _lib.ptr(C),
                                   _lib.ptr(bias), _lib.ptr(resid), _lib.ptr(aux), M, N, K, _lib.stream(A)), "ebc_gemm")
    return C


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def _operands(dt, M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    return A, B, bias, g


# (M, N, K, expected cfg, (bm, bn)): every instance the 16-/32-crop train step and the eval batch run
BENCH_PRODUCTS = [
    (3664, 3072, 768, 3, (256, 192)),     # c_fc (+GELU) and GELU' at 16 crops
    (3664, 2304, 768, 4, (192, 192)),     # QKV at 16 crops
    (3664, 768, 3072, 16, (128, 96)),     # c_proj (+resid) / dX of c_fc at 16 crops
    (3664, 768, 2304, 16, (128, 96)),     # dX of QKV
    (3664, 768, 768, 15, (128, 96)),      # out-proj (+resid) / its dX
    (7328, 768, 3072, 5, (128, 96)),      # the same at 32 crops (config 4)
    (7328, 768, 768, 5, (128, 96)),
    (7328, 3072, 768, 3, (256, 192)),
    (12544, 512, 768, 1, (128, 128)),     # projection 1x1 conv at 16 crops (f32 out)
    (12544, 768, 512, 2, (128, 64)),      # projection dX
    (32060, 3072, 768, 7, (256, 256)),    # eval batch (140 tiles): c_fc
    (32060, 2304, 768, 3, (256, 192)),    # QKV
    (32060, 768, 3072, 3, (256, 192)),    # c_proj + resid
    (32060, 768, 768, 3, (256, 192)),     # out-proj + resid
]


@pytest.mark.parametrize("dname", ["f16", "bf16"])
@pytest.mark.parametrize("M,N,K,cfg,tile", BENCH_PRODUCTS)
def test_bench_shape_products(dname, M, N, K, cfg, tile):
    dt = DT[dname]
    got, (bm, bn, splits) = gemm_cfg(dt, M, N, K)
    assert got == cfg and (bm, bn) == tile and splits == 1, (got, bm, bn, splits)
    A, B, bias, g = _operands(dt, M, N, K, M + N + K)
    pre = A.double() @ B.double().t() + bias.double()
    tol = TOL[dname] + 4e-3
    if N == 3072:
        # MLP c_fc + QuickGELU with the pre-activation store, then the GELU' epilogue on the same tile
        aux = torch.empty(M, N, device="cuda", dtype=dt)
        C = _gemm(dt, 1, 0, A, B, bias=bias, aux=aux)
        assert _rel(aux, pre) < tol and _rel(C, pre * torch.sigmoid(1.702 * pre)) < tol
        dG = torch.randn(M, K, device="cuda", generator=g).to(dt)
        Wt = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
        D = _gemm(dt, 3, 0, dG, Wt, aux=aux)
        a = aux.double()
        s = torch.sigmoid(1.702 * a)
        assert _rel(D, (dG.double() @ Wt.double().t()) * (s + 1.702 * a * s * (1 - s))) < tol
    elif N == 768:
        # f32 residual epilogue in place (x += out_proj / c_proj) and the plain 16-bit store (dX products)
        X = torch.randn(M, N, device="cuda", generator=g)
        ref = X.double() + pre
        _gemm(dt, 2, 1, A, B, bias=bias, resid=X, C=X)
        assert _rel(X, ref) < TOL[dname]
        C = _gemm(dt, 0, 0, A, B)
        assert C.dtype == dt and _rel(C, pre - bias.double()) < tol
    else:
        out_f32 = N == 512                           # the projection writes f32 Z for the head
        C = _gemm(dt, 0, out_f32, A, B, bias=bias)
        assert _rel(C, pre) < (TOL[dname] if out_f32 else tol)


def _block(C):
    from ebc_amd.model import BasicBlock
    torch.manual_seed(0)
    blk = BasicBlock(C, C)
    with torch.no_grad():
        for bn in (blk.bn1, blk.bn2):
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.2, 0.2)
            bn.running_mean.uniform_(-0.1, 0.1)
            bn.running_var.uniform_(0.5, 2.0)
    return blk


def _decoder_ref(feat, w1, g1, b1, w2, g2, b2, rm, rv):
    x = F.interpolate(feat.permute(0, 3, 1, 2), scale_factor=2, mode="bilinear")
    o = F.relu(F.batch_norm(F.conv2d(x, w1, padding=1), rm[0], rv[0], g1, b1, True, 0.1, 1e-5))
    o = F.batch_norm(F.conv2d(o, w2, padding=1), rm[1], rv[1], g2, b2, True, 0.1, 1e-5)
    return F.relu(o + x).permute(0, 2, 3, 1)


@pytest.mark.parametrize("dname,B", [("f16", 16), ("bf16", 16), ("f16", 32)])
def test_decoder_at_bench_batch(dname, B):
    """BasicBlock(768) after the x2 bilinear adapt at the bench's crop counts (M = B*784 rows): the 256x192
    implicit-GEMM tile for the forward convs (BN statistics epilogue), the data gradients (store and
    ReLU-masked residual-gradient add) and the weight gradients, stream-K where gemm.hip sk_plan takes it."""
    from ebc_amd.model import _DecoderFn
    dt = DT[dname]
    C, h = 768, 14
    M = B * 784
    # 16 crops: 224 tiles of 224x192 (196 of 256x192 would leave 60 CUs idle); 32 crops: 392 of 256x192, 256 whole
    # tiles then 136 shared by 256 workgroups (stream-K)
    assert conv_cfg(dt, 1, M, C, 9 * C) == ((17, (224, 192, 1)) if B == 16 else (3, (256, 192, -256)))
    geo = (ctypes.c_long * 6)()                         # {Hp, Wp, HWp, Kq, Q, Qs}: K of the wgrad = Kq
    _lib.check(_lib.lib().ebc_dec_geometry(_lib.dtype_code(dt), B, 2 * h, 2 * h, C, geo), "ebc_dec_geometry")
    assert geo[3] == B * 784                            # the interior pixels only (r03: B * 14 * 64 padded)
    cfg2, (_, _, splits) = conv_cfg(dt, 2, C, 9 * C, geo[3])
    # 108 tiles x 196 k-tiles: stream-K, shares of 84 k-tiles (7 start offsets) on 252 workgroups; x 392 k-tiles
    # (32 crops): 2-way split-K (gemm.hip sk_plan)
    assert cfg2 == 3 and splits == (-252 if B == 16 else 2), (cfg2, splits)
    blk = _block(C)
    g = torch.Generator(device="cuda").manual_seed(B)
    feat = torch.randn(B, h, h, C, device="cuda", generator=g)
    gy = torch.randn(B, 2 * h, 2 * h, C, device="cuda", generator=g)
    # reference in f32 on the GPU (MIOpen; no xf32 on gfx950): ~1e-6 relative, far inside the 16-bit bars
    params = [p.detach().cuda().float().requires_grad_() for p in
              (blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias)]
    fr = feat.clone().requires_grad_()
    rm = [blk.bn1.running_mean.cuda().float().clone(), blk.bn2.running_mean.cuda().float().clone()]
    rv = [blk.bn1.running_var.cuda().float().clone(), blk.bn2.running_var.cuda().float().clone()]
    yr = _decoder_ref(fr, *params, rm, rv)
    (yr * gy).sum().backward()
    blk = blk.cuda().train()
    fd = feat.clone().requires_grad_()
    y = _DecoderFn.apply(fd, blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
                         blk.bn2.bias, blk, 2, dt, True)
    (y.float() * gy).sum().backward()
    tol = {"f16": 2e-2, "bf16": 6e-2}[dname]
    gtol = {"f16": 4e-2, "bf16": 1.2e-1}[dname]
    assert _rel(y.detach().float(), yr.detach()) < tol
    assert _rel(fd.grad, fr.grad) < gtol
    for p, r in zip((blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias),
                    params):
        assert _rel(p.grad, r.grad) < gtol, tuple(p.shape)
    for bn, m, v in zip((blk.bn1, blk.bn2), rm, rv):
        assert _rel(bn.running_mean, m) < tol and _rel(bn.running_var, v) < tol
        assert int(bn.num_batches_tracked) == 1


def _argmax_ok(logits, ref_logits, tol):
    top2 = np.sort(ref_logits, axis=1)[:, -2:]
    sure = (top2[:, 1] - top2[:, 0]) > tol * np.abs(top2[:, 1]).clip(min=1.0)
    return bool((logits.argmax(1) == ref_logits.argmax(1))[sure].all())


@pytest.mark.parametrize("B", [16, 32])
def test_fp16_train_step_at_bench_batch(B):
    """The bench's workload itself (12 layers, deep VPT, decoder, head, DACE/DMCount, fp16 autocast) at 16
    and 32 crops against the fp32 CPU oracle (mixed-precision tolerances as test_gpu_model.py)."""
    from ebc_amd.losses import DACELoss
    from ebc_amd.model import get_model
    txt = torch.from_numpy(golden("f6_text.npz")["text_features_word"])
    m = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", text_features=txt,
                  weights_seed=0).cuda().train()
    img, pts, dens = syn.synthetic_crops(B, 224, seed=900 + B)
    x = torch.from_numpy(img).cuda()
    with torch.autocast("cuda", dtype=torch.float16):
        logits, exp = m(x)
        loss, info = DACELoss(BINS, 8, count_loss="dmcount", input_size=224)(
            logits, exp, torch.from_numpy(dens).cuda(), [torch.from_numpy(p).cuda() for p in pts])
    loss.backward()
    torch.cuda.synchronize()
    p = ref.params_from_state(syn.full_state(0, layers=12, include_text=False))
    ol, oe, _ = ref.forward(p, torch.from_numpy(img), txt, ANCHORS_NWPU, 12)
    oloss, oinfo = ref.dace_loss(ol, oe, torch.from_numpy(dens), pts, BINS)
    oloss.backward()
    lg, ol = logits.detach().float().cpu().numpy(), ol.detach().numpy()
    tol = 2e-2
    assert rel_l2(lg, ol) < tol
    assert rel_l2(exp.detach().float().cpu().numpy(), oe.detach().numpy()) < tol
    assert _argmax_ok(lg, ol, 5 * tol)
    for k in ("loss", "ce_loss", "count_loss"):
        assert abs(float(info[k]) - float(oinfo[k])) <= tol * abs(float(oinfo[k])) + 1e-3, k
    gv = np.stack([getattr(m, f"vpt_{i}").grad.cpu().numpy() for i in range(12)])
    ogv = np.stack([p[f"vpt_{i}"].grad.numpy() for i in range(12)])
    assert rel_l2(gv, ogv) < 5 * tol
    assert rel_l2(m.projection.weight.grad.cpu().numpy(), p["projection.weight"].grad.numpy()) < 5 * tol
    assert rel_l2(m.image_decoder[0].conv1.weight.grad.cpu().numpy(),
                  p["image_decoder.0.conv1.weight"].grad.numpy()) < 10 * tol

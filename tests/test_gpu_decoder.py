"""Decoder BasicBlock on the HIP implicit-GEMM path vs a torch f64 CPU restatement.

Reference semantics: F.interpolate(x, scale_factor=up, mode="bilinear") (models/clip/model.py:195-196)
then BasicBlock (models/utils.py:254-303): conv3x3-bn-relu-conv3x3-bn-(+x)-relu, BatchNorm2d in
training mode (batch statistics, running-stat update) or eval mode (running statistics).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu

# forward rel-L2 bars; gradients get GTOL (BatchNorm backward subtracts batch means: f32 summation-order
# differences of the 7k-deep convolutions are amplified ~10x)
TOL = {torch.float32: 2e-5, torch.float16: 2e-2, torch.bfloat16: 6e-2}
GTOL = {torch.float32: 5e-4, torch.float16: 4e-2, torch.bfloat16: 1.2e-1}
# fp32 gradients against the f64 reference that follows the HIP forward's ReLU masks (the backward's own arithmetic;
# r05 measured 0.7e-7..2.7e-6 at 1, 2, 3 and 16 crops)
GTOL_MASKED = 1e-5
# fp32: bn1's pre-activation z1 * scale + shift vs the f64 reference's, max abs (values ~N(beta, gamma) ~ O(1)):
# a 6912-deep f32 convolution and the f32 batch mean / rstd
PRE_TOL = 5e-5
# ReLU decisions that differ between the f32 forward and the f64 reference, per mask element: only pre-activations
# within the forward's error of zero can flip (r05: 11 of 2 x 9.6 M at 16 crops, 3 of 2 x 1.8 M at 3 crops)
FLIP_RATE = 5e-6


def _ref(feat, w1, g1, b1, w2, g2, b2, up, rm, rv, training, masks=None, pre=None):
    """The reference block in f64.  masks = (m1, m2) replaces the two ReLUs by products with those {0, 1} masks
    (NCHW): the f64 restatement then follows the HIP forward's own ReLU decisions, so a pre-activation that lies
    within f32 resolution of zero (and took the other sign in the f32 forward) cannot move the comparison.
    pre: a list that receives the two f64 pre-activations (NCHW)."""
    x = feat.permute(0, 3, 1, 2)
    if up > 1:
        x = F.interpolate(x, scale_factor=up, mode="bilinear")
    o = F.conv2d(x, w1, padding=1)
    o = F.batch_norm(o, rm[0], rv[0], g1, b1, training, 0.1, 1e-5)
    if pre is not None:
        pre.append(o.detach())
    o = F.relu(o) if masks is None else o * masks[0]
    o = F.conv2d(o, w2, padding=1)
    o = F.batch_norm(o, rm[1], rv[1], g2, b2, training, 0.1, 1e-5) + x
    if pre is not None:
        pre.append(o.detach())
    return (F.relu(o) if masks is None else o * masks[1]).permute(0, 2, 3, 1)


def _hip_masks(y):
    """The HIP forward's two ReLU masks (NCHW f64), read from the saved tensors of y's _DecoderFn node: the
    conv2 input image hpad (relu(bn1(z1)), zero-padded NHWC) and y itself (relu(bn2(z2) + x)).  Call before
    backward (backward drops the node's state)."""
    from ebc_amd import _lib
    import ctypes
    node = y.grad_fn
    xpad, hpad, yy = node.saved_tensors[:3]
    B, h, w, H, W, C, N = node.meta[:7]
    geo = (ctypes.c_long * 6)()
    _lib.check(_lib.lib().ebc_dec_geometry(_lib.dtype_code(node.meta[8]), B, H, W, C, geo), "geo")
    Hp, Wp = geo[0], geo[1]
    h1 = hpad.view(B, Hp, Wp, N)[:, 1:H + 1, 1:W + 1]
    return ((h1 > 0).permute(0, 3, 1, 2).double().cpu(), (yy > 0).permute(0, 3, 1, 2).double().cpu())


def _hip_pre1(y):
    """bn1's pre-activation as the HIP forward formed it (z1 * scale + shift, f32 operands, NCHW f64)."""
    node = y.grad_fn
    B, h, w, H, W, C, N = node.meta[:7]
    z, _, _, scale, shift = node.outs[0][:5]
    pre = z.double() * scale.double() + shift.double()
    return pre.view(B, H, W, N).permute(0, 3, 1, 2).cpu()


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


def _f64_params(blk):
    params = [p.detach().double().requires_grad_() for p in
              (blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias)]
    rm = [blk.bn1.running_mean.double().clone(), blk.bn2.running_mean.double().clone()]
    rv = [blk.bn1.running_var.double().clone(), blk.bn2.running_var.double().clone()]
    return params, rm, rv


@pytest.mark.parametrize("dtype,B,h,C,up", [(torch.float32, 2, 14, 768, 2), (torch.float16, 2, 14, 768, 2),
                                            # three crops: 2352 rows, a partial last row tile in every conv and
                                            # BatchNorm partial (r04's dropped case)
                                            (torch.float32, 3, 14, 768, 2),
                                            # the bench's 16 crops
                                            (torch.float32, 16, 14, 768, 2), (torch.float16, 16, 14, 768, 2),
                                            # one crop: the weight gradient's K = 784 columns in 832 (its last k-tile
                                            # past the image)
                                            (torch.float32, 1, 14, 768, 2),
                                            (torch.bfloat16, 2, 14, 768, 2), (torch.float32, 3, 7, 128, 1),
                                            (torch.float16, 3, 10, 192, 2),
                                            # H = W = 14: 196 pixels per image, the weight gradient's K padded to 200
                                            # per image (a 16-B K chunk never spans two images), K tail past 5 images
                                            (torch.bfloat16, 5, 7, 128, 2)])
def test_decoder_train_fwd_bwd(dtype, B, h, C, up):
    """Forward, BN running statistics and every gradient vs the f64 restatement.  In fp32 the gradients are held
    to GTOL_MASKED against the f64 reference run on the HIP forward's own ReLU masks, and the masks themselves are
    checked: every decision that differs from the f64 reference's sits at a pre-activation within the f32
    forward's error of zero (PRE_TOL), at the expected rate.  r04 found 2e-3..3.4e-3 on three crops against the
    unmasked reference (dropped then): those were such flips, not a kernel error."""
    from ebc_amd.model import _DecoderFn
    blk = _block(C)
    g = torch.Generator().manual_seed(1)
    feat = torch.randn(B, h, h, C, generator=g)
    H = h * up
    gy = torch.randn(B, H, H, C, generator=g)
    # reference (f64, CPU), its own ReLUs
    params, rm, rv = _f64_params(blk)
    fr = feat.double().requires_grad_()
    pre = []
    yr = _ref(fr, *params, up, rm, rv, True, pre=pre)
    (yr * gy.double()).sum().backward()
    # HIP
    blk = blk.cuda().train()
    fd = feat.cuda().requires_grad_()
    y = _DecoderFn.apply(fd, blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
                         blk.bn2.bias, blk, up, dtype, True)
    assert y.shape == (B, H, H, C) and y.dtype == dtype
    masks = _hip_masks(y)
    pre1_hip = _hip_pre1(y) if dtype == torch.float32 else None
    (y.float() * gy.cuda()).sum().backward()
    tol = TOL[dtype]
    assert rel_l2(y.detach().float().cpu().numpy(), yr.detach().numpy()) < tol
    mods = (blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias)
    for bn, m, v in zip((blk.bn1, blk.bn2), rm, rv):
        assert rel_l2(bn.running_mean.cpu().numpy(), m.numpy()) < tol
        assert rel_l2(bn.running_var.cpu().numpy(), v.numpy()) < tol
        assert int(bn.num_batches_tracked) == 1
    flips = [int((mk != (p > 0).double()).sum()) for mk, p in zip(masks, pre)]
    if dtype != torch.float32:
        assert rel_l2(fd.grad.cpu().numpy(), fr.grad.numpy()) < GTOL[dtype]
        for p, r in zip(mods, params):
            assert rel_l2(p.grad.cpu().numpy(), r.grad.numpy()) < GTOL[dtype], p.shape
        return
    err_pre = float((pre1_hip - pre[0]).abs().max())
    # the f64 reference again, on the HIP forward's masks
    params_m, rm_m, rv_m = _f64_params(_block(C))
    fr_m = feat.double().requires_grad_()
    yrm = _ref(fr_m, *params_m, up, rm_m, rv_m, True, masks=masks)
    (yrm * gy.double()).sum().backward()
    errs = {"dfeat": rel_l2(fd.grad.cpu().numpy(), fr_m.grad.numpy())}
    errs.update({n: rel_l2(p.grad.cpu().numpy(), r.grad.numpy())
                 for n, p, r in zip(("w1", "g1", "b1", "w2", "g2", "b2"), mods, params_m)})
    unmasked = rel_l2(fd.grad.cpu().numpy(), fr.grad.numpy())
    print(f"B={B} C={C}: flips {flips} of {masks[0].numel()} per mask, bn1 pre-activation max err {err_pre:.2e}, "
          f"masked grads " + " ".join(f"{k} {v:.1e}" for k, v in errs.items()) + f", dfeat unmasked {unmasked:.1e}")
    assert err_pre < PRE_TOL
    for f, mk, p in zip(flips, masks, pre):
        assert f <= max(2, FLIP_RATE * mk.numel()), (f, mk.numel())
        sel = mk != (p > 0).double()
        if f:
            assert float(p[sel].abs().max()) < PRE_TOL            # a flip only where |pre-activation| < f32 error
    for k, v in errs.items():
        assert v < GTOL_MASKED, (k, v)
    if sum(flips) == 0:                           # no decision differs: the plain comparison is the same one
        assert unmasked < GTOL_MASKED


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_decoder_eval_uses_running_stats(dtype):
    from ebc_amd.model import _DecoderFn
    C, B, h, up = 256, 2, 14, 2
    blk = _block(C)
    feat = torch.randn(B, h, h, C, generator=torch.Generator().manual_seed(2))
    rm = [blk.bn1.running_mean.double().clone(), blk.bn2.running_mean.double().clone()]
    rv = [blk.bn1.running_var.double().clone(), blk.bn2.running_var.double().clone()]
    with torch.no_grad():
        yr = _ref(feat.double(), *(p.double() for p in (blk.conv1.weight, blk.bn1.weight, blk.bn1.bias,
                                                         blk.conv2.weight, blk.bn2.weight, blk.bn2.bias)),
                  up, rm, rv, False)
        blk = blk.cuda().eval()
        y = _DecoderFn.apply(feat.cuda(), blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight,
                             blk.bn2.weight, blk.bn2.bias, blk, up, dtype, False)
    assert rel_l2(y.float().cpu().numpy(), yr.numpy()) < TOL[dtype]
    assert int(blk.bn1.num_batches_tracked) == 0


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_decoder_eval_backward(dtype):
    """Backward through the decoder with its BatchNorms on the running statistics (model.eval(): frozen-BN
    fine-tuning): the input gradient is gamma * rstd * g, no batch-mean terms (torch batch_norm_backward with
    training=False); d gamma / d beta are the column sums.  ADVICE r02."""
    from ebc_amd.model import _DecoderFn
    C, B, h, up = 256, 2, 14, 2
    blk = _block(C)
    g = torch.Generator().manual_seed(4)
    feat = torch.randn(B, h, h, C, generator=g)
    gy = torch.randn(B, h * up, h * up, C, generator=g)
    params = [p.detach().double().requires_grad_() for p in
              (blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias)]
    fr = feat.double().requires_grad_()
    rm = [blk.bn1.running_mean.double().clone(), blk.bn2.running_mean.double().clone()]
    rv = [blk.bn1.running_var.double().clone(), blk.bn2.running_var.double().clone()]
    yr = _ref(fr, *params, up, rm, rv, False)
    (yr * gy.double()).sum().backward()
    blk = blk.cuda().eval()
    fd = feat.cuda().requires_grad_()
    y = _DecoderFn.apply(fd, blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
                         blk.bn2.bias, blk, up, dtype, False)
    (y.float() * gy.cuda()).sum().backward()
    assert rel_l2(y.detach().float().cpu().numpy(), yr.detach().numpy()) < TOL[dtype]
    assert rel_l2(fd.grad.cpu().numpy(), fr.grad.numpy()) < GTOL[dtype]
    for p, r in zip((blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias),
                    params):
        assert rel_l2(p.grad.cpu().numpy(), r.grad.numpy()) < GTOL[dtype], p.shape
    assert int(blk.bn1.num_batches_tracked) == 0


def test_conv3x3_abi_matches_torch():
    """ebc_conv3x3_fwd (implicit GEMM, f16) on a padded NHWC image vs torch conv2d, incl. BN column sums."""
    from ebc_amd import _lib
    import ctypes
    L = _lib.lib()
    B, H, W, C, N = 2, 28, 28, 768, 768
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, C, H, W, generator=g)
    wt = torch.randn(N, C, 3, 3, generator=g) / 80
    geo = (ctypes.c_long * 6)()
    _lib.check(L.ebc_dec_geometry(_lib.EBC_F16, B, H, W, C, geo), "geo")
    Hp, Wp, Q = geo[0], geo[1], geo[4]
    xpad = torch.zeros(B, Hp, Wp, C)
    xpad[:, 1:H + 1, 1:W + 1] = x.permute(0, 2, 3, 1)
    xpad = xpad.reshape(Q, C).half().cuda()
    wk = wt.permute(0, 2, 3, 1).half().contiguous().cuda()
    out = torch.empty(B * H * W, N, dtype=torch.float16, device="cuda")
    colsum = torch.empty(2, N, dtype=torch.float64, device="cuda")
    ws = torch.zeros(L.ebc_dec_workspace_bytes(_lib.EBC_F16, B, H, W, C, N), dtype=torch.uint8, device="cuda")
    _lib.check(L.ebc_conv3x3_fwd(_lib.EBC_F16, _lib.ptr(xpad), _lib.ptr(wk), _lib.ptr(out), _lib.ptr(colsum), None,
                                 None, _lib.ptr(ws), ws.numel(), B, H, W, C, N, _lib.stream()), "conv")
    ref = F.conv2d(x.half().double(), wt.half().double(), padding=1).permute(0, 2, 3, 1).reshape(-1, N)
    assert rel_l2(out.float().cpu().numpy(), ref.numpy()) < 2e-3
    np.testing.assert_allclose(colsum[0].cpu().numpy(), ref.sum(0).numpy(), rtol=1e-2, atol=1e-1)
    np.testing.assert_allclose(colsum[1].cpu().numpy(), (ref ** 2).sum(0).numpy(), rtol=2e-3)


@pytest.mark.parametrize("B,H,C,N,plan", [
    (16, 28, 256, 768, (224, 192, 1)),       # 196 tiles of 256x192 < 256 CUs: 224 tiles of 224x192, one launch
    (8, 56, 512, 2048, (256, 256, -64)),     # 784 tiles of 256x256: 768 whole, then 16 tiles on 64 workgroups
    (8, 56, 256, 1024, (256, 256, -256)),    # 392 tiles: 256 whole, then 136 tiles on 256 workgroups
    (8, 56, 128, 1024, (256, 256, 1))])      # 18 k-tiles a tile: too short to share, plain launch
def test_conv3x3_stream_k(B, H, C, N, plan):
    """ebc_conv3x3_fwd at shapes whose last wave of tiles would leave CUs idle (gemm.hip sk_plan): the whole waves
    as a plain launch, the other tiles' k-tiles shared by the stream-K grid (a tile cut between workgroups summed by
    its last piece), with and without the BN column-sum epilogue, vs torch conv2d; bitwise equal across launches."""
    from ebc_amd import _lib
    import ctypes
    L = _lib.lib()
    W = H
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(B, C, H, W, generator=g, device=dev).half()
    wt = (torch.randn(N, C, 3, 3, generator=g, device=dev) / (3 * C ** 0.5)).half()
    geo = (ctypes.c_long * 6)()
    _lib.check(L.ebc_dec_geometry(_lib.EBC_F16, B, H, W, C, geo), "geo")
    Hp, Wp, Q = geo[0], geo[1], geo[4]
    xpad = torch.zeros(B, Hp, Wp, C, device=dev, dtype=torch.float16)
    xpad[:, 1:H + 1, 1:W + 1] = x.permute(0, 2, 3, 1)
    xpad = xpad.reshape(Q, C)
    wk = wt.permute(0, 2, 3, 1).contiguous()
    ref = F.conv2d(x.float(), wt.float(), padding=1).permute(0, 2, 3, 1).reshape(-1, N).double()
    cfg_out = (ctypes.c_int * 3)()
    L.ebc_conv_tile_config(_lib.EBC_F16, 1, B * H * W, N, 9 * C, cfg_out)
    assert tuple(cfg_out) == plan
    ws = torch.zeros(L.ebc_dec_workspace_bytes(_lib.EBC_F16, B, H, W, C, N), dtype=torch.uint8, device=dev)
    for stats in (True, False):
        outs = []
        colsum = torch.empty(2, N, dtype=torch.float64, device=dev)
        for _ in range(2):                         # twice: the arrival counters must come back re-armed
            out = torch.empty(B * H * W, N, dtype=torch.float16, device=dev)
            _lib.check(L.ebc_conv3x3_fwd(_lib.EBC_F16, _lib.ptr(xpad), _lib.ptr(wk), _lib.ptr(out),
                                         _lib.ptr(colsum) if stats else None, None, None, _lib.ptr(ws), ws.numel(),
                                         B, H, W, C, N, _lib.stream()), "conv")
            outs.append(out)
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1])       # the pieces' sum order is fixed: deterministic
        out = outs[1]
        assert rel_l2(out.double(), ref) < 2e-3
        if stats:
            torch.testing.assert_close(colsum[0], ref.sum(0), rtol=1e-2, atol=2.0)
            torch.testing.assert_close(colsum[1], (ref ** 2).sum(0), rtol=3e-3, atol=1.0)
    assert int(ws[:16384].view(torch.int32).abs().sum()) == 0


@pytest.mark.parametrize("B,plan", [(16, (256, 192, -252)),     # stream-K: 252 shares of 84 k-tiles (7 start offsets)
                                    (32, (256, 192, 2)),        # 392 k-tiles a tile: 2-way split-K
                                    (3, None)])                 # 3 crops: 2352 pixels, a K tail
def test_conv3x3_wgrad_abi_matches_torch(B, plan):
    """ebc_conv3x3_wgrad (MODE 2 implicit GEMM over the interior pixels) on f16 operands vs torch's conv2d weight
    gradient of the same f16 values in f64: only the f32 accumulation order differs (rel-L2 < 1e-5); bitwise equal
    across launches (the stream-K pieces / split partials are summed in a fixed order)."""
    from ebc_amd import _lib
    import ctypes
    L = _lib.lib()
    dt, H, W, C = torch.float16, 28, 28, 768
    N = C
    dev = torch.device("cuda")
    geo = (ctypes.c_long * 6)()
    _lib.check(L.ebc_dec_geometry(_lib.EBC_F16, B, H, W, C, geo), "geo")
    Hp, Wp, HWp, Kq, Q, Qs = (int(v) for v in geo)
    if plan is not None:
        out = (ctypes.c_int * 3)()
        L.ebc_conv_tile_config(_lib.EBC_F16, 2, N, 9 * C, Kq, out)
        assert tuple(out) == plan
    g = torch.Generator(device=dev).manual_seed(50 + B)
    x = torch.randn(B, H, W, C, generator=g, device=dev).to(dt)
    dz = (torch.randn(B, H, W, N, generator=g, device=dev) / 8).to(dt)
    xpad = torch.zeros(B, Hp, Wp, C, device=dev, dtype=dt)
    xpad[:, 1:H + 1, 1:W + 1] = x
    xT3 = torch.empty(3, C, Qs, device=dev, dtype=dt)
    _lib.check(L.ebc_dec_transpose3(_lib.EBC_F16, _lib.ptr(xpad), _lib.ptr(xT3), B, H, W, C, _lib.stream()), "t3")
    dzT = torch.zeros(N, Qs, device=dev, dtype=dt)
    dzT[:, :B * HWp].view(N, B, HWp)[:, :, :H * W] = dz.reshape(B, H * W, N).permute(2, 0, 1)
    ws = torch.zeros(L.ebc_dec_workspace_bytes(_lib.EBC_F16, B, H, W, C, N), dtype=torch.uint8, device=dev)
    outs = []
    for _ in range(2):
        dw = torch.empty(N, C, 3, 3, device=dev)
        _lib.check(L.ebc_conv3x3_wgrad(_lib.EBC_F16, _lib.ptr(dzT), _lib.ptr(xT3), _lib.ptr(dw), _lib.ptr(ws), ws.numel(),
                                       B, H, W, C, N, _lib.stream()), "wgrad")
        outs.append(dw)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).cpu().double(), (N, C, 3, 3),
                                      dz.permute(0, 3, 1, 2).cpu().double(), padding=1)
    err = rel_l2(outs[1].cpu().double(), ref)
    print(f"B={B}: wgrad rel-L2 vs f64 {err:.2e}")
    assert err < 1e-5
    assert int(ws[:16384].view(torch.int32).abs().sum()) == 0          # arrival counters re-armed


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,B", [(torch.float16, 16), (torch.bfloat16, 3), (torch.float32, 2)])
def test_transpose3_matches_definition(dtype, B):
    """ebc_dec_transpose3 bit for bit against its definition: xT3[kx][c][pos] = xpad[(b Hp + yp) Wp + x + kx][c] for
    pos = b Pimg + yp W + x (b < B), 0 past the last image; the pad cells are copied as they are."""
    from ebc_amd import _lib
    import ctypes
    L = _lib.lib()
    H, W, C = 28, 28, 768
    code = {torch.float16: _lib.EBC_F16, torch.bfloat16: _lib.EBC_BF16, torch.float32: _lib.EBC_F32}[dtype]
    dev = torch.device("cuda")
    geo = (ctypes.c_long * 6)()
    _lib.check(L.ebc_dec_geometry(code, B, H, W, C, geo), "geo")
    Hp, Wp, HWp, Kq, Q, Qs = (int(v) for v in geo)
    g = torch.Generator(device=dev).manual_seed(7 + B)
    xpad = torch.randn(B, Hp, Wp, C, generator=g, device=dev).to(dtype)      # pad cells non-zero too: copied as they are
    xT3 = torch.full((3, C, Qs), 7.0, device=dev, dtype=dtype)
    _lib.check(L.ebc_dec_transpose3(code, _lib.ptr(xpad), _lib.ptr(xT3), B, H, W, C, _lib.stream()), "t3")
    torch.cuda.synchronize()
    ref = torch.zeros(3, C, Qs, dtype=dtype)
    xp = xpad.cpu()
    for kx in range(3):
        blk = xp[:, :, kx:kx + W, :]                                            # [B, Hp, W, C]: x + kx
        ref[kx, :, :B * Hp * W] = blk.reshape(B * Hp * W, C).t()
    assert torch.equal(xT3.cpu(), ref)

"""CLIP-EBC with the CLIP ResNet-50 backbone (config 2: clip_resnet50, 448 crops, reduction 8, bf16).

Reference surface:
  * image encoder `ModifiedResNet(features_only=True, out_indices=(-1,), reduction)` with its stem, the
    anti-aliased Bottleneck stages and layer4 at stride 1 when reduction <= 16 (models/clip/_clip/
    image_encoder.py:10-115, blocks.py:56-101).  It is TRAINABLE for the ResNet backbones
    (models/clip/model.py:51-52: no freezing) and runs on PyTorch-ROCm (MIOpen convolutions, channels_last,
    the caller's autocast) -- SURVEY.md §8 keeps the encoder off the HIP path for this config.
  * decoder `Bottleneck(2048, 2048, expansion=1)` (models/utils.py:306-363, cfg [2048] from
    models/clip/model.py:234-238, `_init_weights` :366-379) and the projection + similarity head: on
    libebc_hip.so (`_BottleneckFn`, `model._HeadFn` at embed width 1024).

Layout on the HIP side: the encoder's NHWC (channels_last) layer4 output is taken as f32 rows
[B, h, w, 2048]; every decoder activation is an unpadded row matrix [P = B*H*W][2048] in the compute dtype,
except conv2's input, which is the zero-padded image the implicit-GEMM 3x3 conv reads.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import Any, List, Optional, Tuple

import torch
from torch import Tensor, nn

from . import _lib


# ----------------------------------------------------------------------------- encoder (PyTorch-ROCm)
class AttnBottleneck(nn.Module):
    """blocks.py:56-101: 1x1 -> 3x3 -> avgpool(stride) -> 1x1 (x4), downsample = avgpool + 1x1 + BN."""
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu2 = nn.ReLU(inplace=True)
        self.avgpool = nn.AvgPool2d(stride) if stride > 1 else nn.Identity()
        self.conv3 = nn.Conv2d(planes, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu3 = nn.ReLU(inplace=True)
        self.downsample = None
        self.stride = stride
        if stride > 1 or inplanes != planes * self.expansion:
            self.downsample = nn.Sequential(OrderedDict([
                ("-1", nn.AvgPool2d(stride)),
                ("0", nn.Conv2d(inplanes, planes * self.expansion, 1, stride=1, bias=False)),
                ("1", nn.BatchNorm2d(planes * self.expansion))]))

    def forward(self, x: Tensor) -> Tensor:
        out = self.relu1(self.bn1(self.conv1(x)))
        out = self.relu2(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(self.avgpool(out)))
        idt = x if self.downsample is None else self.downsample(x)
        return self.relu3(out + idt)


class ModifiedResNet(nn.Module):
    """image_encoder.py:10-115 with features_only=True, out_indices=(-1,): returns layer4's output."""

    def __init__(self, layers: Tuple[int, int, int, int] = (3, 4, 6, 3), output_dim: int = 1024,
                 input_resolution: int = 224, width: int = 64, heads: int = 32, reduction: Optional[int] = 32,
                 **kw: Any) -> None:
        super().__init__()
        reduction = 32 if reduction is None else reduction
        self.input_resolution = (input_resolution, input_resolution)
        self.downsampling_rate = 32
        self.conv1 = nn.Conv2d(3, width // 2, 3, stride=2, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(width // 2)
        self.relu1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(width // 2, width // 2, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width // 2)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(width // 2, width, 3, padding=1, bias=False)
        self.bn3 = nn.BatchNorm2d(width)
        self.relu3 = nn.ReLU(inplace=True)
        self.avgpool = nn.AvgPool2d(2)
        self._inplanes = width
        self.layer1 = self._make_layer(width, layers[0])
        self.layer2 = self._make_layer(width * 2, layers[1], stride=2)
        self.layer3 = self._make_layer(width * 4, layers[2], stride=2)
        self.layer4 = self._make_layer(width * 8, layers[3], stride=1 if reduction <= 16 else 2)
        self.features_only, self.out_indices = True, [4]
        self.channels = width * 32
        self.reduction = self.downsampling_rate // 2 if reduction <= 16 else self.downsampling_rate
        self.clip_embed_dim = output_dim

    def _make_layer(self, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        layers = [AttnBottleneck(self._inplanes, planes, stride)]
        self._inplanes = planes * AttnBottleneck.expansion
        for _ in range(1, blocks):
            layers.append(AttnBottleneck(self._inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x: Tensor) -> Tensor:
        x = x.type(self.conv1.weight.dtype)
        x = self.relu1(self.bn1(self.conv1(x)))
        x = self.relu2(self.bn2(self.conv2(x)))
        x = self.relu3(self.bn3(self.conv3(x)))
        x = self.avgpool(x)
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))


# ----------------------------------------------------------------------------- decoder (HIP)
class Bottleneck(nn.Module):
    """Parameter layout of models/utils.py:306-363 (ResNet v1.5 Bottleneck; the decoder uses expansion 1 and
    in_channels == out_channels, so `downsample` is the identity)."""

    def __init__(self, in_channels: int, out_channels: int, expansion: int = 1, **kw: Any) -> None:
        super().__init__()
        if expansion != 1 or in_channels != out_channels:
            raise NotImplementedError("decoder Bottleneck: expansion 1, in_channels == out_channels only "
                                      "(clip_resnet50's cfg [2048], models/clip/model.py:237-238)")
        w = out_channels
        self.expansion = expansion
        self.conv1 = nn.Conv2d(in_channels, w, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(w)
        self.conv2 = nn.Conv2d(w, w, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(w)
        self.conv3 = nn.Conv2d(w, out_channels, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU(inplace=True)
        self.stride = 1
        self.downsample = nn.Identity()




def _batch_norm_fwd(L, bn: nn.Module, colsum: Optional[Tensor], P: int, N: int, training: bool, dev, st, src=None):
    """BatchNorm2d statistics -> (mean, rstd, scale, shift, count, group, colsum); SyncBatchNorm all-reduces
    [sum | sum of squares | this rank's count] in one f64 buffer (as model._DecoderFn).  src = (dtype code, z, ws):
    the statistics of z are taken here -- without an exchange, column sums and finalize in one launch
    (ebc_bn_stats_finalize), else ebc_bn_stats into colsum first."""
    from .model import _bn_group, _bn_momentum
    f32 = dict(device=dev, dtype=torch.float32)
    use_batch = colsum is not None
    pg = _bn_group(bn) if use_batch else None
    count = float(P)
    fused = src is not None and use_batch and pg is None
    if src is not None and use_batch and not fused:
        dt, z, ws = src
        _lib.check(L.ebc_bn_stats(dt, _lib.ptr(z), _lib.ptr(colsum), _lib.ptr(ws), ws.numel(), P, N, st), "ebc_bn_stats")
    if pg is not None:
        colsum[2 * N].fill_(float(P))
        torch.distributed.all_reduce(colsum, group=pg)
        count = -1.0
    mean, rstd, scale, shift = (torch.empty(N, **f32) for _ in range(4))
    upd = use_batch and training and bn.track_running_stats
    nbt = None                                     # num_batches_tracked += 1 inside the finalize launch
    if upd:
        if bn.momentum is None:                    # cumulative average: the factor needs the updated count now
            bn.num_batches_tracked.add_(1)
        else:
            nbt = _lib.ptr(bn.num_batches_tracked)
    mom = _bn_momentum(bn) if upd else 0.0
    if fused:
        dt, z, ws = src
        _lib.check(L.ebc_bn_stats_finalize(dt, _lib.ptr(z), _lib.ptr(ws), ws.numel(), P, N, float(bn.eps), mom,
                                           _lib.ptr(bn.weight.detach()), _lib.ptr(bn.bias.detach()), _lib.ptr(mean),
                                           _lib.ptr(rstd), _lib.ptr(scale), _lib.ptr(shift),
                                           _lib.ptr(bn.running_mean) if upd else None,
                                           _lib.ptr(bn.running_var) if upd else None, None, nbt, st), "ebc_bn_stats_finalize")
        return mean, rstd, scale, shift, count, pg, colsum
    _lib.check(L.ebc_bn_finalize(_lib.ptr(colsum) if use_batch else None, count, float(bn.eps), mom,
                                 _lib.ptr(bn.weight.detach()), _lib.ptr(bn.bias.detach()), _lib.ptr(mean),
                                 _lib.ptr(rstd), _lib.ptr(scale), _lib.ptr(shift),
                                 _lib.ptr(bn.running_mean) if (upd or not use_batch) else None,
                                 _lib.ptr(bn.running_var) if (upd or not use_batch) else None, nbt, N, st),
               "ebc_bn_finalize")
    return mean, rstd, scale, shift, count, pg, colsum


def _batch_norm_bwd(L, gamma: Tensor, state, dnext: Tensor, mask: Optional[Tensor], z: Tensor, ws: Tensor, P: int,
                    N: int, dev, st):
    """Column sums of the BatchNorm backward -> (d gamma, d beta, coef); SyncBatchNorm: d gamma / d beta
    from this rank's sums, the input-gradient coefficients from the all-reduced sums and count."""
    mean, rstd, scale, shift, count, pg, colsum = state
    f32 = dict(device=dev, dtype=torch.float32)
    if pg is None:                    # no exchange: column sums and finalize in one launch
        dg, db, coef = torch.empty(N, **f32), torch.empty(N, **f32), torch.empty(3, N, **f32)
        _lib.check(L.ebc_bn_bwd_reduce_finalize(_lib.dtype_code(z.dtype), _lib.ptr(dnext), _lib.ptr(mask), _lib.ptr(z),
                                                _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(scale), _lib.ptr(shift),
                                                _lib.ptr(gamma.detach()), _lib.ptr(dg), _lib.ptr(db), _lib.ptr(coef),
                                                _lib.ptr(ws), ws.numel(), P, N, st), "ebc_bn_bwd_reduce_finalize")
        return dg, db, _eval_coef(coef, colsum)
    sums = torch.empty(2 * N + (pg is not None), device=dev, dtype=torch.float64)
    _lib.check(L.ebc_bn_bwd_reduce(_lib.dtype_code(z.dtype), _lib.ptr(dnext), _lib.ptr(mask), _lib.ptr(z),
                                   _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(sums),
                                   _lib.ptr(ws), ws.numel(), P, N, st), "ebc_bn_bwd_reduce")
    dg, db, coef = torch.empty(N, **f32), torch.empty(N, **f32), torch.empty(3, N, **f32)
    g = _lib.ptr(gamma.detach())
    _lib.check(L.ebc_bn_bwd_finalize(_lib.ptr(sums), float(P), g, _lib.ptr(rstd), _lib.ptr(dg), _lib.ptr(db),
                                     _lib.ptr(coef), N, st), "ebc_bn_bwd_finalize")
    if pg is not None:
        torch.distributed.all_reduce(sums[: 2 * N], group=pg)
        sums[2 * N:].copy_(colsum[2 * N:])
        _lib.check(L.ebc_bn_bwd_finalize(_lib.ptr(sums), count, g, _lib.ptr(rstd), None, None, _lib.ptr(coef), N, st),
                   "ebc_bn_bwd_finalize(sync)")
    return dg, db, _eval_coef(coef, colsum)


def _eval_coef(coef: Tensor, colsum: Optional[Tensor]) -> Tensor:
    """BatchNorm normalised with its running statistics (eval mode, or track_running_stats with use of the running
    estimates: no batch statistics, colsum None) has the input gradient gamma * rstd * g: the batch-mean terms
    coef[1] = mean(g), coef[2] = mean(g * xhat) of the train-mode backward are zero (torch batch_norm_backward with
    training=False); d gamma / d beta are the same column sums."""
    if colsum is None:
        coef[1:].zero_()
    return coef


def _prep_1x1(L, w: Tensor, cdtype: torch.dtype, st) -> Tuple[Tensor, Tensor]:
    """1x1 conv weight [N, K, 1, 1] f32 -> ([N, K], [K, N]) in the compute dtype, one launch (ebc_prep_weights_1x1)."""
    N, K = w.shape[0], w.shape[1]
    wk = torch.empty(N, K, device=w.device, dtype=cdtype)
    wt = torch.empty(K, N, device=w.device, dtype=cdtype)
    _lib.check(L.ebc_prep_weights_1x1(_lib.dtype_code(cdtype), _lib.ptr(w.detach().float().contiguous()), _lib.ptr(wk),
                                      _lib.ptr(wt), N, K, st), "ebc_prep_weights_1x1")
    return wk, wt


# BatchNorm num_batches_tracked increments of one forward, applied by ONE foreach launch (flush_bn_counters)
# instead of one add kernel per BatchNorm (56 per clip_resnet50 step)
_PENDING_NBT: List[Tensor] = []


def flush_bn_counters() -> None:
    if _PENDING_NBT:
        torch._foreach_add_(_PENDING_NBT, 1)
        _PENDING_NBT.clear()


def _ws(L, dev, dt, B, H, W, C, N, P, Cmax):
    """Stream-owned scratch for one block: the 3x3 conv's (split-K counters + BN partials) and the flat BN kernels'
    column partials over P rows of up to Cmax channels."""
    from .model import _dec_workspace
    rpb = 8 * max(1, 512 // max(1, Cmax // 8))
    need = max(L.ebc_dec_workspace_bytes(dt, B, H, W, C, N), 16384 + (-(-P // rpb)) * 8 * Cmax)
    return _dec_workspace(dev, need)


class _ResBlockFn(torch.autograd.Function):
    """One ModifiedResNet Bottleneck (blocks.py:56-101) on libebc_hip.so, NHWC rows in the compute dtype:
    conv1 1x1 -> bn1 -> relu -> conv2 3x3 -> bn2 -> relu -> avgpool(stride) -> conv3 1x1 -> bn3 (+ identity:
    x, or avgpool(stride) -> 1x1 -> bn for the downsample branch) -> relu.  x [B,H,W,Cin] -> y [B,H/s,W/s,4p]."""

    @staticmethod
    def forward(ctx, x, w1, w2, w3, wd, g1, b1, g2, b2, g3, b3, gd, bd, blk, cdtype, training):
        with _lib.on(x):
            return _ResBlockFn._forward(ctx, x, (w1, w2, w3, wd), blk, cdtype, training)

    @staticmethod
    def _forward(ctx, x, wts, blk, cdtype, training):
        L = _lib.lib()
        x = x.detach()
        if x.dtype != cdtype or not x.is_contiguous():
            x = x.to(cdtype).contiguous()
        B, H, W, Cin = x.shape
        s = blk.stride
        Ho, Wo = H // s, W // s
        P, Po = B * H * W, B * Ho * Wo
        planes, Cout = wts[0].shape[0], wts[2].shape[0]
        down = blk.downsample is not None
        dev, dt, st = x.device, _lib.dtype_code(cdtype), _lib.stream(x)
        ws = _ws(L, dev, dt, B, H, W, planes, planes, P, max(Cin, Cout, planes))
        use_batch = training or not blk.bn1.track_running_stats
        bns = (blk.bn1, blk.bn2, blk.bn3) + ((blk.downsample[2],) if down else ())
        from .model import _bn_group

        def colsum_for(bn):
            return torch.empty(2 * bn.num_features + (_bn_group(bn) is not None), device=dev, dtype=torch.float64) \
                if use_batch else None

        def stats(z, bn, rows, C):
            return _batch_norm_fwd(L, bn, colsum_for(bn), rows, C, training, dev, st, src=(dt, z, ws))

        W1, W1t = _prep_1x1(L, wts[0], cdtype, st)
        W3, W3t = _prep_1x1(L, wts[2], cdtype, st)
        Wd, Wdt = _prep_1x1(L, wts[3], cdtype, st) if down else (None, None)
        geo = (ctypes.c_long * 6)()
        _lib.check(L.ebc_dec_geometry(dt, B, H, W, planes, geo), "ebc_dec_geometry")
        Q = geo[4]
        wk2 = torch.empty(planes, 3, 3, planes, device=dev, dtype=cdtype)
        wf2 = torch.empty(planes, 3, 3, planes, device=dev, dtype=cdtype)
        _lib.check(L.ebc_dec_prep_weights(dt, _lib.ptr(wts[1].detach().float().contiguous()), _lib.ptr(wk2), _lib.ptr(wf2),
                                          planes, planes, st), "ebc_dec_prep_weights")
        # conv1 1x1 -> bn1 -> relu1, into the zero-padded conv2 input
        z1 = torch.empty(P, planes, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(x), _lib.ptr(W1), _lib.ptr(z1), None, None, None, P, planes, Cin, st),
                   "ebc_gemm(conv1)")
        s1 = stats(z1, bns[0], P, planes)
        h1pad = torch.empty(Q, planes, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_relu_pad(dt, _lib.ptr(z1), _lib.ptr(s1[2]), _lib.ptr(s1[3]), _lib.ptr(h1pad), B, H, W, planes,
                                     st), "ebc_bn_relu_pad")
        # conv2 3x3 (BN statistics in the epilogue) -> bn2 -> relu2 -> avgpool(stride)
        z2 = torch.empty(P, planes, device=dev, dtype=cdtype)
        cs2 = colsum_for(bns[1])
        _lib.check(L.ebc_conv3x3_fwd(dt, _lib.ptr(h1pad), _lib.ptr(wk2), _lib.ptr(z2), _lib.ptr(cs2), None, None,
                                     _lib.ptr(ws), ws.numel(), B, H, W, planes, planes, st), "ebc_conv3x3_fwd")
        s2 = _batch_norm_fwd(L, bns[1], cs2, P, planes, training, dev, st)
        h2p = torch.empty(Po, planes, device=dev, dtype=cdtype)
        if s > 1:
            _lib.check(L.ebc_bn_relu_avgpool(dt, _lib.ptr(z2), _lib.ptr(s2[2]), _lib.ptr(s2[3]), _lib.ptr(h2p), B, H, W,
                                             planes, st), "ebc_bn_relu_avgpool")
        else:
            _lib.check(L.ebc_bn_relu(dt, _lib.ptr(z2), _lib.ptr(s2[2]), _lib.ptr(s2[3]), _lib.ptr(h2p), P, planes, st),
                       "ebc_bn_relu")
        # conv3 1x1 -> bn3
        z3 = torch.empty(Po, Cout, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(h2p), _lib.ptr(W3), _lib.ptr(z3), None, None, None, Po, Cout, planes, st),
                   "ebc_gemm(conv3)")
        s3 = stats(z3, bns[2], Po, Cout)
        # identity: x, or avgpool(stride) -> 1x1 -> bn (downsample "-1", "0", "1")
        xd = zd = sd = None
        if down:
            if s > 1:
                xd = torch.empty(Po, Cin, device=dev, dtype=cdtype)
                _lib.check(L.ebc_avgpool2(dt, dt, _lib.ptr(x), _lib.ptr(xd), B, H, W, Cin, st), "ebc_avgpool2")
            else:
                xd = x.view(P, Cin)
            zd = torch.empty(Po, Cout, device=dev, dtype=cdtype)
            _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(xd), _lib.ptr(Wd), _lib.ptr(zd), None, None, None, Po, Cout, Cin, st),
                       "ebc_gemm(downsample)")
            sd = stats(zd, bns[3], Po, Cout)
        y = torch.empty(B, Ho, Wo, Cout, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_add_relu_flat(dt, _lib.ptr(z3), _lib.ptr(s3[2]), _lib.ptr(s3[3]),
                                          _lib.ptr(zd if down else x), _lib.ptr(sd[2]) if down else None,
                                          _lib.ptr(sd[3]) if down else None, _lib.ptr(y), Po, Cout, st), "ebc_bn_add_relu_flat")
        ctx.save_for_backward(x, z1, h1pad, z2, h2p, z3, y, W1t, wf2, W3t, *(() if not down else (xd, zd, Wdt)))
        ctx.states = (s1, s2, s3, sd)
        ctx.gammas = tuple(bn.weight for bn in bns)
        ctx.meta = (B, H, W, Cin, s, Ho, Wo, P, Po, planes, Cout, down, cdtype, x.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        with _lib.on(gy):
            return _ResBlockFn._backward(ctx, gy)

    @staticmethod
    def _backward(ctx, gy):
        from .model import _wgrad_rows
        L = _lib.lib()
        B, H, W, Cin, s, Ho, Wo, P, Po, planes, Cout, down, cdtype, xdt = ctx.meta
        saved = ctx.saved_tensors
        x, z1, h1pad, z2, h2p, z3, y, W1t, wf2, W3t = saved[:10]
        xd, zd, Wdt = saved[10:] if down else (None, None, None)
        s1, s2, s3, sd = ctx.states
        g1, g2, g3 = ctx.gammas[:3]
        dev, dt, st = y.device, _lib.dtype_code(cdtype), _lib.stream(y)
        gy = gy.to(cdtype).contiguous().view(Po, Cout)
        ws = _ws(L, dev, dt, B, H, W, planes, planes, P, max(Cin, Cout, planes))
        geo = (ctypes.c_long * 6)()
        _lib.check(L.ebc_dec_geometry(dt, B, H, W, planes, geo), "ebc_dec_geometry")
        Q, Qs = geo[4], geo[5]
        f32 = dict(device=dev, dtype=torch.float32)

        def apply_flat(g, mask, z, st_, coef, gmask=None):
            dz = torch.empty(z.shape, device=dev, dtype=cdtype)
            _lib.check(L.ebc_bn_bwd_apply_flat(dt, _lib.ptr(g), _lib.ptr(mask), _lib.ptr(z), _lib.ptr(st_[0]),
                                               _lib.ptr(st_[1]), _lib.ptr(st_[2]), _lib.ptr(st_[3]), _lib.ptr(coef),
                                               _lib.ptr(dz), _lib.ptr(gmask), z.shape[0], z.shape[1], st),
                       "ebc_bn_bwd_apply_flat")
            return dz

        # bn3 (+ relu3 through y); without a downsample the identity's gradient is g = gy * (y > 0) itself (f32)
        dg3, db3, coef3 = _batch_norm_bwd(L, g3, s3, gy, y, z3, ws, Po, Cout, dev, st)
        gid = None if down else torch.empty(Po, Cout, **f32)
        dz3 = apply_flat(gy, y, z3, s3, coef3, gid)
        dw3 = _wgrad_rows(L, dz3, h2p, cdtype, dev, st)
        dh2p = torch.empty(Po, planes, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(dz3), _lib.ptr(W3t), _lib.ptr(dh2p), None, None, None,
                              Po, planes, Cout, st), "ebc_gemm(conv3 dX)")
        del dz3
        dwd = dgd = dbd = None
        if down:
            # downsample bn (same masked gradient) -> 1x1 -> avgpool: the identity's input gradient, f32
            dgd, dbd, coefd = _batch_norm_bwd(L, ctx.gammas[3], sd, gy, y, zd, ws, Po, Cout, dev, st)
            dzd = apply_flat(gy, y, zd, sd, coefd)
            dwd = _wgrad_rows(L, dzd, xd, cdtype, dev, st)
            dxd = torch.empty(Po, Cin, **f32)
            _lib.check(L.ebc_gemm(dt, 0, 1, _lib.ptr(dzd), _lib.ptr(Wdt), _lib.ptr(dxd), None, None, None,
                                  Po, Cin, Cout, st), "ebc_gemm(downsample dX)")
            del dzd
            if s > 1:
                gid = torch.empty(P, Cin, **f32)
                _lib.check(L.ebc_avgpool2_bwd(_lib.EBC_F32, _lib.EBC_F32, _lib.ptr(dxd), _lib.ptr(gid), B, H, W, Cin, st),
                           "ebc_avgpool2_bwd(downsample)")
                del dxd
            else:
                gid = dxd
        # avgpool -> relu2 -> bn2 (ReLU mask recomputed from z2) -> conv2's gradients
        if s > 1:
            dh2 = torch.empty(P, planes, device=dev, dtype=cdtype)
            _lib.check(L.ebc_avgpool2_bwd(dt, dt, _lib.ptr(dh2p), _lib.ptr(dh2), B, H, W, planes, st), "ebc_avgpool2_bwd")
            del dh2p
        else:
            dh2 = dh2p
        dg2, db2, coef2 = _batch_norm_bwd(L, g2, s2, dh2, None, z2, ws, P, planes, dev, st)
        dz2pad = torch.empty(Q, planes, device=dev, dtype=cdtype)
        dz2T = torch.empty(planes, Qs, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_bwd_apply(dt, _lib.ptr(dh2), None, _lib.ptr(z2), _lib.ptr(s2[0]), _lib.ptr(s2[1]),
                                      _lib.ptr(s2[2]), _lib.ptr(s2[3]), _lib.ptr(coef2), _lib.ptr(dz2pad), _lib.ptr(dz2T),
                                      B, H, W, planes, st), "ebc_bn_bwd_apply(bn2)")
        del dh2
        xT3 = torch.empty(3, planes, Qs, device=dev, dtype=cdtype)
        _lib.check(L.ebc_dec_transpose3(dt, _lib.ptr(h1pad), _lib.ptr(xT3), B, H, W, planes, st), "ebc_dec_transpose3")
        dw2 = torch.empty(planes, planes, 3, 3, **f32)
        _lib.check(L.ebc_conv3x3_wgrad(dt, _lib.ptr(dz2T), _lib.ptr(xT3), _lib.ptr(dw2), _lib.ptr(ws), ws.numel(),
                                       B, H, W, planes, planes, st), "ebc_conv3x3_wgrad")
        del xT3, dz2T
        dh1 = torch.empty(P, planes, device=dev, dtype=cdtype)
        _lib.check(L.ebc_conv3x3_fwd(dt, _lib.ptr(dz2pad), _lib.ptr(wf2), _lib.ptr(dh1), None, None, None, _lib.ptr(ws),
                                     ws.numel(), B, H, W, planes, planes, st), "ebc_conv3x3_fwd(dgrad)")
        del dz2pad
        # bn1 (ReLU mask recomputed from z1) -> conv1: dx = dz1 W1 + the identity's gradient
        dg1, db1, coef1 = _batch_norm_bwd(L, g1, s1, dh1, None, z1, ws, P, planes, dev, st)
        dz1 = apply_flat(dh1, None, z1, s1, coef1)
        del dh1
        dw1 = _wgrad_rows(L, dz1, x.view(P, Cin), cdtype, dev, st)
        dx = torch.empty(B, H, W, Cin, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 2, 0, _lib.ptr(dz1), _lib.ptr(W1t), _lib.ptr(dx), None, _lib.ptr(gid),
                              None, P, Cin, planes, st), "ebc_gemm(conv1 dX + identity)")
        ctx.states = None
        return (dx.to(xdt) if xdt != cdtype else dx, dw1.view(planes, Cin, 1, 1), dw2, dw3.view(Cout, planes, 1, 1),
                None if dwd is None else dwd.view(Cout, Cin, 1, 1), dg1, db1, dg2, db2, dg3, db3, dgd, dbd,
                None, None, None)


def encoder_forward(enc: "ModifiedResNet", x: Tensor, cdtype: torch.dtype, training: bool) -> Tensor:
    """ModifiedResNet forward with the 16 Bottlenecks on libebc_hip.so: the 3-conv stem + avgpool on
    PyTorch-ROCm (3- and 32-channel convolutions), then NHWC rows through `_ResBlockFn`.
    Returns layer4's output as NHWC [B, h, w, 2048] in the compute dtype."""
    h = x.type(enc.conv1.weight.dtype).contiguous(memory_format=torch.channels_last)
    h = enc.relu1(enc.bn1(enc.conv1(h)))
    h = enc.relu2(enc.bn2(enc.conv2(h)))
    h = enc.avgpool(enc.relu3(enc.bn3(enc.conv3(h))))
    h = h.permute(0, 2, 3, 1)
    with torch.autocast("cuda", enabled=False):
        for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
            for blk in layer:
                d = blk.downsample
                h = _ResBlockFn.apply(h, blk.conv1.weight, blk.conv2.weight, blk.conv3.weight,
                                      None if d is None else d[1].weight, blk.bn1.weight, blk.bn1.bias, blk.bn2.weight,
                                      blk.bn2.bias, blk.bn3.weight, blk.bn3.bias, None if d is None else d[2].weight,
                                      None if d is None else d[2].bias, blk, cdtype, training)
    flush_bn_counters()
    return h


class _BottleneckFn(torch.autograd.Function):
    """Bottleneck(C, C, expansion=1) decoder after the x`up` bilinear adapt (models/clip/model.py:195-197;
    models/utils.py:346-363): conv1x1-BN-ReLU, conv3x3-BN-ReLU, conv1x1-BN, + x, ReLU.
    feat [B,h,w,C] f32 (NHWC) -> y [B,H,W,C] in the compute dtype."""

    @staticmethod
    def forward(ctx, feat, w1, w2, w3, g1, b1, g2, b2, g3, b3, blk, up, cdtype, training):
        with _lib.on(feat):
            return _BottleneckFn._forward(ctx, feat, (w1, w2, w3), (g1, g2, g3), blk, up, cdtype, training)

    @staticmethod
    def _forward(ctx, feat, wts, gammas, blk, up, cdtype, training):
        from .model import _bn_group, _dec_workspace
        L = _lib.lib()
        feat = feat.detach().contiguous()
        B, h, w, C = feat.shape
        H, W = h * up, w * up
        N = wts[0].shape[0]
        if N != C or C % 256:
            raise NotImplementedError("fused Bottleneck decoder: C == N, C % 256 == 0")
        dev, dt, st = feat.device, _lib.dtype_code(cdtype), _lib.stream(feat)
        P = B * H * W
        geo = (ctypes.c_long * 6)()
        _lib.check(L.ebc_dec_geometry(dt, B, H, W, C, geo), "ebc_dec_geometry")
        Q = geo[4]
        ws = _dec_workspace(dev, L.ebc_dec_workspace_bytes(dt, B, H, W, C, N))
        use_batch = training or not blk.bn1.track_running_stats
        bns = (blk.bn1, blk.bn2, blk.bn3)

        def colsum_for(bn):
            if not use_batch:
                return None
            return torch.empty(2 * N + (_bn_group(bn) is not None), device=dev, dtype=torch.float64)

        x = torch.empty(P, C, device=dev, dtype=cdtype)
        _lib.check(L.ebc_dec_upsample(dt, _lib.ptr(feat), _lib.ptr(x), B, h, w, C, up, st), "ebc_dec_upsample")
        W1, W1t = _prep_1x1(L, wts[0], cdtype, st)
        W3, W3t = _prep_1x1(L, wts[2], cdtype, st)
        wk2 = torch.empty(N, 3, 3, N, device=dev, dtype=cdtype)
        wf2 = torch.empty(N, 3, 3, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_dec_prep_weights(dt, _lib.ptr(wts[1].detach().float().contiguous()), _lib.ptr(wk2),
                                          _lib.ptr(wf2), N, N, st), "ebc_dec_prep_weights")
        # conv1 (1x1) + bn1 + relu -> padded conv2 input
        z1 = torch.empty(P, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(x), _lib.ptr(W1), _lib.ptr(z1), None, None, None, P, N, C, st),
                   "ebc_gemm(conv1)")
        s1 = _batch_norm_fwd(L, bns[0], colsum_for(bns[0]), P, N, training, dev, st, src=(dt, z1, ws))
        h1pad = torch.empty(Q, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_relu_pad(dt, _lib.ptr(z1), _lib.ptr(s1[2]), _lib.ptr(s1[3]), _lib.ptr(h1pad), B, H, W, N,
                                     st), "ebc_bn_relu_pad")
        # conv2 (3x3, BN statistics in the GEMM epilogue) + bn2 + relu
        z2 = torch.empty(P, N, device=dev, dtype=cdtype)
        cs2 = colsum_for(bns[1])
        _lib.check(L.ebc_conv3x3_fwd(dt, _lib.ptr(h1pad), _lib.ptr(wk2), _lib.ptr(z2), _lib.ptr(cs2), None, None,
                                     _lib.ptr(ws), ws.numel(), B, H, W, N, N, st), "ebc_conv3x3_fwd")
        s2 = _batch_norm_fwd(L, bns[1], cs2, P, N, training, dev, st)
        h2 = torch.empty(P, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_relu(dt, _lib.ptr(z2), _lib.ptr(s2[2]), _lib.ptr(s2[3]), _lib.ptr(h2), P, N, st),
                   "ebc_bn_relu")
        # conv3 (1x1) + bn3 + identity + relu
        z3 = torch.empty(P, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(h2), _lib.ptr(W3), _lib.ptr(z3), None, None, None, P, N, N, st),
                   "ebc_gemm(conv3)")
        s3 = _batch_norm_fwd(L, bns[2], colsum_for(bns[2]), P, N, training, dev, st, src=(dt, z3, ws))
        y = torch.empty(B, H, W, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_add_relu(dt, _lib.ptr(z3), _lib.ptr(s3[2]), _lib.ptr(s3[3]), _lib.ptr(feat), up, _lib.ptr(y),
                                     B, H, W, N, st), "ebc_bn_add_relu")
        ctx.save_for_backward(x, z1, h1pad, z2, h2, z3, y, W1t, wf2, W3t, *gammas)
        ctx.states = (s1, s2, s3)
        ctx.meta = (B, h, w, H, W, C, N, up, cdtype, P)
        return y

    @staticmethod
    def backward(ctx, gy):
        with _lib.on(gy):
            return _BottleneckFn._backward(ctx, gy)

    @staticmethod
    def _backward(ctx, gy):
        from .model import _dec_workspace, _wgrad_rows
        L = _lib.lib()
        x, z1, h1pad, z2, h2, z3, y, W1t, wf2, W3t, g1, g2, g3 = ctx.saved_tensors
        s1, s2, s3 = ctx.states
        B, h, w, H, W, C, N, up, cdtype, P = ctx.meta
        dev, dt, st = y.device, _lib.dtype_code(cdtype), _lib.stream(y)
        gy = gy.to(cdtype).contiguous().view(P, N)
        ws = _dec_workspace(dev, L.ebc_dec_workspace_bytes(dt, B, H, W, C, N))
        geo = (ctypes.c_long * 6)()
        _lib.check(L.ebc_dec_geometry(dt, B, H, W, C, geo), "ebc_dec_geometry")
        Q, Qs = geo[4], geo[5]
        # bn3 (+ relu through the block output y); the identity branch keeps g = gy * (y > 0) in f32
        dg3, db3, coef3 = _batch_norm_bwd(L, g3, s3, gy, y, z3, ws, P, N, dev, st)
        dz3 = torch.empty(P, N, device=dev, dtype=cdtype)
        gid = torch.empty(P, C, device=dev, dtype=torch.float32)
        mean3, rstd3, sc3, sh3 = s3[:4]
        _lib.check(L.ebc_bn_bwd_apply_flat(dt, _lib.ptr(gy), _lib.ptr(y), _lib.ptr(z3), _lib.ptr(mean3), _lib.ptr(rstd3),
                                           _lib.ptr(sc3), _lib.ptr(sh3), _lib.ptr(coef3), _lib.ptr(dz3), _lib.ptr(gid),
                                           P, N, st), "ebc_bn_bwd_apply_flat(bn3)")
        # conv3: dW3 = dz3^T h2, dh2 = dz3 W3
        dw3 = _wgrad_rows(L, dz3, h2, cdtype, dev, st)
        dh2 = torch.empty(P, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(dz3), _lib.ptr(W3t), _lib.ptr(dh2), None, None, None,
                              P, N, N, st), "ebc_gemm(conv3 dX)")
        del dz3
        # bn2 (+ relu through h2) -> padded / transposed dz2 for the 3x3 conv's gradients
        dg2, db2, coef2 = _batch_norm_bwd(L, g2, s2, dh2, h2, z2, ws, P, N, dev, st)
        mean2, rstd2, sc2, sh2 = s2[:4]
        dz2pad = torch.empty(Q, N, device=dev, dtype=cdtype)
        dz2T = torch.empty(N, Qs, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_bwd_apply(dt, _lib.ptr(dh2), _lib.ptr(h2), _lib.ptr(z2), _lib.ptr(mean2), _lib.ptr(rstd2),
                                      _lib.ptr(sc2), _lib.ptr(sh2), _lib.ptr(coef2), _lib.ptr(dz2pad), _lib.ptr(dz2T),
                                      B, H, W, N, st), "ebc_bn_bwd_apply(bn2)")
        del dh2
        xT3 = torch.empty(3, N, Qs, device=dev, dtype=cdtype)
        _lib.check(L.ebc_dec_transpose3(dt, _lib.ptr(h1pad), _lib.ptr(xT3), B, H, W, N, st), "ebc_dec_transpose3")
        dw2 = torch.empty(N, N, 3, 3, device=dev, dtype=torch.float32)
        _lib.check(L.ebc_conv3x3_wgrad(dt, _lib.ptr(dz2T), _lib.ptr(xT3), _lib.ptr(dw2), _lib.ptr(ws), ws.numel(),
                                       B, H, W, N, N, st), "ebc_conv3x3_wgrad")
        del xT3, dz2T
        dh1 = torch.empty(P, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_conv3x3_fwd(dt, _lib.ptr(dz2pad), _lib.ptr(wf2), _lib.ptr(dh1), None, None, None, _lib.ptr(ws),
                                     ws.numel(), B, H, W, N, N, st), "ebc_conv3x3_fwd(dgrad)")
        del dz2pad
        # bn1 (ReLU mask recomputed from z1)
        dg1, db1, coef1 = _batch_norm_bwd(L, g1, s1, dh1, None, z1, ws, P, N, dev, st)
        mean1, rstd1, sc1, sh1 = s1[:4]
        dz1 = torch.empty(P, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_bwd_apply_flat(dt, _lib.ptr(dh1), None, _lib.ptr(z1), _lib.ptr(mean1), _lib.ptr(rstd1),
                                           _lib.ptr(sc1), _lib.ptr(sh1), _lib.ptr(coef1), _lib.ptr(dz1), None, P, N, st),
                   "ebc_bn_bwd_apply_flat(bn1)")
        del dh1
        # conv1: dW1 = dz1^T x, dx = dz1 W1 + the identity branch's gradient (f32, in place over gid)
        dw1 = _wgrad_rows(L, dz1, x, cdtype, dev, st)
        _lib.check(L.ebc_gemm(dt, 2, 1, _lib.ptr(dz1), _lib.ptr(W1t), _lib.ptr(gid), None,
                              _lib.ptr(gid), None, P, C, N, st), "ebc_gemm(conv1 dX + identity)")
        dfeat = torch.empty(B, h, w, C, device=dev, dtype=torch.float32)
        _lib.check(L.ebc_dec_upsample_bwd(_lib.EBC_F32, _lib.ptr(gid), _lib.ptr(dfeat), B, h, w, C, up, st),
                   "ebc_dec_upsample_bwd")
        ctx.states = None
        return (dfeat, dw1.view(N, C, 1, 1), dw2, dw3.view(N, N, 1, 1), dg1, db1, dg2, db2, dg3, db3,
                None, None, None, None)

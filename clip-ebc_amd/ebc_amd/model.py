"""Drop-in CLIP-EBC model (ViT-B/16 + deep VPT) whose hot path runs in libebc_hip.so.

Reference surface kept:
  * `get_model(backbone, input_size, reduction, bins, anchor_points, **kw)`  (models/__init__.py:10-44)
  * `CLIP_EBC.forward(x) -> (logits [B,N,H/r,W/r], exp [B,1,H/r,W/r])` in train mode, `exp` in eval
    (models/clip/model.py:191-217); attributes `.bins`, `.anchor_points`, `.reduction`,
    `.encoder_reduction`, `.num_vpt`, `.deep_vpt`; identical `state_dict()` keys
    (`image_encoder.*`, `vpt_{l}`, `image_decoder.0.*`, `projection.*`, `text_encoder.*`, `logit_scale`).
  * mixed precision follows the caller's `torch.autocast` (the reference trains under
    `torch.cuda.amp.autocast`, train.py:36-40): fp16/bf16 GEMM inputs, fp32 residual stream and
    statistics; without autocast the whole path is exact-f32 (parity mode).

Execution: the 12-block encoder forward/backward is ONE C-ABI call each (`ebc_vit_forward/backward`);
the BasicBlock decoder (models/utils.py:254-303) runs as implicit-GEMM 3x3 convs with BatchNorm statistics
in the GEMM epilogue plus fused BN/ReLU/residual kernels (`_DecoderFn`); the projection + similarity head
is an MFMA GEMM + a fused head kernel (`_HeadFn`).  The clip_resnet50 backbone (config 2) is in resnet.py.
"""
from __future__ import annotations

import ctypes
import math
from collections import OrderedDict
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor, nn

from . import _lib
from . import synthetic
from .text import CLIPTextEncoder, format_count, prompt_tokens

WIDTH, HEADS, PATCH, EMBED = 768, 12, 16, 512


# ----------------------------------------------------------------------------- parameter containers
class _Block(nn.Module):
    """Parameter layout of ResidualAttentionBlock (models/clip/_clip/blocks.py:22-42)."""

    def __init__(self, width: int = WIDTH, heads: int = HEADS):
        super().__init__()
        self.attn = nn.MultiheadAttention(width, heads)
        self.ln_1 = nn.LayerNorm(width)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(width, 4 * width)), ("gelu", nn.Identity()),
                                              ("c_proj", nn.Linear(4 * width, width))]))
        self.ln_2 = nn.LayerNorm(width)


class _Transformer(nn.Module):
    def __init__(self, width, layers, heads):
        super().__init__()
        self.width, self.layers = width, layers
        self.resblocks = nn.Sequential(*[_Block(width, heads) for _ in range(layers)])


class VisionTransformer(nn.Module):
    """Parameter layout + geometry of the CLIP visual tower, features_only (image_encoder.py:118-198)."""

    def __init__(self, input_resolution: int = 224, patch_size: int = PATCH, output_dim: int = EMBED,
                 width: int = WIDTH, layers: int = 12, heads: int = HEADS):
        super().__init__()
        self.input_resolution = (input_resolution, input_resolution)
        self.patch_size = (patch_size, patch_size)
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch_size, stride=patch_size, bias=False)
        self.num_patches_h = self.num_patches_w = input_resolution // patch_size
        self.class_embedding = nn.Parameter(torch.zeros(width))
        self.positional_embedding = nn.Parameter(torch.zeros(self.num_patches_h * self.num_patches_w + 1, width))
        self.ln_pre = nn.LayerNorm(width)
        self.transformer = _Transformer(width, layers, heads)
        self.ln_post = nn.LayerNorm(width)
        self.channels, self.reduction, self.clip_embed_dim = width, patch_size, output_dim

    def _interpolate_pos_embed(self, h: int, w: int) -> Tensor:
        """image_encoder.py:183-198 (bicubic resize of the patch grid; identity at the native size)."""
        if h == self.num_patches_h and w == self.num_patches_w:
            return self.positional_embedding
        pe = self.positional_embedding[1:].reshape(self.num_patches_h, self.num_patches_w, -1).permute(2, 0, 1)[None]
        pe = F.interpolate(pe, size=(h, w), mode="bicubic")[0].permute(1, 2, 0).reshape(h * w, -1)
        return torch.cat([self.positional_embedding[:1], pe], dim=0)


class BasicBlock(nn.Module):
    """models/utils.py:254-303 (the ViT decoder block, in_channels == out_channels)."""
    expansion = 1

    def __init__(self, in_channels: int, out_channels: int, **kw: Any) -> None:
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(out_channels)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(out_channels)
        self.downsample = nn.Identity()
        if in_channels != out_channels:
            self.downsample = nn.Sequential(nn.Conv2d(in_channels, out_channels, 1, bias=False), nn.BatchNorm2d(out_channels))

    def forward(self, x: Tensor) -> Tensor:
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out = out + self.downsample(x)
        return self.relu(out)


# ----------------------------------------------------------------------------- C structs
_VP = ctypes.c_void_p


class EbcVitLayer(ctypes.Structure):
    _fields_ = [(n, _VP) for n in ("w_qkv", "b_qkv", "w_out", "b_out", "w_fc", "b_fc", "w_proj", "b_proj",
                                   "ln1_g", "ln1_b", "ln2_g", "ln2_b", "wt_qkv", "wt_out", "wt_fc", "wt_proj",
                                   "w_qkv_ln", "b_qkv_ln", "s_qkv_ln", "w_fc_ln", "b_fc_ln", "s_fc_ln",
                                   "wt_qkv_ln", "wt_fc_ln")]


class EbcVitWeights(ctypes.Structure):
    _fields_ = [("layers", ctypes.c_int), ("width", ctypes.c_int), ("heads", ctypes.c_int), ("patch", ctypes.c_int),
                ("num_vpt", ctypes.c_int)] + [(n, _VP) for n in ("w_patch", "cls", "pos", "ln_pre_g", "ln_pre_b",
                                                                 "ln_post_g", "ln_post_b")] + [("layer", ctypes.POINTER(EbcVitLayer))]


def _p(t: Tensor) -> int:
    return t.data_ptr()


class _EncoderCache:
    """Frozen encoder weights in the compute dtype (+ transposes for the dX backward), kept resident."""

    def __init__(self, enc: VisionTransformer, num_vpt: int, dtype: torch.dtype, device: torch.device,
                 ln_fold: bool = True):
        self.dtype, self.device = dtype, device
        keep: List[Tensor] = []

        def cvt(t: Tensor, dt=dtype) -> Tensor:
            r = t.detach().to(device=device, dtype=dt).contiguous()
            keep.append(r)
            return r

        layers = len(enc.transformer.resblocks)
        # ln_fold False keeps ln_1 / ln_2 as LayerNorm launches (tests, A/B measurements); f32 never folds
        fold_ln = dtype != torch.float32 and ln_fold
        self.layer_arr = (EbcVitLayer * layers)()
        for i, blk in enumerate(enc.transformer.resblocks):
            L = self.layer_arr[i]
            mats = {"qkv": blk.attn.in_proj_weight, "out": blk.attn.out_proj.weight,
                    "fc": blk.mlp.c_fc.weight, "proj": blk.mlp.c_proj.weight}
            for k, w in mats.items():
                setattr(L, "w_" + k, _p(cvt(w)))
                setattr(L, "wt_" + k, _p(cvt(w.detach().t())))
            L.b_qkv = _p(cvt(blk.attn.in_proj_bias, torch.float32))
            L.b_out = _p(cvt(blk.attn.out_proj.bias, torch.float32))
            L.b_fc = _p(cvt(blk.mlp.c_fc.bias, torch.float32))
            L.b_proj = _p(cvt(blk.mlp.c_proj.bias, torch.float32))
            L.ln1_g, L.ln1_b = _p(cvt(blk.ln_1.weight, torch.float32)), _p(cvt(blk.ln_1.bias, torch.float32))
            L.ln2_g, L.ln2_b = _p(cvt(blk.ln_2.weight, torch.float32)), _p(cvt(blk.ln_2.bias, torch.float32))
            if fold_ln:
                # ln_1 / ln_2 folded into the QKV / c_fc products (vit.hip): W' = W diag(gamma) in the compute dtype,
                # its row sums from the rounded W' (so the epilogue's mean term cancels what the MFMA sums), and
                # b' = b + W beta, in f64
                for pre, w, bias, ln in (("qkv", blk.attn.in_proj_weight, blk.attn.in_proj_bias, blk.ln_1),
                                         ("fc", blk.mlp.c_fc.weight, blk.mlp.c_fc.bias, blk.ln_2)):
                    w64 = w.detach().to(device, torch.float64)
                    wf = cvt(w64 * ln.weight.detach().to(device, torch.float64)[None, :])
                    setattr(L, f"w_{pre}_ln", _p(wf))
                    if pre == "fc":
                        # (W')^T for the backward's dX product: its epilogue then finishes ln_2's backward (vit.hip)
                        L.wt_fc_ln = _p(cvt(wf.t()))
                    setattr(L, f"s_{pre}_ln", _p(cvt(wf.double().sum(1), torch.float32)))
                    setattr(L, f"b_{pre}_ln", _p(cvt(bias.detach().to(device, torch.float64)
                                                     + w64 @ ln.bias.detach().to(device, torch.float64), torch.float32)))
        self.w_patch = cvt(enc.conv1.weight.reshape(WIDTH, -1))
        self.cls = cvt(enc.class_embedding, torch.float32)
        self.ln = [cvt(t, torch.float32) for t in (enc.ln_pre.weight, enc.ln_pre.bias, enc.ln_post.weight, enc.ln_post.bias)]
        self.enc, self.num_vpt, self.layers = enc, num_vpt, layers
        self.bwd_flags = 0              # EBC_VIT_BWD_FULL_LAYER0 (1): tests compare the trimmed layer-0 backward
        self.keep = keep
        self.structs: Dict[Tuple[int, int], Tuple[EbcVitWeights, Tensor]] = {}

    def weights(self, gh: int, gw: int) -> EbcVitWeights:
        if (gh, gw) not in self.structs:
            with torch.no_grad():
                pos = self.enc._interpolate_pos_embed(gh, gw).detach().to(self.device, torch.float32).contiguous()
            w = EbcVitWeights()
            w.layers, w.width, w.heads, w.patch, w.num_vpt = self.layers, WIDTH, HEADS, PATCH, self.num_vpt
            w.w_patch, w.cls, w.pos = _p(self.w_patch), _p(self.cls), _p(pos)
            w.ln_pre_g, w.ln_pre_b, w.ln_post_g, w.ln_post_b = (_p(t) for t in self.ln)
            w.layer = ctypes.cast(self.layer_arr, ctypes.POINTER(EbcVitLayer))
            self.structs[(gh, gw)] = (w, pos)
        return self.structs[(gh, gw)][0]


class _VitFn(torch.autograd.Function):
    """ebc_vit_forward / ebc_vit_backward: image -> ln_post(patch tokens) [B, G, 768] f32."""

    @staticmethod
    def forward(ctx, cache, image, vpt_bstride, training, *vpts):
        with _lib.on(image):
            return _VitFn._forward(ctx, cache, image, vpt_bstride, training, *vpts)

    @staticmethod
    def _forward(ctx, cache, image, vpt_bstride, training, *vpts):
        L = _lib.lib()
        B, _, H, W = image.shape
        gh, gw = H // PATCH, W // PATCH
        dt = _lib.dtype_code(cache.dtype)
        dev = image.device
        image = image.detach().float().contiguous()
        nbytes = L.ebc_vit_workspace_bytes(B, H, W, cache.layers, cache.num_vpt, dt, int(training))
        ws = torch.empty(nbytes, device=dev, dtype=torch.uint8)
        feat = torch.empty(B, gh * gw, WIDTH, device=dev, dtype=torch.float32)
        vp = [v.detach().float().contiguous() for v in vpts]
        arr = (_VP * cache.layers)(*([_p(v) for v in vp] + [None] * (cache.layers - len(vp))))
        w = cache.weights(gh, gw)
        rc = L.ebc_vit_forward(ctypes.byref(w), _lib.ptr(image), B, H, W, arr, vpt_bstride, dt, int(training),
                               _lib.ptr(ws), nbytes, _lib.ptr(feat), _lib.stream(dev))
        _lib.check(rc, "ebc_vit_forward")
        ctx.cache, ctx.ws, ctx.shape, ctx.bstride = cache, ws, (B, H, W), vpt_bstride
        ctx.vpt_shapes = [v.shape for v in vpts]
        ctx.vp_keep = vp
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        with _lib.on(dfeat):
            return _VitFn._backward(ctx, dfeat)

    @staticmethod
    def _backward(ctx, dfeat):
        L = _lib.lib()
        cache = ctx.cache
        B, H, W = ctx.shape
        dvpt = [torch.empty(s, device=dfeat.device, dtype=torch.float32) for s in ctx.vpt_shapes]
        arr = (_VP * cache.layers)(*([_p(v) for v in dvpt] + [None] * (cache.layers - len(dvpt))))
        w = cache.weights(H // PATCH, W // PATCH)
        rc = L.ebc_vit_backward(ctypes.byref(w), B, H, W, _lib.dtype_code(cache.dtype), _lib.ptr(ctx.ws), ctx.ws.numel(),
                                _lib.ptr(dfeat.float().contiguous()), arr, ctx.bstride, cache.bwd_flags, _lib.stream(dfeat))
        _lib.check(rc, "ebc_vit_backward")
        ctx.ws = None
        return (None, None, None, None) + tuple(dvpt)


class _HeadFn(torch.autograd.Function):
    """Projection (1x1 conv as MFMA GEMM) + similarity head (models/clip/model.py:198-217).

    `y` is the decoder output, NHWC [B,H,W,C] in the compute dtype when `nhwc` (the fused decoder's
    layout: the GEMM reads it in place), else NCHW; the input gradient comes back in the same layout."""

    @staticmethod
    def forward(ctx, y, weight, bias, logit_scale, text, anchors, cdtype, nhwc=False):
        with _lib.on(y):
            return _HeadFn._forward(ctx, y, weight, bias, logit_scale, text, anchors, cdtype, nhwc)

    @staticmethod
    def _forward(ctx, y, weight, bias, logit_scale, text, anchors, cdtype, nhwc):
        L = _lib.lib()
        st = _lib.stream(y)
        if nhwc:
            B, Hh, Ww, C = y.shape
        else:
            B, C, Hh, Ww = y.shape
        P, HW, NB = B * Hh * Ww, Hh * Ww, text.shape[0]
        dt = _lib.dtype_code(cdtype)
        if nhwc and y.dtype == cdtype and y.is_contiguous():
            Y = y.detach().reshape(P, C)
        else:
            Y = (y.detach() if nhwc else y.detach().permute(0, 2, 3, 1)).to(cdtype).reshape(P, C).contiguous()
        E = weight.shape[0]                                        # CLIP joint width: 512 / 1024 (RN50)
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            from .resnet import _prep_1x1
            Wc, Wt = _prep_1x1(L, weight, cdtype, st)              # [E, C] and [C, E], one launch
        else:
            Wc, Wt = weight.detach().reshape(E, C).to(cdtype).contiguous(), None
        bf = bias.detach().float().contiguous()
        Z = torch.empty(P, E, device=y.device, dtype=torch.float32)
        _lib.check(L.ebc_gemm(dt, 0, 1, _lib.ptr(Y), _lib.ptr(Wc), _lib.ptr(Z), _lib.ptr(bf), None, None,
                              P, E, C, st), "ebc_gemm(projection)")
        ls = logit_scale.detach().float().reshape(1).contiguous()
        logits = torch.empty(B, NB, Hh, Ww, device=y.device, dtype=torch.float32)
        expo = torch.empty(B, 1, Hh, Ww, device=y.device, dtype=torch.float32)
        _lib.check(L.ebc_head_fwd(_lib.EBC_F32, _lib.ptr(Z), _lib.ptr(text), _lib.ptr(ls), _lib.ptr(anchors),
                                  _lib.ptr(logits), _lib.ptr(expo), P, HW, NB, E, st), "ebc_head_fwd")
        ctx.save_for_backward(Y, Wc, Wt, Z, ls, text, anchors)
        ctx.meta = (B, C, Hh, Ww, cdtype, y.dtype, weight.shape, nhwc)
        return logits, expo

    @staticmethod
    def backward(ctx, dlogits, dexp):
        with _lib.on(ctx.saved_tensors[3]):
            return _HeadFn._backward(ctx, dlogits, dexp)

    @staticmethod
    def _backward(ctx, dlogits, dexp):
        L = _lib.lib()
        Y, Wc, Wt, Z, ls, text, anchors = ctx.saved_tensors
        st = _lib.stream(Z)
        B, C, Hh, Ww, cdtype, ydt, wshape, nhwc = ctx.meta
        P, HW, NB = B * Hh * Ww, Hh * Ww, text.shape[0]
        dev = Z.device
        dl = torch.zeros(B, NB, Hh, Ww, device=dev) if dlogits is None else dlogits.float().contiguous()
        de = torch.zeros(B, 1, Hh, Ww, device=dev) if dexp is None else dexp.float().contiguous()
        dt = _lib.dtype_code(cdtype)
        E = Wc.shape[0]
        dZ = torch.empty(P, E, device=dev, dtype=cdtype)
        dbs = torch.empty(E + 1, device=dev, dtype=torch.float32)     # dbias | dscale
        dbias, dscale = dbs[:E], dbs[E:]
        # per-block partial column sums, reduced in block order by a second launch (bit-reproducible)
        ws = _dec_workspace(dev, L.ebc_head_bwd_workspace_bytes(P, E), slot=3)
        _lib.check(L.ebc_head_bwd(_lib.EBC_F32, dt, _lib.ptr(Z), _lib.ptr(text), _lib.ptr(ls), _lib.ptr(anchors),
                                  _lib.ptr(dl), _lib.ptr(de), None, _lib.ptr(dZ), _lib.ptr(dbias), _lib.ptr(dscale),
                                  P, HW, NB, E, _lib.ptr(ws), ws.numel(), st), "ebc_head_bwd")
        if Wt is None:
            Wt = Wc.t().contiguous()                               # [C, E]
        dY = torch.empty(P, C, device=dev, dtype=cdtype)
        _lib.check(L.ebc_gemm(dt, 0, 0, _lib.ptr(dZ), _lib.ptr(Wt), _lib.ptr(dY), None, None, None,
                              P, C, E, st), "ebc_gemm(projection dX)")
        dW = _wgrad_rows(L, dZ, Y, cdtype, dev, st).reshape(wshape)
        dy = dY.view(B, Hh, Ww, C) if nhwc else dY.view(B, Hh, Ww, C).permute(0, 3, 1, 2).to(ydt)
        return dy, dW, dbias, dscale.reshape(()), None, None, None, None


# ----------------------------------------------------------------------------- decoder
_DEC_WS: Dict[Tuple[torch.device, int], Tensor] = {}


def _dec_workspace(dev: torch.device, nbytes: int, slot: int = 0) -> Tensor:
    """Scratch of the decoder calls on the caller's stream (slot 0: convolutions, slot 1: the weight-gradient
    GEMMs, slot 2: the projection's dW GEMM); its first 16 KiB (split-K counters) start zeroed and every kernel
    leaves them zero.  (The weight gradients on a side stream beside the data-gradient chain measured 2.7 %
    slower per step, r01: the data-gradient chain is the critical path.)"""
    ws = _DEC_WS.get((dev, slot))
    if ws is None or ws.numel() < nbytes:
        ws = torch.zeros(max(nbytes, 1 << 20), device=dev, dtype=torch.uint8)
        _DEC_WS[(dev, slot)] = ws
    return ws


def _wgrad_rows(L, dZ: Tensor, Y: Tensor, cdtype: torch.dtype, dev: torch.device, st) -> Tensor:
    """dW [E, C] f32 = dZ^T Y for row matrices dZ [P, E], Y [P, C] (a 1x1 conv's weight gradient over
    K = B*H*W pixels): both operands transposed to K-contiguous, then the split-K MFMA GEMM (K padded with
    zero columns to the GEMM's K step when P is not a multiple of it)."""
    dt = _lib.dtype_code(cdtype)
    P, E = dZ.shape
    C = Y.shape[1]
    kstep = 32 if cdtype == torch.float32 else 64
    Pp = -(-P // kstep) * kstep
    alloc = torch.empty if Pp == P else torch.zeros
    dZT = alloc(E, Pp, device=dev, dtype=cdtype)
    YT = alloc(C, Pp, device=dev, dtype=cdtype)
    _lib.check(L.ebc_transpose(dt, _lib.ptr(dZ), _lib.ptr(dZT), P, E, Pp, st), "ebc_transpose(dZ)")
    _lib.check(L.ebc_transpose(dt, _lib.ptr(Y), _lib.ptr(YT), P, C, Pp, st), "ebc_transpose(Y)")
    dW = torch.empty(E, C, device=dev, dtype=torch.float32)
    ws = _dec_workspace(dev, L.ebc_gemm_wgrad_workspace_bytes(dt, E, C, Pp), slot=2)
    _lib.check(L.ebc_gemm_wgrad(dt, _lib.ptr(dZT), _lib.ptr(YT), _lib.ptr(dW), E, C, Pp, _lib.ptr(ws), ws.numel(), st),
               "ebc_gemm_wgrad")
    return dW


def _bn_group(bn: nn.Module):
    """SyncBatchNorm (DDP, trainer.py:147): statistics are all-reduced over its process group."""
    if isinstance(bn, nn.SyncBatchNorm) and torch.distributed.is_available() and torch.distributed.is_initialized():
        pg = bn.process_group or torch.distributed.group.WORLD
        if torch.distributed.get_world_size(pg) > 1:
            return pg
    return None


def _bn_momentum(bn: nn.Module) -> float:
    """nn.BatchNorm2d's exponential_average_factor (momentum None: cumulative average)."""
    if bn.momentum is not None:
        return float(bn.momentum)
    return 1.0 / float(bn.num_batches_tracked.item())


class DecoderMaskTap:
    """Test hook on the decoder's two ReLU decisions (tests/test_gpu_ddp.py): while ``capture`` is a list, every
    _DecoderFn forward appends (m1, m2, pre1, pre2): its masks (relu(bn1) > 0 as [P, N], the block output > 0 as
    [B, H, W, N], bool) and the two pre-activations they were decided on (bn1(z1), bn2(z2) + x; f32, recomputed
    here by torch); while ``replay`` is a non-empty list, every backward pops one entry and uses its masks in place
    of its own (the backward kernels then take the given decisions).  Both None in normal use."""
    capture: Optional[list] = None
    replay: Optional[list] = None


class _DecoderFn(torch.autograd.Function):
    """BasicBlock(768, 768) (models/utils.py:254-303) after the x`up` bilinear reduction adapt
    (models/clip/model.py:195-196), on libebc_hip.so: implicit-GEMM 3x3 convs, BatchNorm statistics in
    the conv epilogue, fused BN/ReLU/residual kernels and the whole backward (ebc_dec_* / ebc_conv3x3_* /
    ebc_bn_* in include/ebc_hip.h).  feat [B,h,w,C] f32 (NHWC) -> y [B,H,W,C] in the compute dtype."""

    @staticmethod
    def forward(ctx, feat, w1, g1, b1, w2, g2, b2, blk, up, cdtype, training):
        with _lib.on(feat):
            return _DecoderFn._forward(ctx, feat, w1, g1, b1, w2, g2, b2, blk, up, cdtype, training)

    @staticmethod
    def _forward(ctx, feat, w1, g1, b1, w2, g2, b2, blk, up, cdtype, training):
        L = _lib.lib()
        feat = feat.detach().contiguous()
        B, h, w, C = feat.shape
        H, W, N = h * up, w * up, w1.shape[0]
        if N != C or w2.shape[0] != C or C % 64:
            raise NotImplementedError("fused decoder: BasicBlock(C, C) with C % 64 == 0 only")
        dev, dt, st = feat.device, _lib.dtype_code(cdtype), _lib.stream(feat)
        geo = (ctypes.c_long * 6)()
        _lib.check(L.ebc_dec_geometry(dt, B, H, W, C, geo), "ebc_dec_geometry")
        Q, Qs = geo[4], geo[5]
        P = B * H * W
        nbytes = L.ebc_dec_workspace_bytes(dt, B, H, W, C, N)
        ws = _dec_workspace(dev, nbytes)
        f32 = dict(device=dev, dtype=torch.float32)
        xpad = torch.empty(Q, C, device=dev, dtype=cdtype)
        _lib.check(L.ebc_dec_upsample_pad(dt, _lib.ptr(feat), _lib.ptr(xpad), B, h, w, C, up, st), "upsample_pad")
        outs, wflip = [], []
        inp = xpad
        bns = (blk.bn1, blk.bn2)
        for i, (wt, gm, bt) in enumerate(((w1, g1, b1), (w2, g2, b2))):
            bn = bns[i]
            wk = torch.empty(N, 3, 3, C, device=dev, dtype=cdtype)                 # [N][3][3][C]
            wf = torch.empty(C, 3, 3, N, device=dev, dtype=cdtype)                 # [C][3][3][N], flipped
            _lib.check(L.ebc_dec_prep_weights(dt, _lib.ptr(wt.detach().float().contiguous()), _lib.ptr(wk),
                                              _lib.ptr(wf), N, C, st), "ebc_dec_prep_weights")
            wflip.append(wf)
            z = torch.empty(P, N, device=dev, dtype=cdtype)
            use_batch = training or not bn.track_running_stats
            pg = _bn_group(bn) if use_batch else None
            # SyncBatchNorm: [sum | sum of squares | this rank's count] all-reduced in ONE f64 buffer, the total
            # count read on device (count = -1), so ranks may hold different batch sizes (torch.nn.SyncBatchNorm
            # gathers the per-rank counts the same way)
            colsum = torch.empty(2 * N + (pg is not None), device=dev, dtype=torch.float64) if use_batch else None
            fused_bn = use_batch and pg is None and training and bn.track_running_stats and bn.momentum is not None
            if not fused_bn:
                _lib.check(L.ebc_conv3x3_fwd(dt, _lib.ptr(inp), _lib.ptr(wk), _lib.ptr(z), _lib.ptr(colsum), None, None,
                                             _lib.ptr(ws), ws.numel(), B, H, W, C, N, st), "ebc_conv3x3_fwd")
            count = float(P)
            if pg is not None:
                colsum[2 * N].fill_(float(P))
                torch.distributed.all_reduce(colsum, group=pg)
                count = -1.0
            mean, rstd, scale, shift = (torch.empty(N, **f32) for _ in range(4))
            upd = use_batch and training and bn.track_running_stats
            nbt = None                             # num_batches_tracked += 1 inside the finalize launch
            if upd:
                if bn.momentum is None:            # cumulative average: the factor needs the updated count now
                    bn.num_batches_tracked.add_(1)
                else:
                    nbt = _lib.ptr(bn.num_batches_tracked)
            mom = _bn_momentum(bn) if upd else 0.0
            if fused_bn:
                # no SyncBatchNorm exchange: the conv, then its column sums reduced and finalized in one launch
                _lib.check(L.ebc_conv3x3_fwd_bn(dt, _lib.ptr(inp), _lib.ptr(wk), _lib.ptr(z), _lib.ptr(ws), ws.numel(),
                                                B, H, W, C, N, float(bn.eps), mom, _lib.ptr(gm.detach()),
                                                _lib.ptr(bt.detach()), _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(scale),
                                                _lib.ptr(shift), _lib.ptr(bn.running_mean), _lib.ptr(bn.running_var),
                                                nbt, _lib.ptr(colsum), st), "ebc_conv3x3_fwd_bn")
            else:
                _lib.check(L.ebc_bn_finalize(_lib.ptr(colsum), count, float(bn.eps), mom, _lib.ptr(gm.detach()),
                                             _lib.ptr(bt.detach()), _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(scale),
                                             _lib.ptr(shift), _lib.ptr(bn.running_mean) if (upd or not use_batch) else None,
                                             _lib.ptr(bn.running_var) if (upd or not use_batch) else None, nbt, N, st),
                           "ebc_bn_finalize")
            outs.append((z, mean, rstd, scale, shift, count, pg, colsum))
            if i == 0:
                hpad = torch.empty(Q, N, device=dev, dtype=cdtype)
                _lib.check(L.ebc_bn_relu_pad(dt, _lib.ptr(z), _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(hpad),
                                             B, H, W, N, st), "ebc_bn_relu_pad")
                inp = hpad
        z2, _, _, scale2, shift2, _, _, _ = outs[1]
        y = torch.empty(B, H, W, N, device=dev, dtype=cdtype)
        _lib.check(L.ebc_bn_add_relu(dt, _lib.ptr(z2), _lib.ptr(scale2), _lib.ptr(shift2), _lib.ptr(feat), up,
                                     _lib.ptr(y), B, H, W, N, st), "ebc_bn_add_relu")
        if DecoderMaskTap.capture is not None:
            Hp, Wp = geo[0], geo[1]
            h1 = hpad.view(B, Hp, Wp, N)[:, 1:H + 1, 1:W + 1]
            (z1, _, _, sc1, sh1), (z2, _, _, sc2, sh2) = (o[:5] for o in outs)
            xu = xpad.view(B, Hp, Wp, C)[:, 1:H + 1, 1:W + 1].float().reshape(P, N)
            DecoderMaskTap.capture.append(((h1 > 0).reshape(P, N), y > 0, z1.float() * sc1 + sh1,
                                           (z2.float() * sc2 + sh2 + xu).view(B, H, W, N)))
        ctx.save_for_backward(xpad, hpad, y, wflip[0], g1, wflip[1], g2)
        from .resnet import flush_bn_counters
        flush_bn_counters()                        # both BatchNorms' num_batches_tracked in one launch
        ctx.outs = outs
        ctx.meta = (B, h, w, H, W, C, N, up, cdtype, Q, Qs, P)
        return y

    @staticmethod
    def backward(ctx, gy):
        with _lib.on(gy):
            return _DecoderFn._backward(ctx, gy)

    @staticmethod
    def _backward(ctx, gy):
        L = _lib.lib()
        xpad, hpad, y, wf1, g1, wf2, g2 = ctx.saved_tensors
        B, h, w, H, W, C, N, up, cdtype, Q, Qs, P = ctx.meta
        dev, dt, st = y.device, _lib.dtype_code(cdtype), _lib.stream(y)
        gy = gy.to(cdtype).contiguous()
        nbytes = L.ebc_dec_workspace_bytes(dt, B, H, W, C, N)
        ws = _dec_workspace(dev, nbytes)
        ws_w = _dec_workspace(dev, nbytes, 1)
        f32 = dict(device=dev, dtype=torch.float32)
        grads = []
        dnext = gy                                    # gradient at the current BN output's ReLU
        mask = y                                      # ReLU mask source (None: recompute from z)
        ymask, mask1 = y, None
        if DecoderMaskTap.replay:
            m1, m2 = DecoderMaskTap.replay.pop(0)[:2]
            mask1 = m1.to(cdtype).reshape(P, N).contiguous()
            mask = ymask = m2.to(cdtype).reshape(B, H, W, N).contiguous()
        for i in (1, 0):
            z, mean, rstd, scale, shift, count, pg, colsum = ctx.outs[i]
            gm = (g1, g2)[i]
            dg, db, coef = torch.empty(N, **f32), torch.empty(N, **f32), torch.empty(3, N, **f32)
            fused = pg is None and count == float(P)
            if fused:
                # no exchange: column sums and finalize in one launch (ebc_bn_bwd_reduce_finalize, count = P)
                _lib.check(L.ebc_bn_bwd_reduce_finalize(dt, _lib.ptr(dnext), _lib.ptr(mask), _lib.ptr(z), _lib.ptr(mean),
                                                        _lib.ptr(rstd), _lib.ptr(scale), _lib.ptr(shift),
                                                        _lib.ptr(gm.detach()), _lib.ptr(dg), _lib.ptr(db), _lib.ptr(coef),
                                                        _lib.ptr(ws), ws.numel(), P, N, st), "ebc_bn_bwd_reduce_finalize")
            else:
                sums = torch.empty(2 * N + (pg is not None), device=dev, dtype=torch.float64)
                _lib.check(L.ebc_bn_bwd_reduce(dt, _lib.ptr(dnext), _lib.ptr(mask), _lib.ptr(z), _lib.ptr(mean),
                                               _lib.ptr(rstd), _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(sums),
                                               _lib.ptr(ws), ws.numel(), P, N, st), "ebc_bn_bwd_reduce")
            if not fused and pg is not None:
                # SyncBatchNorm backward (torch nn/modules/_functions.py, C5): d gamma / d beta come from THIS
                # rank's sums (DDP then averages them over the ranks); the input gradient uses the all-reduced
                # sums and the all-reduced count
                _lib.check(L.ebc_bn_bwd_finalize(_lib.ptr(sums), float(P), _lib.ptr(gm.detach()), _lib.ptr(rstd),
                                                 _lib.ptr(dg), _lib.ptr(db), _lib.ptr(coef), N, st), "ebc_bn_bwd_finalize")
                torch.distributed.all_reduce(sums[: 2 * N], group=pg)     # sum_dy, sum_dy_xmu
                sums[2 * N:].copy_(colsum[2 * N:])                          # the forward's all-reduced count
                _lib.check(L.ebc_bn_bwd_finalize(_lib.ptr(sums), count, _lib.ptr(gm.detach()), _lib.ptr(rstd),
                                                 None, None, _lib.ptr(coef), N, st), "ebc_bn_bwd_finalize(sync)")
            elif not fused:
                _lib.check(L.ebc_bn_bwd_finalize(_lib.ptr(sums), count, _lib.ptr(gm.detach()), _lib.ptr(rstd),
                                                 _lib.ptr(dg), _lib.ptr(db), _lib.ptr(coef), N, st), "ebc_bn_bwd_finalize")
            if colsum is None:                            # running statistics (eval mode): dz = gamma * rstd * g
                coef[1:].zero_()
            dzpad = torch.empty(Q, N, device=dev, dtype=cdtype)
            dzT = torch.empty(N, Qs, device=dev, dtype=cdtype)
            _lib.check(L.ebc_bn_bwd_apply(dt, _lib.ptr(dnext), _lib.ptr(mask), _lib.ptr(z), _lib.ptr(mean),
                                          _lib.ptr(rstd), _lib.ptr(scale), _lib.ptr(shift), _lib.ptr(coef),
                                          _lib.ptr(dzpad), _lib.ptr(dzT), B, H, W, N, st), "ebc_bn_bwd_apply")
            src = hpad if i == 1 else xpad                # the conv's input image
            xT3 = torch.empty(3, C, Qs, device=dev, dtype=cdtype)
            _lib.check(L.ebc_dec_transpose3(dt, _lib.ptr(src), _lib.ptr(xT3), B, H, W, C, st), "ebc_dec_transpose3")
            dw = torch.empty(N, C, 3, 3, **f32)
            _lib.check(L.ebc_conv3x3_wgrad(dt, _lib.ptr(dzT), _lib.ptr(xT3), _lib.ptr(dw), _lib.ptr(ws_w),
                                           ws_w.numel(), B, H, W, C, N, st), "ebc_conv3x3_wgrad")
            del xT3, dzT
            wf = (wf1, wf2)[i]                                                    # [C][3][3][N]
            dx = torch.empty(P, C, device=dev, dtype=cdtype)
            # conv1's data gradient also takes the residual branch's gradient (gy through the final ReLU)
            add = (_lib.ptr(gy), _lib.ptr(ymask)) if i == 0 else (None, None)
            _lib.check(L.ebc_conv3x3_fwd(dt, _lib.ptr(dzpad), _lib.ptr(wf), _lib.ptr(dx), None, *add, _lib.ptr(ws),
                                         ws.numel(), B, H, W, N, C, st), "ebc_conv3x3_fwd(dgrad)")
            grads.append((dw, dg, db))
            dnext, mask = dx, mask1
        dfeat = torch.empty(B, h, w, C, **f32)
        _lib.check(L.ebc_dec_upsample_bwd(dt, _lib.ptr(dnext), _lib.ptr(dfeat), B, h, w, C, up, st),
                   "ebc_dec_upsample_bwd")
        (dw2, dg2, db2), (dw1, dg1, db1) = grads
        ctx.outs = None
        return dfeat, dw1, dg1, db1, dw2, dg2, db2, None, None, None, None


# ----------------------------------------------------------------------------- model
resnet_backbones = ["resnet50", "resnet101", "resnet50x4", "resnet50x16", "resnet50x64"]
vit_backbones = ["vit_b_16"]


class CLIP_EBC(nn.Module):
    """models/clip/model.py:30-217 for the vit_b_16 (deep VPT, frozen encoder) and resnet50 (trainable
    ModifiedResNet, Bottleneck decoder; ebc_amd/resnet.py) backbones."""

    def __init__(self, backbone: str, bins: List[Tuple[float, float]], anchor_points: List[float],
                 reduction: Optional[int] = None, freeze_text_encoder: bool = True, prompt_type: str = "number",
                 input_size: Optional[int] = None, num_vpt: Optional[int] = None, deep_vpt: Optional[bool] = None,
                 vpt_drop: Optional[float] = None, decoder_cfg: Optional[List[int]] = None, vit_layers: int = 12,
                 text_layers: int = 12, text_features: Optional[Tensor] = None, weights_seed: Optional[int] = None,
                 **kwargs: Any) -> None:
        super().__init__()
        if backbone not in vit_backbones + ["resnet50"]:
            raise NotImplementedError(f"backbone {backbone!r}: vit_b_16 and resnet50 are on the MI355X path (SURVEY.md §8)")
        self.backbone = backbone
        if backbone == "resnet50":
            from .resnet import Bottleneck, ModifiedResNet
            from .synthetic import RN50_CHANNELS, RN50_EMBED
            # models/clip/model.py:51-52 (trainable encoder), :83-95 (decoder cfg [2048] + projection)
            self.image_encoder = ModifiedResNet(reduction=reduction).to(memory_format=torch.channels_last)
            self.encoder_reduction = self.image_encoder.reduction
            self.reduction = self.encoder_reduction if reduction is None else reduction
            decoder_cfg = decoder_cfg or [RN50_CHANNELS]
            if list(decoder_cfg) != [RN50_CHANNELS]:
                raise NotImplementedError("resnet50 decoder is Bottleneck [2048] (models/clip/model.py:237-238)")
            if self.encoder_reduction % self.reduction or self.encoder_reduction // self.reduction not in (1, 2):
                raise NotImplementedError("resnet50: reduction must give a x1 / x2 bilinear adapt")
            self.image_decoder = nn.Sequential(Bottleneck(RN50_CHANNELS, RN50_CHANNELS, expansion=1))
            embed = RN50_EMBED
        else:
            assert input_size is not None, "Expected input_size to be an integer, got None."
            assert num_vpt is not None, "Expected num_vpt to be an integer, got None."
            assert deep_vpt is not None, "Expected deep_vpt to be a boolean, got None."
            assert vpt_drop is not None, "Expected vpt_drop to be a float, got None."
            self.image_encoder = VisionTransformer(input_size, PATCH, EMBED, WIDTH, vit_layers, HEADS)
            self.image_encoder_depth = vit_layers
            for p in self.image_encoder.parameters():
                p.requires_grad = False
            self.num_vpt, self.deep_vpt, self.vpt_drop = num_vpt, deep_vpt, vpt_drop
            _check_tokens(input_size, input_size, num_vpt)
            val = math.sqrt(6.0 / float(3 * PATCH + WIDTH))
            for idx in range(vit_layers if deep_vpt else 1):
                setattr(self, f"vpt_{idx}", nn.Parameter(torch.empty(num_vpt, WIDTH).uniform_(-val, val)))
            self.encoder_reduction = PATCH
            self.reduction = self.encoder_reduction if reduction is None else reduction
            decoder_cfg = decoder_cfg or [WIDTH]
            if list(decoder_cfg) != [WIDTH]:
                raise NotImplementedError("vit_b_16 decoder is BasicBlock [768] (models/clip/model.py:250-251)")
            if reduction is not None and (PATCH % reduction or PATCH // reduction not in (1, 2)):
                raise NotImplementedError("reduction must be 16 or 8 for vit_b_16 (x1 / x2 bilinear adapt)")
            self.image_decoder = nn.Sequential(BasicBlock(WIDTH, WIDTH))
            embed = EMBED
        self.channels, self.clip_embed_dim = decoder_cfg[-1], embed
        self.projection = nn.Conv2d(self.channels, embed, kernel_size=1)
        self.prompt_type = prompt_type
        self.text_encoder = CLIPTextEncoder(embed, 77, 49408, 512, 8, text_layers)
        self.freeze_text_encoder = freeze_text_encoder
        for p in self.text_encoder.parameters():
            p.requires_grad = False
        self.bins = bins
        self.anchor_points = torch.tensor(anchor_points, dtype=torch.float32, requires_grad=False).view(1, -1, 1, 1)
        self.logit_scale = nn.Parameter(torch.ones([]) * np.log(1 / 0.07), requires_grad=True)
        pb = [b[0] if b[0] == b[1] else b for b in self.bins]
        self.text_prompts = [format_count(b, self.prompt_type) for b in pb]
        if weights_seed is not None:
            self._load_synthetic(weights_seed, vit_layers, text_layers, input_size)
        self._given_text = text_features
        self.register_buffer("text_features", torch.zeros(len(bins), embed), persistent=False)
        self.register_buffer("_anchors", self.anchor_points.reshape(-1).clone(), persistent=False)
        self._refresh_text()
        self._cache: Optional[_EncoderCache] = None
        self._cache_key = None
        self.vit_bwd_flags = 0          # ebc_vit_backward flags (include/ebc_hip.h), for parity tests only
        self.vit_ln_fold = True         # 16-bit: ln_1 / ln_2 folded into the QKV / c_fc products (vit.hip)

    # -- weights ---------------------------------------------------------------------------
    def _load_synthetic(self, seed, vit_layers, text_layers, input_size):
        if self.backbone == "resnet50":
            sd = synthetic.resnet50_full_state(seed, text_layers=text_layers)
        else:
            sd = synthetic.full_state(seed, layers=vit_layers, text_layers=text_layers, input_size=input_size)
        own = self.state_dict()
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items() if k in own}
        self.load_state_dict(sd, strict=False)

    def _refresh_text(self):
        if getattr(self, "_given_text", None) is not None:
            tf = torch.as_tensor(self._given_text, dtype=torch.float32)
        else:
            tf = self.text_encoder(prompt_tokens(self.text_prompts).to(self.text_encoder.positional_embedding.device)).float()
        with torch.no_grad():
            self.text_features.copy_(tf.to(self.text_features.device))

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        res = super().load_state_dict(state_dict, strict=strict, assign=assign)
        if hasattr(self, "text_features"):
            self._refresh_text()
        self._cache = None
        return res

    def _apply(self, fn, recurse=True):
        self._cache = None
        return super()._apply(fn, recurse)

    def _encoder_cache(self, dtype: torch.dtype, device: torch.device) -> _EncoderCache:
        ver = sum(p._version for p in self.image_encoder.parameters())
        key = (dtype, device, ver, bool(self.vit_ln_fold))
        if self._cache is None or self._cache_key != key:
            self._cache = _EncoderCache(self.image_encoder, self.num_vpt, dtype, device, bool(self.vit_ln_fold))
            self._cache_key = key
        self._cache.bwd_flags = int(self.vit_bwd_flags)
        return self._cache

    # -- forward ---------------------------------------------------------------------------
    def _compute_dtype(self, x: Tensor) -> torch.dtype:
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            return torch.get_autocast_dtype("cuda")
        return torch.float32

    def _prepare_vpts(self, B: int) -> Tuple[List[Tensor], int]:
        n = self.image_encoder_depth if self.deep_vpt else 1
        vpts = [getattr(self, f"vpt_{i}") for i in range(n)]
        if self.training and self.vpt_drop and self.vpt_drop > 0:          # model.py:131-140 (per-crop dropout)
            vpts = [F.dropout(v.unsqueeze(0).expand(B, -1, -1), self.vpt_drop, True).contiguous() for v in vpts]
            return vpts, self.num_vpt * WIDTH
        return vpts, 0

    def _forward_vpt_nhwc(self, x: Tensor) -> Tensor:
        """[B,3,H,W] -> ln_post patch tokens [B,H/16,W/16,768] f32 (NHWC), models/clip/model.py:142-189."""
        B, _, H, W = x.shape
        cache = self._encoder_cache(self._compute_dtype(x), x.device)
        vpts, bstride = self._prepare_vpts(B)
        training = torch.is_grad_enabled() and any(v.requires_grad for v in vpts)
        with torch.autocast("cuda", enabled=False):
            feat = _VitFn.apply(cache, x, bstride, training, *vpts)
        return feat.view(B, H // PATCH, W // PATCH, WIDTH)

    def _forward_vpt(self, x: Tensor) -> Tensor:
        """[B,3,H,W] -> [B,768,H/16,W/16] (channels_last memory), models/clip/model.py:142-189."""
        return self._forward_vpt_nhwc(x).permute(0, 3, 1, 2)

    def _forward_resnet(self, x: Tensor, cdt: torch.dtype) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        """models/clip/model.py:191-217 for the resnet50 backbone: the trainable ModifiedResNet (stem on PyTorch-ROCm,
        its 16 Bottlenecks on HIP), then the HIP Bottleneck decoder and head."""
        from .resnet import _BottleneckFn, encoder_forward, flush_bn_counters
        feat = encoder_forward(self.image_encoder, x, cdt, self.training)   # stem on MIOpen, 16 blocks on HIP
        feat = feat.float().contiguous()                                     # NHWC rows, f32
        up = self.encoder_reduction // self.reduction
        blk = self.image_decoder[0]
        with torch.autocast("cuda", enabled=False):
            y = _BottleneckFn.apply(feat, blk.conv1.weight, blk.conv2.weight, blk.conv3.weight, blk.bn1.weight,
                                    blk.bn1.bias, blk.bn2.weight, blk.bn2.bias, blk.bn3.weight, blk.bn3.bias, blk, up,
                                    cdt, self.training)
            logits, exp = _HeadFn.apply(y, self.projection.weight, self.projection.bias, self.logit_scale,
                                        self.text_features, self._anchors, cdt, True)
        flush_bn_counters()
        return (logits, exp) if self.training else exp

    def forward(self, x: Tensor) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        if not x.is_cuda:
            raise RuntimeError("ebc_amd.CLIP_EBC runs on the MI355X HIP path only (input is on the CPU)")
        cdt = self._compute_dtype(x)
        if self.backbone == "resnet50":
            return self._forward_resnet(x, cdt)
        _check_tokens(x.shape[-2], x.shape[-1], self.num_vpt)
        feat = self._forward_vpt_nhwc(x)
        up = self.encoder_reduction // self.reduction                      # model.py:195-196 (x2 for reduction 8)
        blk = self.image_decoder[0]
        with torch.autocast("cuda", enabled=False):
            y = _DecoderFn.apply(feat, blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight,
                                 blk.bn2.weight, blk.bn2.bias, blk, up, cdt, self.training)
            logits, exp = _HeadFn.apply(y, self.projection.weight, self.projection.bias, self.logit_scale,
                                        self.text_features, self._anchors, cdt, True)
        return (logits, exp) if self.training else exp


def _clip_ebc(backbone: str, bins, anchor_points, reduction=None, freeze_text_encoder=True, prompt_type="number",
              input_size=None, num_vpt=None, deep_vpt=None, vpt_drop=None, decoder_block=None, decoder_cfg=None,
              **kw) -> CLIP_EBC:
    """models/clip/model.py:220-270 (vit_b_16: BasicBlock decoder [768]; resnet50: Bottleneck decoder [2048])."""
    return CLIP_EBC(backbone, bins, anchor_points, reduction=reduction, freeze_text_encoder=freeze_text_encoder,
                    prompt_type=prompt_type, input_size=input_size, num_vpt=num_vpt, deep_vpt=deep_vpt,
                    vpt_drop=vpt_drop, decoder_cfg=decoder_cfg, **kw)


MAX_TOKENS = 16384    # attention.hip L_MAX (sequences past 256 tokens stream K / V through LDS in chunks)


def _check_tokens(h: int, w: int, num_vpt: int) -> None:
    """The ViT sequence (CLS + prompts + (h/16)(w/16) patches) must fit the attention kernels' bound."""
    tokens = 1 + num_vpt + (h // PATCH) * (w // PATCH)
    if tokens > MAX_TOKENS:
        raise NotImplementedError(
            f"clip_vit_b_16 on {h}x{w} inputs with {num_vpt} prompts is a sequence of {tokens} tokens; the HIP attention "
            f"kernels take up to {MAX_TOKENS} tokens")


def get_model(backbone: str, input_size: int, reduction: int, bins: Optional[List[Tuple[float, float]]] = None,
              anchor_points: Optional[List[float]] = None, **kwargs: Any) -> nn.Module:
    """models/__init__.py:10-44.  clip_vit_b_16 and clip_resnet50 are on the MI355X path; vgg19_ae (configs[0]) is
    the reference's DM-Count VGG-19 encoder-decoder (ebc_amd/vgg.py)."""
    backbone = backbone.lower()
    if "clip" not in backbone:
        from . import vgg                     # BASELINE configs[0]: vgg19_ae (models/model.py:94-111)
        return vgg.build(backbone, input_size, reduction, bins, anchor_points, **kwargs)
    backbone = backbone[5:]
    assert bins is not None and anchor_points is not None, "CLIP-EBC needs bins and anchor_points"
    kwargs.setdefault("prompt_type", "number")
    kwargs.setdefault("num_vpt", 32)
    kwargs.setdefault("vpt_drop", 0.0)
    kwargs.setdefault("deep_vpt", True)
    return _clip_ebc(backbone=backbone, input_size=input_size, reduction=reduction, bins=bins,
                     anchor_points=anchor_points, **kwargs)

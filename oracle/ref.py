"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

torch-fp32 CPU restatement of the CLIP-EBC ViT-B/16 + deep-VPT training step.
Each function cites the reference lines it restates.
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def oracle_lib() -> ctypes.CDLL:
    """The compiled C restatement (built by `make -C oracle` / __graft_entry__.build())."""
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle_sinkhorn.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", HERE])
        lib = ctypes.CDLL(path)
        f = lib.oracle_ot_crop
        fp = ctypes.POINTER(ctypes.c_float)
        dp = ctypes.POINTER(ctypes.c_double)
        f.argtypes = [fp, ctypes.c_int, fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                      ctypes.c_float, ctypes.c_int, fp, fp, fp, fp, ctypes.POINTER(ctypes.c_int), fp, dp, dp, dp]
        f.restype = ctypes.c_int
        s = lib.oracle_sinkhorn
        s.argtypes = [fp, fp, fp, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_float,
                      ctypes.c_int, ctypes.c_int, fp, fp, fp, fp, fp, fp, ctypes.POINTER(ctypes.c_int)]
        s.restype = ctypes.c_int
        _LIB = lib
    return _LIB


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def ot_crop(points: np.ndarray, pred_density: np.ndarray, size: int, reduction: int = 8, reg: float = 10.0,
            max_iter: int = 100, stop_thr: float = 1e-9, eval_freq: int = 10, norm_cood: bool = False) -> Dict[str, np.ndarray]:
    """One crop of OTLoss.forward (losses/dm_loss.py:49-77) + sinkhorn (bregman_pytorch.py:11-144)."""
    lib = oracle_lib()
    g = size // reduction
    M = g * g
    n = len(points)
    pts = np.ascontiguousarray(points, np.float32).reshape(-1)
    pd = np.ascontiguousarray(pred_density, np.float32).reshape(-1)
    assert pd.size == M
    beta = np.zeros(M, np.float32); v = np.zeros(M, np.float32); grad = np.zeros(M, np.float32)
    u = np.zeros(max(n, 1), np.float32); err = np.full(max_iter // eval_freq + 1, -1.0, np.float32)
    ne = ctypes.c_int(0); wd = ctypes.c_double(0); obj = ctypes.c_double(0); loss = ctypes.c_double(0)
    it = lib.oracle_ot_crop(_fp(pts), n, _fp(pd), size, reduction, int(norm_cood), reg, max_iter, stop_thr, eval_freq,
                            _fp(beta), _fp(u), _fp(v), _fp(err), ctypes.byref(ne), _fp(grad),
                            ctypes.byref(wd), ctypes.byref(obj), ctypes.byref(loss))
    return dict(beta=beta, u=u[:n], v=v, err=err[:ne.value], ot_grad=grad, wd=wd.value, ot_obj=obj.value,
                loss=loss.value, iters=abs(it), rolled_back=it < 0)



def sinkhorn(a: np.ndarray, b: np.ndarray, C: np.ndarray, reg: float, max_iter: int, stop_thr: float = 1e-9,
             eval_freq: int = 10, log: bool = True) -> Dict[str, np.ndarray]:
    """bregman_pytorch.py:11-144 on a general dense cost (the C restatement)."""
    lib = oracle_lib()
    na, nb = C.shape
    a = np.ascontiguousarray(a, np.float32); b = np.ascontiguousarray(b, np.float32)
    C = np.ascontiguousarray(C, np.float32)
    P = np.zeros((na, nb), np.float32); u = np.zeros(na, np.float32); v = np.zeros(nb, np.float32)
    alpha = np.zeros(na, np.float32); beta = np.zeros(nb, np.float32)
    err = np.zeros(max(1, -(-max_iter // eval_freq)), np.float32); ne = ctypes.c_int(0)
    it = lib.oracle_sinkhorn(_fp(a), _fp(b), _fp(C), na, nb, reg, max_iter, stop_thr, eval_freq, int(log), _fp(P),
                             _fp(u), _fp(v), _fp(alpha), _fp(beta), _fp(err), ctypes.byref(ne))
    return dict(P=P, u=u, v=v, alpha=alpha, beta=beta, err=err[:ne.value], iters=abs(it), rolled_back=it < 0,
                roll=-it if it < 0 else 0)

# ----------------------------------------------------------------------------- loss
def reshape_density(d: torch.Tensor, r: int) -> torch.Tensor:
    """losses/utils.py:4-9 — r x r block sums."""
    B, _, H, W = d.shape
    return d.reshape(B, 1, H // r, r, W // r, r).sum(dim=(-1, -3))


def bin_count(density: torch.Tensor, bins: Sequence[Tuple[float, float]]) -> torch.Tensor:
    """losses/dace_loss.py:42-47 — inclusive bins, later bins win."""
    cls = torch.zeros_like(density, dtype=torch.long)
    for idx, (lo, hi) in enumerate(bins):
        cls[(density >= lo) & (density <= hi)] = idx
    return cls.squeeze(1)


class _OTGrad(torch.autograd.Function):
    """loss = sum(pred * grad.detach()) (dm_loss.py:76): its gradient w.r.t. pred is the OT gradient."""
    @staticmethod
    def forward(ctx, pred, grad):
        ctx.save_for_backward(grad)
        return (pred * grad).sum().reshape(1)

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return g * grad, None


def dace_loss(pred_class: torch.Tensor, pred_density: torch.Tensor, target_density: torch.Tensor,
              points: List[np.ndarray], bins, reduction: int = 8, input_size: int = 224,
              weight_count_loss: float = 1.0, weight_ot: float = 0.1, weight_tv: float = 0.01,
              norm_cood: bool = False):
    """DACELoss(count_loss='dmcount').forward — dace_loss.py:49-70 with DMLoss dm_loss.py:99-124."""
    if target_density.shape[-2:] != pred_density.shape[-2:]:
        target_density = reshape_density(target_density, reduction)
    target_class = bin_count(target_density, bins)
    ce = F.cross_entropy(pred_class, target_class, reduction="none").sum(dim=(-1, -2)).mean()
    B = pred_density.shape[0]
    pred_count = pred_density.view(B, -1).sum(dim=1)
    normed_pred = pred_density / (pred_count.view(-1, 1, 1, 1) + 1e-8)
    dev = pred_density.device                     # the oracle also runs on the GPU (AMP calibration, tests only)
    target_count = torch.tensor([len(p) for p in points], dtype=torch.float32, device=dev)
    normed_target = target_density / (target_count.view(-1, 1, 1, 1) + 1e-8)
    grads = np.zeros((B,) + tuple(pred_density.shape[1:]), np.float32)
    pdn = pred_density.detach().cpu().numpy()
    for b, p in enumerate(points):
        if len(p) > 0:
            grads[b] = ot_crop(p, pdn[b, 0], input_size, reduction, norm_cood=norm_cood)["ot_grad"].reshape(pdn.shape[1:])
    ot_loss = _OTGrad.apply(pred_density, torch.from_numpy(grads).to(dev))
    tv = ((normed_pred - normed_target).abs().sum(dim=(1, 2, 3)) * target_count).mean()
    cnt = (pred_count - target_count).abs().mean()
    dm = ot_loss * weight_ot + tv * weight_tv + cnt
    loss = ce + weight_count_loss * dm
    info = {"loss": loss.detach(), "ot_loss": ot_loss.detach(), "tv_loss": tv.detach(),
            "count_loss": cnt.detach(), "ce_loss": ce.detach()}
    return loss, info


# ----------------------------------------------------------------------------- model
def layer_norm(x, w, b):
    """blocks.py:8-14 — LayerNorm in fp32, eps 1e-5."""
    return F.layer_norm(x if x.dtype == torch.float64 else x.float(), (x.shape[-1],), w, b, 1e-5)


def block(x, p, pre, heads=12):
    """ResidualAttentionBlock.forward (blocks.py:39-42); x is [B, L, D] (batch-first here)."""
    B, L, D = x.shape
    h = layer_norm(x, p[pre + "ln_1.weight"], p[pre + "ln_1.bias"])
    qkv = F.linear(h, p[pre + "attn.in_proj_weight"], p[pre + "attn.in_proj_bias"])
    q, k, v = qkv.split(D, dim=-1)
    hd = D // heads
    q = q.view(B, L, heads, hd).transpose(1, 2)
    k = k.view(B, L, heads, hd).transpose(1, 2)
    v = v.view(B, L, heads, hd).transpose(1, 2)
    s = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(hd)
    o = torch.matmul(s.softmax(-1), v).transpose(1, 2).reshape(B, L, D)
    x = x + F.linear(o, p[pre + "attn.out_proj.weight"], p[pre + "attn.out_proj.bias"])
    h = layer_norm(x, p[pre + "ln_2.weight"], p[pre + "ln_2.bias"])
    a = F.linear(h, p[pre + "mlp.c_fc.weight"], p[pre + "mlp.c_fc.bias"])
    a = a * torch.sigmoid(1.702 * a)                                  # QuickGELU blocks.py:17-19
    return x + F.linear(a, p[pre + "mlp.c_proj.weight"], p[pre + "mlp.c_proj.bias"])


def vit_vpt_forward(p: Dict[str, torch.Tensor], x: torch.Tensor, layers: int, num_vpt: int = 32,
                    deep_vpt: bool = True, vpt_masks: Optional[List[torch.Tensor]] = None) -> torch.Tensor:
    """CLIP_EBC._forward_vpt (models/clip/model.py:142-189): deep VPT (vpt_l inserted before block l) or
    shallow (vpt_0 before block 0, then each block's output prompt rows carried into the next, model.py:174-178).

    vpt_masks (vpt_drop > 0, training): _prepare_vpt (model.py:131-140) expands vpt_l to [B, num_vpt, 768] and
    passes it through its own nn.Dropout `vpt_drop_l` (model.py:76,137); vpt_masks[l] is that dropout's per-element
    multiplier (0 or 1/(1-p), [B, num_vpt, 768]) -- applied to the expanded prompt of every layer that prepares one
    (all layers deep; layer 0 only shallow)."""
    B, _, H, W = x.shape
    gh, gw = H // 16, W // 16
    e = "image_encoder."
    f = F.conv2d(x, p[e + "conv1.weight"], stride=16).reshape(B, 768, -1).permute(0, 2, 1)
    cls = p[e + "class_embedding"].view(1, 1, -1).expand(B, 1, 768)
    f = torch.cat([cls, f], dim=1) + p[e + "positional_embedding"]
    f = layer_norm(f, p[e + "ln_pre.weight"], p[e + "ln_pre.bias"])
    def prepare(l):
        v = p[f"vpt_{l}"].unsqueeze(0).expand(B, -1, -1)
        return v * vpt_masks[l] if vpt_masks is not None else v
    vpt = prepare(0)
    for l in range(layers):
        if deep_vpt and l > 0:
            vpt = prepare(l)
        f = torch.cat([f[:, :1], vpt, f[:, 1:]], dim=1)
        f = block(f, p, f"{e}transformer.resblocks.{l}.")
        vpt = f[:, 1:1 + num_vpt]
        f = torch.cat([f[:, :1], f[:, 1 + num_vpt:]], dim=1)
    f = layer_norm(f, p[e + "ln_post.weight"], p[e + "ln_post.bias"])
    return f[:, 1:].permute(0, 2, 1).reshape(B, 768, gh, gw)


def batch_norm_train(x, w, b):
    return F.batch_norm(x, None, None, w, b, training=True, momentum=0.1, eps=1e-5)


def batch_norm_eval(x, w, b, rm, rv):
    """BatchNorm2d in eval mode: the running statistics."""
    return F.batch_norm(x, rm, rv, w, b, training=False, momentum=0.1, eps=1e-5)


def decoder(p, x, train: bool = True):
    """BasicBlock (models/utils.py:290-303) after bilinear x2 (models/clip/model.py:195-196); train=False: the
    BatchNorms use their running statistics (model.eval(), eval.py / utils/eval_utils.py)."""
    x = F.interpolate(x, scale_factor=2.0, mode="bilinear")
    d = "image_decoder.0."

    def bn(o, name):
        if train:
            return batch_norm_train(o, p[d + name + ".weight"], p[d + name + ".bias"])
        return batch_norm_eval(o, p[d + name + ".weight"], p[d + name + ".bias"], p[d + name + ".running_mean"],
                               p[d + name + ".running_var"])
    o = F.conv2d(x, p[d + "conv1.weight"], padding=1)
    o = F.relu(bn(o, "bn1"))
    o = F.conv2d(o, p[d + "conv2.weight"], padding=1)
    o = bn(o, "bn2")
    return F.relu(o + x)


def head(p, x, text_features, anchors):
    """projection + similarity head (models/clip/model.py:198-212)."""
    x = F.conv2d(x, p["projection.weight"], p["projection.bias"])
    img = F.normalize(x.permute(0, 2, 3, 1), p=2, dim=-1)
    txt = F.normalize(text_features, p=2, dim=-1)
    logits = (p["logit_scale"].exp() * img @ txt.t()).permute(0, 3, 1, 2)
    probs = logits.softmax(dim=1)
    exp = (probs * torch.as_tensor(anchors, dtype=probs.dtype, device=probs.device).view(1, -1, 1, 1)).sum(dim=1, keepdim=True)
    return logits, exp


TRAINABLE_PREFIXES = ("vpt_", "image_decoder.", "projection.", "logit_scale")


def params_from_state(sd: Dict[str, np.ndarray], requires_grad: bool = True) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in sd.items():
        t = torch.tensor(np.asarray(v))
        if requires_grad and k.startswith(TRAINABLE_PREFIXES) and t.is_floating_point():
            t.requires_grad_(True)
        out[k] = t
    return out


def forward(p, x, text_features, anchors, layers: int, deep_vpt: bool = True, train: bool = True, vpt_masks=None):
    feats = vit_vpt_forward(p, x, layers, deep_vpt=deep_vpt, vpt_masks=vpt_masks)
    return head(p, decoder(p, feats, train), text_features, anchors) + (feats,)


# ----------------------------------------------------------------------------- clip_resnet50 (config 2)
RESNET_TRAINABLE_PREFIXES = ("image_encoder.", "image_decoder.", "projection.", "logit_scale")


def _bn_conv(p, x, conv, bn, stride=1, padding=0):
    o = F.conv2d(x, p[conv + ".weight"], stride=stride, padding=padding)
    return batch_norm_train(o, p[bn + ".weight"], p[bn + ".bias"])


def resnet_encoder(p, x, layers=(3, 4, 6, 3), reduction: int = 8):
    """ModifiedResNet features_only, out_indices=(-1,) (models/clip/_clip/image_encoder.py:36-115): 3-conv stem +
    avgpool, Bottleneck stages (blocks.py:56-101: avgpool before conv3 and in the downsample when strided),
    layer4 at stride 1 when reduction <= 16."""
    e = "image_encoder."
    x = F.relu(_bn_conv(p, x, e + "conv1", e + "bn1", stride=2, padding=1))
    x = F.relu(_bn_conv(p, x, e + "conv2", e + "bn2", padding=1))
    x = F.relu(_bn_conv(p, x, e + "conv3", e + "bn3", padding=1))
    x = F.avg_pool2d(x, 2)
    for li, n in enumerate(layers):
        stride = 1 if li == 0 else (2 if li < 3 or reduction > 16 else 1)
        for bi in range(n):
            q = f"{e}layer{li + 1}.{bi}."
            s = stride if bi == 0 else 1
            o = F.relu(_bn_conv(p, x, q + "conv1", q + "bn1"))
            o = F.relu(_bn_conv(p, o, q + "conv2", q + "bn2", padding=1))
            if s > 1:
                o = F.avg_pool2d(o, s)
            o = _bn_conv(p, o, q + "conv3", q + "bn3")
            if q + "downsample.0.weight" in p:
                idt = F.avg_pool2d(x, s) if s > 1 else x
                idt = _bn_conv(p, idt, q + "downsample.0", q + "downsample.1")
            else:
                idt = x
            x = F.relu(o + idt)
    return x


def bottleneck_decoder(p, x, up: int = 2):
    """Bottleneck(2048, 2048, expansion=1) (models/utils.py:346-363) after the bilinear x`up` adapt
    (models/clip/model.py:195-196)."""
    if up != 1:
        x = F.interpolate(x, scale_factor=float(up), mode="bilinear")
    d = "image_decoder.0."
    o = F.relu(_bn_conv(p, x, d + "conv1", d + "bn1"))
    o = F.relu(_bn_conv(p, o, d + "conv2", d + "bn2", padding=1))
    o = _bn_conv(p, o, d + "conv3", d + "bn3")
    return F.relu(o + x)


def resnet_params_from_state(sd: Dict[str, np.ndarray]) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in sd.items():
        t = torch.tensor(np.asarray(v))
        if k.startswith(RESNET_TRAINABLE_PREFIXES) and t.is_floating_point() and "running_" not in k:
            t.requires_grad_(True)
        out[k] = t
    return out


def resnet_forward(p, x, text_features, anchors, reduction: int = 8):
    feats = resnet_encoder(p, x, reduction=reduction)
    return head(p, bottleneck_decoder(p, feats, 16 // reduction if reduction <= 16 else 1), text_features,
                anchors) + (feats,)

"""Drop-in DACE / DMCount losses backed by the fused gfx950 kernel (`ebc_dace_loss`).

Mirrors the reference surface:
  * `DACELoss(bins, reduction, weight_count_loss=1.0, count_loss="mae", **kwargs)`
    (losses/dace_loss.py:9-70), `forward(pred_class, pred_density, target_density, target_points)
    -> (loss, loss_info)` with keys `loss, ot_loss, tv_loss, count_loss, ce_loss` (dmcount) or
    `ce_loss, {mae,mse}_loss, loss`;
  * `DMLoss(input_size, reduction, norm_cood=False, weight_ot=0.1, weight_tv=0.01, ...)`
    (losses/dm_loss.py:82-124), `forward(pred_density, target_density, target_points)`.

Forward AND backward run in one kernel launch (+ a 1-block finalize): the loss is the last node of
the graph, so its gradients are produced with the value and replayed (times the upstream scalar)
in `backward`.
"""
from __future__ import annotations

from typing import Any, Dict, List, Sequence, Tuple

import torch
from torch import Tensor, nn

from . import _lib

_INFO_DM = ("loss", "ot_loss", "tv_loss", "count_loss", "ce_loss")


class _DaceFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred_class, pred_density, target_density, points, offsets, order, bins_lo, bins_hi,
                cfg):
        (B, N, size, red, mode, norm, wc, wot, wtv, reg, iters, thr, freq, total, reduced) = cfg
        dev = pred_density.device
        g = size // red
        pc = pred_class.detach().float().contiguous()
        pd = pred_density.detach().float().contiguous()
        td = target_density.detach().float().contiguous()
        grad_c = torch.empty_like(pc)
        grad_d = torch.empty_like(pd)
        losses = torch.empty(5, device=dev, dtype=torch.float32)
        stats = torch.empty(B, 8, device=dev, dtype=torch.float32)
        L = _lib.lib()
        ws_bytes = L.ebc_dace_workspace_bytes(B, total, size, red)
        ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
        rc = L.ebc_dace_loss(_lib.ptr(pc), _lib.ptr(pd), _lib.ptr(td), int(reduced), _lib.ptr(points),
                             _lib.ptr(offsets), _lib.ptr(order), _lib.ptr(bins_lo), _lib.ptr(bins_hi),
                             B, N, size, red, mode, int(norm), wc, wot, wtv, reg, iters, thr, freq,
                             _lib.ptr(grad_c), _lib.ptr(grad_d), _lib.ptr(losses), _lib.ptr(stats),
                             None, None, _lib.ptr(ws), ws_bytes, _lib.stream())
        _lib.check(rc, "ebc_dace_loss")
        ctx.save_for_backward(grad_c, grad_d)
        ctx.dtypes = (pred_class.dtype, pred_density.dtype)
        ctx.mark_non_differentiable(stats)
        return losses, stats

    @staticmethod
    def backward(ctx, g_losses, g_stats):
        grad_c, grad_d = ctx.saved_tensors
        s = g_losses[0]
        return ((grad_c * s).to(ctx.dtypes[0]), (grad_d * s).to(ctx.dtypes[1]),
                None, None, None, None, None, None, None)


def _pack_points(target_points: Sequence[Tensor], device) -> Tuple[Tensor, Tensor, Tensor, int]:
    counts = [int(p.shape[0]) for p in target_points]
    total = sum(counts)
    if total:
        pts = torch.cat([p.reshape(-1, 2).to(device=device, dtype=torch.float32) for p in target_points], 0).contiguous()
    else:
        pts = torch.zeros(1, 2, device=device, dtype=torch.float32)
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    order = sorted(range(len(counts)), key=lambda i: -counts[i])        # heaviest crops first
    meta = torch.tensor(offs + order, dtype=torch.int32).pin_memory() if torch.cuda.is_available() else torch.tensor(offs + order, dtype=torch.int32)
    meta = meta.to(device, non_blocking=True)
    return pts, meta[: len(offs)], meta[len(offs):], total


class DACELoss(nn.Module):
    """losses/dace_loss.py:9-70 on the fused HIP kernel."""

    def __init__(self, bins: List[Tuple[float, float]], reduction: int, weight_count_loss: float = 1.0,
                 count_loss: str = "mae", **kwargs: Any) -> None:
        super().__init__()
        assert len(bins) > 0, f"Expected at least one bin, got {bins}"
        assert all([len(b) == 2 for b in bins]), f"Expected all bins to be of length 2, got {bins}"
        assert all([b[0] <= b[1] for b in bins]), f"Expected all bins to be in increasing order, got {bins}"
        self.bins = bins
        self.reduction = reduction
        count_loss = count_loss.lower()
        assert count_loss in ["mae", "mse", "dmcount"], f"Expected count_loss to be one of ['mae', 'mse', 'dmcount'], got {count_loss}"
        self.count_loss = count_loss
        self.use_dm_loss = count_loss == "dmcount"
        if self.use_dm_loss:
            assert "input_size" in kwargs, f"Expected input_size to be in kwargs when count_loss='dmcount', got {kwargs}"
            self.count_loss_fn = DMLoss(reduction=reduction, **kwargs)
        self.weight_count_loss = weight_count_loss
        self.register_buffer("bins_lo", torch.tensor([float(b[0]) for b in bins], dtype=torch.float32), persistent=False)
        self.register_buffer("bins_hi", torch.tensor([float(b[1]) for b in bins], dtype=torch.float32), persistent=False)

    def forward(self, pred_class: Tensor, pred_density: Tensor, target_density: Tensor,
                target_points: List[Tensor]) -> Tuple[Tensor, Dict[str, Tensor]]:
        B, N, h, w = pred_class.shape
        assert N == len(self.bins), f"pred_class has {N} channels, expected {len(self.bins)} bins"
        assert pred_density.shape == (B, 1, h, w), f"Expected pred_density [B,1,H,W], got {pred_density.shape}"
        assert h == w, "square crops only"
        reduced = tuple(target_density.shape[-2:]) == (h, w)
        size = h * self.reduction
        if not reduced:
            assert tuple(target_density.shape[-2:]) == (size, size), \
                f"target_density {tuple(target_density.shape)} does not match pred_density {tuple(pred_density.shape)}"
        dm = self.count_loss_fn if self.use_dm_loss else None
        if dm is not None:
            assert dm.ot_loss.input_size == size, f"DMLoss input_size {dm.ot_loss.input_size} != crop size {size}"
        mode = {"dmcount": _lib.EBC_COUNT_DMCOUNT, "mae": _lib.EBC_COUNT_MAE, "mse": _lib.EBC_COUNT_MSE}[self.count_loss]
        dev = pred_density.device
        pts, offs, order, total = _pack_points(target_points, dev)
        lo, hi = self.bins_lo.to(dev), self.bins_hi.to(dev)
        cfg = (B, N, size, self.reduction, mode,
               dm.ot_loss.norm_cood if dm else False,
               float(self.weight_count_loss),
               float(dm.weight_ot) if dm else 0.0, float(dm.weight_tv) if dm else 0.0,
               float(dm.ot_loss.reg) if dm else 10.0, int(dm.ot_loss.num_of_iter_in_ot) if dm else 0,
               1e-9, 10, total, reduced)
        losses, _ = _DaceFn.apply(pred_class, pred_density, target_density, pts, offs, order, lo, hi, cfg)
        d = losses.detach()
        if self.use_dm_loss:
            info = {k: d[i] for i, k in enumerate(_INFO_DM)}
        else:
            info = {"ce_loss": d[4], f"{self.count_loss}_loss": d[3], "loss": d[0]}
        return losses[0], info


class _OTParams:
    def __init__(self, input_size, reduction, norm_cood, num_of_iter_in_ot=100, reg=10.0):
        assert input_size % reduction == 0
        self.input_size, self.reduction, self.norm_cood = input_size, reduction, norm_cood
        self.num_of_iter_in_ot, self.reg = num_of_iter_in_ot, reg


class DMLoss(nn.Module):
    """losses/dm_loss.py:82-124 (OT + TV + count) on the fused HIP kernel."""

    def __init__(self, input_size: int, reduction: int, norm_cood: bool = False, weight_ot: float = 0.1,
                 weight_tv: float = 0.01, **kwargs: Any) -> None:
        super().__init__()
        self.ot_loss = _OTParams(input_size, reduction, norm_cood, **kwargs)
        self.weight_ot = weight_ot
        self.weight_tv = weight_tv

    def forward(self, pred_density: Tensor, target_density: Tensor, target_points: List[Tensor]):
        B, _, h, w = pred_density.shape
        dev = pred_density.device
        size = self.ot_loss.input_size
        reduced = tuple(target_density.shape[-2:]) == (h, w)
        pts, offs, order, total = _pack_points(target_points, dev)
        # one dummy bin: the CE part of the fused kernel is computed on zero logits and discarded
        zero_class = torch.zeros(B, 1, h, w, device=dev, dtype=torch.float32)
        lo = torch.zeros(1, device=dev); hi = torch.full((1,), float("inf"), device=dev)
        cfg = (B, 1, size, self.ot_loss.reduction, _lib.EBC_COUNT_DMCOUNT, self.ot_loss.norm_cood, 1.0,
               float(self.weight_ot), float(self.weight_tv), float(self.ot_loss.reg),
               int(self.ot_loss.num_of_iter_in_ot), 1e-9, 10, total, reduced)
        losses, _ = _DaceFn.apply(zero_class, pred_density, target_density, pts, offs, order, lo, hi, cfg)
        d = losses.detach()
        loss = losses[0] - losses[4]   # remove the dummy CE (log 1 = 0 anyway)
        info = {"loss": d[0] - d[4], "ot_loss": d[1], "tv_loss": d[2], "count_loss": d[3]}
        return loss, info

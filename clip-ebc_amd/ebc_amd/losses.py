"""Drop-in DACE / DMCount / OT losses and `sinkhorn`, backed by gfx950 kernels.

Mirrors the reference surface:
  * `DACELoss(bins, reduction, weight_count_loss=1.0, count_loss="mae", **kwargs)`
    (losses/dace_loss.py:9-70), `forward(pred_class, pred_density, target_density, target_points)
    -> (loss, loss_info)` with keys `loss, ot_loss, tv_loss, count_loss, ce_loss` (dmcount) or
    `ce_loss, {mae,mse}_loss, loss`;
  * `DMLoss(input_size, reduction, norm_cood=False, weight_ot=0.1, weight_tv=0.01, ...)`
    (losses/dm_loss.py:82-124), `forward(pred_density, target_density, target_points)`;
  * `OTLoss(input_size, reduction, norm_cood, num_of_iter_in_ot=100, reg=10.0)` (losses/dm_loss.py:12-79),
    `forward(pred_density, normed_pred_density, target_points) -> (loss, wd, ot_obj_values)`;
  * `sinkhorn(a, b, C, reg=1e-1, maxIter=1000, stopThr=1e-9, verbose=False, log=True, eval_freq=10,
    print_freq=200) -> P | (P, log)` (losses/bregman_pytorch.py:11-144), log keys err/u/v/alpha/beta.

DACE/DMCount forward AND backward run in one kernel launch (+ a 1-block finalize): the loss is the last
node of the graph, so its gradients are produced with the value and replayed (times the upstream
scalar) in `backward`.  The Sinkhorn internals of the last call (beta [B, g*g], status [B]: iterations,
negative = NaN/Inf rollback, and the per-crop err of the last check) are kept on the DMLoss / OTLoss
module when it is built with `keep_internals=True` (off by default: an extra [B, g*g] write).

Geometry: the fused kernel takes any density grid g = input_size / reduction up to 64 x 64 (reduction
8 / 16 / 32 at any crop size up to 512 at reduction 8; fixtures F1 / F1g pin eight geometries); larger grids raise
NotImplementedError at construction.
"""
from __future__ import annotations

import ctypes

from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn

from . import _lib

_INFO_DM = ("loss", "ot_loss", "tv_loss", "count_loss", "ce_loss")
MAX_GRID = 64       # density grids g = input_size / reduction up to 64 x 64 (the kernel's LDS-resident state)
M_EPS = 1e-16      # bregman_pytorch.py:8


def _check_geometry(input_size: int, reduction: int) -> None:
    assert input_size % reduction == 0, f"input_size {input_size} is not a multiple of reduction {reduction}"
    g = input_size // reduction
    if g > MAX_GRID or reduction % 4:
        raise NotImplementedError(
            f"ebc_amd DMCount kernel: density grid input_size/reduction = {g} (reduction {reduction}); "
            f"built for grids up to {MAX_GRID} with reduction % 4 == 0")


class _Internals:
    """Per-crop Sinkhorn results of one fused call (device tensors)."""

    def __init__(self, beta: Tensor, status: Tensor, stats: Tensor):
        self.beta = beta                 # [B, g*g]  reg * log(v + 1e-16)   (bregman_pytorch.py:137)
        self.status = status             # [B] int32 iterations run, negative = rolled back at that iteration
        self.crop_stats = stats          # [B, 8] ce, tv*n, count, ot, wd, iters, rolled, err of the last check

    @property
    def err_last(self) -> Tensor:
        return self.crop_stats[:, 7]

    @property
    def wd(self) -> Tensor:
        return self.crop_stats[:, 4]


def _run_dace(pred_class, pred_density, target_density, points, offsets, order, bins_lo, bins_hi, cfg,
              keep: bool):
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
    beta = torch.empty(B, g * g, device=dev, dtype=torch.float32) if keep else None
    status = torch.empty(B, device=dev, dtype=torch.int32) if keep else None
    L = _lib.lib()
    with _lib.on(dev):
        ws_bytes = L.ebc_dace_workspace_bytes(B, total, size, red)
        ws = torch.empty(ws_bytes, device=dev, dtype=torch.uint8)
        # offsets / order: host ctypes arrays (B <= 64: kernel arguments, ebc_dace_loss_h) or device tensors
        host = not isinstance(offsets, torch.Tensor)
        fn = L.ebc_dace_loss_h if host else L.ebc_dace_loss
        rc = fn(_lib.ptr(pc), _lib.ptr(pd, dev), _lib.ptr(td, dev), int(reduced), _lib.ptr(points, dev),
                             offsets if host else _lib.ptr(offsets, dev), order if host else _lib.ptr(order, dev),
                             _lib.ptr(bins_lo, dev), _lib.ptr(bins_hi, dev),
                             B, N, size, red, mode, int(norm), wc, wot, wtv, reg, iters, thr, freq,
                             _lib.ptr(grad_c), _lib.ptr(grad_d), _lib.ptr(losses), _lib.ptr(stats),
                             _lib.ptr(beta), _lib.ptr(status), _lib.ptr(ws), ws_bytes, _lib.stream(dev))
    _lib.check(rc, "ebc_dace_loss")
    return losses, stats, grad_c, grad_d, (_Internals(beta, status, stats) if keep else None)


class _DaceFn(torch.autograd.Function):
    """Outputs: the total loss (0-dim, differentiable), the 5 loss terms and the per-crop stats (both
    non-differentiable).  The backward gets the total's upstream gradient alone (no materialised zero gradients
    for the other outputs) and scales both kernel-made gradients by it in one foreach launch."""

    @staticmethod
    def forward(ctx, pred_class, pred_density, target_density, points, offsets, order, bins_lo, bins_hi,
                cfg, sink):
        losses, stats, grad_c, grad_d, internals = _run_dace(pred_class, pred_density, target_density, points,
                                                             offsets, order, bins_lo, bins_hi, cfg, sink is not None)
        if sink is not None:
            sink.append(internals)
        ctx.save_for_backward(grad_c, grad_d)
        ctx.dtypes = (pred_class.dtype, pred_density.dtype)
        ctx.set_materialize_grads(False)
        terms = losses.detach()
        ctx.mark_non_differentiable(terms, stats)
        return losses[0], terms, stats

    @staticmethod
    def backward(ctx, g_loss, g_terms, g_stats):
        if g_loss is None:
            return (None,) * 10
        grad_c, grad_d = ctx.saved_tensors
        if g_loss.dtype == torch.float32 and g_loss.numel() == 1 and g_loss.device == grad_c.device:
            gc, gd = torch.empty_like(grad_c), torch.empty_like(grad_d)
            with _lib.on(grad_c.device):
                _lib.check(_lib.lib().ebc_scale2(_lib.ptr(g_loss), _lib.ptr(grad_c), _lib.ptr(gc), grad_c.numel(),
                                                 _lib.ptr(grad_d), _lib.ptr(gd), grad_d.numel(), _lib.stream(grad_c.device)),
                           "ebc_scale2")
        else:
            gc, gd = torch._foreach_mul([grad_c, grad_d], g_loss)
        return (gc.to(ctx.dtypes[0]), gd.to(ctx.dtypes[1]), None, None, None, None, None, None, None, None)


def _packed_views(target_points: Sequence[Tensor], device) -> bool:
    """True when the point lists are row-contiguous f32 [n_i, 2] views laid end to end in one device storage."""
    p0 = target_points[0]
    if p0.device != torch.device(device):
        return False
    store = p0.untyped_storage().data_ptr()
    nxt = store + p0.storage_offset() * 4                 # (an empty view's data_ptr() is 0: use the offsets)
    for p in target_points:
        if (p.dtype != torch.float32 or p.dim() != 2 or p.shape[1] != 2 or p.device != p0.device
                or (p.shape[0] > 1 and p.stride() != (2, 1)) or (p.shape[0] == 1 and p.stride(1) != 1)
                or p.untyped_storage().data_ptr() != store or (p.shape[0] and p.data_ptr() != nxt)):
            return False
        nxt += p.shape[0] * 8
    return True


HMETA_MAX = 64          # dace_loss.hip: up to this many crops the offsets / order travel as kernel arguments


def _pack_points(target_points: Sequence[Tensor], device):
    """The ragged label list -> packed [sum n, 2] f32 + offsets [B+1] + heaviest-first crop order: host ctypes arrays
    for up to HMETA_MAX crops (passed as kernel arguments, no copy), else one H2D of both."""
    counts = [int(p.shape[0]) for p in target_points]
    total = sum(counts)
    if total and _packed_views(target_points, device):
        # the crops' point lists are consecutive rows of one [sum n, 2] f32 device buffer (a collate that uploads the
        # batch's labels in one copy): use it as is, no concatenation launch
        p0 = target_points[0]
        pts = torch.empty(0, device=device, dtype=torch.float32).set_(p0.untyped_storage(), p0.storage_offset(),
                                                                      (total, 2), (2, 1))
    elif total:
        pts = torch.cat([p.reshape(-1, 2).to(device=device, dtype=torch.float32) for p in target_points], 0).contiguous()
    else:
        pts = torch.zeros(1, 2, device=device, dtype=torch.float32)
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    order = sorted(range(len(counts)), key=lambda i: -counts[i])        # heaviest crops first
    if len(counts) <= HMETA_MAX:
        return pts, (ctypes.c_int * len(offs))(*offs), (ctypes.c_int * len(order))(*order), total
    meta = torch.tensor(offs + order, dtype=torch.int32)
    if torch.cuda.is_available():
        meta = meta.pin_memory()
    meta = meta.to(device, non_blocking=True)
    return pts, meta[: len(offs)], meta[len(offs):], total


class _OTParams:
    """OTLoss's configuration (losses/dm_loss.py:12-35)."""

    def __init__(self, input_size, reduction, norm_cood, num_of_iter_in_ot=100, reg=10.0):
        _check_geometry(input_size, reduction)
        self.input_size, self.reduction, self.norm_cood = input_size, reduction, norm_cood
        self.num_of_iter_in_ot, self.reg = num_of_iter_in_ot, reg
        self.output_size = input_size // reduction


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
        elif reduction % 4:
            raise NotImplementedError(f"ebc_amd DACE kernel: reduction {reduction} (needs reduction % 4 == 0)")
        self.weight_count_loss = weight_count_loss
        self.register_buffer("bins_lo", torch.tensor([float(b[0]) for b in bins], dtype=torch.float32), persistent=False)
        self.register_buffer("bins_hi", torch.tensor([float(b[1]) for b in bins], dtype=torch.float32), persistent=False)

    def forward(self, pred_class: Tensor, pred_density: Tensor, target_density: Tensor,
                target_points: List[Tensor]) -> Tuple[Tensor, Dict[str, Tensor]]:
        B, N, h, w = pred_class.shape
        assert N == len(self.bins), f"pred_class has {N} channels, expected {len(self.bins)} bins"
        assert pred_density.shape == (B, 1, h, w), f"Expected pred_density [B,1,H,W], got {pred_density.shape}"
        assert h == w, "square crops only"
        assert len(target_points) == B, f"Expected target_points to have length {B}, but got {len(target_points)}"
        if h != w or h > MAX_GRID:
            raise NotImplementedError(f"ebc_amd DACE kernel: density grid {h}x{w}; built for square grids up to {MAX_GRID}")
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
        sink = [] if (dm is not None and dm.keep_internals) else None
        loss, d, stats = _DaceFn.apply(pred_class, pred_density, target_density, pts, offs, order, lo, hi, cfg, sink)
        if sink:
            dm.internals = sink[0]
        # the 5 terms as one device vector in _INFO_DM order (loss, ot, tv, count, ce): a packed all-reduce
        # needs no stack launch; the per-crop stats [B, 8] (ce, tv*n, count, ot, wd, iterations, rolled back, err)
        self.last_terms = d
        self.last_stats = stats
        if self.use_dm_loss:
            info = {k: d[i] for i, k in enumerate(_INFO_DM)}
        else:
            info = {"ce_loss": d[4], f"{self.count_loss}_loss": d[3], "loss": d[0]}
        return loss, info


def _dummy_class(B: int, h: int, w: int, dev) -> Tuple[Tensor, Tensor, Tensor]:
    """One bin covering every count: the fused kernel's CE part is log-softmax of a single logit = 0."""
    return (torch.zeros(B, 1, h, w, device=dev, dtype=torch.float32), torch.zeros(1, device=dev),
            torch.full((1,), float("inf"), device=dev))


class DMLoss(nn.Module):
    """losses/dm_loss.py:82-124 (OT + TV + count) on the fused HIP kernel."""

    def __init__(self, input_size: int, reduction: int, norm_cood: bool = False, weight_ot: float = 0.1,
                 weight_tv: float = 0.01, keep_internals: bool = False, **kwargs: Any) -> None:
        super().__init__()
        self.ot_loss = _OTParams(input_size, reduction, norm_cood, **kwargs)
        self.weight_ot = weight_ot
        self.weight_tv = weight_tv
        self.keep_internals = keep_internals
        self.internals: Optional[_Internals] = None

    def forward(self, pred_density: Tensor, target_density: Tensor, target_points: List[Tensor]):
        B, _, h, w = pred_density.shape
        assert len(target_points) == B, f"Expected target_points to have length {B}, but got {len(target_points)}"
        dev = pred_density.device
        size = self.ot_loss.input_size
        reduced = tuple(target_density.shape[-2:]) == (h, w)
        pts, offs, order, total = _pack_points(target_points, dev)
        zero_class, lo, hi = _dummy_class(B, h, w, dev)
        cfg = (B, 1, size, self.ot_loss.reduction, _lib.EBC_COUNT_DMCOUNT, self.ot_loss.norm_cood, 1.0,
               float(self.weight_ot), float(self.weight_tv), float(self.ot_loss.reg),
               int(self.ot_loss.num_of_iter_in_ot), 1e-9, 10, total, reduced)
        sink = [] if self.keep_internals else None
        loss, d, _ = _DaceFn.apply(zero_class, pred_density, target_density, pts, offs, order, lo, hi, cfg, sink)
        if sink:
            self.internals = sink[0]
        loss = loss - d[4]             # remove the dummy CE (log 1 = 0 anyway)
        info = {"loss": d[0] - d[4], "ot_loss": d[1], "tv_loss": d[2], "count_loss": d[3]}
        return loss, info


class OTLoss(nn.Module):
    """losses/dm_loss.py:12-79: per crop, the entropic OT between the normalised predicted density and
    the crop's points (uniform weights), returned as the surrogate loss sum(pred_density * gradient) whose
    gradient w.r.t. pred_density is beta/count - <beta, density>/count^2 (dm_loss.py:65-76).

    `normed_pred_density` must be pred_density / (count + 1e-8), which is what the reference's only
    caller passes (dm_loss.py:106-108); the kernel forms it from `pred_density` itself.  `wd` (the
    Wasserstein distance sum(C * P), dm_loss.py:77) is a host float as in the reference (one sync)."""

    def __init__(self, input_size: int, reduction: int, norm_cood: bool, num_of_iter_in_ot: int = 100,
                 reg: float = 10.0, keep_internals: bool = False) -> None:
        super().__init__()
        p = _OTParams(input_size, reduction, norm_cood, num_of_iter_in_ot, reg)
        self.input_size, self.reduction, self.norm_cood = p.input_size, p.reduction, p.norm_cood
        self.num_of_iter_in_ot, self.reg, self.output_size = p.num_of_iter_in_ot, p.reg, p.output_size
        self.keep_internals = keep_internals
        self.internals: Optional[_Internals] = None

    def forward(self, pred_density: Tensor, normed_pred_density: Tensor,
                target_points: List[Tensor]) -> Tuple[Tensor, float, Tensor]:
        B = normed_pred_density.size(0)
        assert len(target_points) == B, f"Expected target_points to have length {B}, but got {len(target_points)}"
        assert self.output_size == normed_pred_density.size(2)
        _, _, h, w = pred_density.shape
        # the kernel forms the Sinkhorn source marginal from pred_density itself: a caller that normalises
        # differently would get a loss, gradient and ot_obj from two different marginals, so refuse it
        pd = pred_density.detach().float()
        own = pd / (pd.sum(dim=(1, 2, 3), keepdim=True) + 1e-8)
        if not torch.allclose(normed_pred_density.detach().float(), own, rtol=1e-4, atol=1e-7):
            raise ValueError("OTLoss: normed_pred_density must be pred_density / (pred_density.sum((1, 2, 3)) + 1e-8) "
                             "(losses/dm_loss.py:106-108), the marginal the fused kernel uses")
        dev = pred_density.device
        pts, offs, order, total = _pack_points(target_points, dev)
        zero_class, lo, hi = _dummy_class(B, h, w, dev)
        dummy_target = torch.zeros(B, 1, h, w, device=dev, dtype=torch.float32)
        cfg = (B, 1, self.input_size, self.reduction, _lib.EBC_COUNT_OT_ONLY, self.norm_cood, 1.0, 1.0, 0.0,
               float(self.reg), int(self.num_of_iter_in_ot), 1e-9, 10, total, True)
        sink = []
        loss, _, stats = _DaceFn.apply(zero_class, pred_density, dummy_target, pts, offs, order, lo, hi, cfg, sink)
        it = sink[0]
        if self.keep_internals:
            self.internals = it
        # ot_obj_values = sum over crops with points of <normed_pred_density, beta> (dm_loss.py:66)
        has = torch.tensor([float(len(p) > 0) for p in target_points], device=dev).view(B, 1)
        ot_obj = (normed_pred_density.detach().float().reshape(B, -1) * it.beta * has).sum().reshape(1)
        wd = float(stats[:, 4].sum())
        return loss.reshape(1), wd, ot_obj               # OT-only mode: losses[0] = losses[1] = sum of the crops' OT


def sinkhorn(a: Tensor, b: Tensor, C: Tensor, reg: float = 1e-1, maxIter: int = 1000, stopThr: float = 1e-9,
             verbose: bool = False, log: bool = True, eval_freq: int = 10, print_freq: int = 200):
    """losses/bregman_pytorch.py:11-144 on one device launch (`ebc_sinkhorn`): every iteration, the
    NaN/Inf rollback and the err checks stay on the GPU; the host reads the iteration count and the err
    list once at the end (the reference syncs ~4 times per iteration).  Returns P, or (P, log) with log
    keys err (list of floats), u, v, alpha, beta."""
    if not (a.is_cuda and b.is_cuda and C.is_cuda):
        raise RuntimeError("ebc_amd.sinkhorn runs on the MI355X HIP path only (inputs on the CPU)")
    dev = a.device
    na, nb = C.shape
    assert na >= 1 and nb >= 1, f"C needs to be 2d. Found C.shape = {C.shape}"
    assert na == a.shape[0] and nb == b.shape[0], f"Shape of a ({a.shape}) or b ({b.shape}) does not match that of C ({C.shape})"
    assert reg > 0, f"reg should be greater than 0. Found reg = {reg}"
    assert bool((a.min() >= 0.) & (b.min() >= 0.)), f"Elements in a and b should be nonnegative. Found a.min() = {a.min()}, b.min() = {b.min()}"
    a32, b32, C32 = (t.detach().float().contiguous() for t in (a, b, C))
    f32 = dict(device=dev, dtype=torch.float32)
    P = torch.empty(na, nb, **f32)
    u, v, alpha, beta = torch.empty(na, **f32), torch.empty(nb, **f32), torch.empty(na, **f32), torch.empty(nb, **f32)
    nerr_max = max(1, -(-int(maxIter) // int(eval_freq)))
    err = torch.empty(nerr_max, **f32)
    info = torch.zeros(2, device=dev, dtype=torch.int32)
    L = _lib.lib()
    with _lib.on(dev):
        wsb = L.ebc_sinkhorn_workspace_bytes(na, nb)
        ws = torch.empty(max(wsb, 1), device=dev, dtype=torch.uint8)
        rc = L.ebc_sinkhorn(_lib.ptr(a32), _lib.ptr(b32, dev), _lib.ptr(C32, dev), na, nb, float(reg), int(maxIter),
                            float(stopThr), int(eval_freq), int(bool(log)), _lib.ptr(P), _lib.ptr(u), _lib.ptr(v),
                            _lib.ptr(alpha), _lib.ptr(beta), _lib.ptr(err), _lib.ptr(info), _lib.ptr(ws), wsb,
                            _lib.stream(dev))
    _lib.check(rc, "ebc_sinkhorn")
    iters, nerr = (int(x) for x in info.cpu())
    if iters < 0:
        print("Warning: numerical errors at iteration", -iters)          # bregman_pytorch.py:113
    errs = [float(e) for e in err[:nerr].cpu()] if log else []
    if verbose:
        for k, e in enumerate(errs):
            if ((k + 1) * eval_freq) % print_freq == 0:
                print("iteration {:5d}, constraint error {:5e}".format((k + 1) * eval_freq, e))
    if log:
        return P, {"err": errs, "u": u, "v": v, "alpha": alpha, "beta": beta}
    return P

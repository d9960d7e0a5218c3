"""Sliding-window evaluation and error metrics (utils/eval_utils.py, eval.py), on device.

`sliding_window_predict(model, image, window_size, stride)` keeps the reference signature and
result (a CPU tensor [1, 1, H/r, W/r], overlaps averaged); tiles are gathered and the map assembled
by HIP kernels (`ebc_tile_gather` / `ebc_tile_assemble`) and the model runs once per tile batch.
Sharding the tiles of one image across ranks (BASELINE config 5) is OPT-IN (`shard=True`, every rank
of `group` must call): the reference trainer evaluates on rank 0 alone while the other ranks wait in
`dist.barrier()` (trainer.py:161-177,194), so a collective inside the default call would hang there.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple, Union

import numpy as np
import torch
import torch.distributed as dist
from torch import Tensor, nn

from . import _lib
from .distributed import gather_shards, shard_range


def calculate_errors(pred_counts: np.ndarray, gt_counts: np.ndarray) -> Dict[str, float]:
    """utils/eval_utils.py:8-16."""
    assert isinstance(pred_counts, np.ndarray), f"Expected numpy.ndarray, got {type(pred_counts)}"
    assert isinstance(gt_counts, np.ndarray), f"Expected numpy.ndarray, got {type(gt_counts)}"
    assert len(pred_counts) == len(gt_counts), f"Length of predictions and ground truths should be equal, but got {len(pred_counts)} and {len(gt_counts)}"
    return {"mae": np.mean(np.abs(pred_counts - gt_counts)), "rmse": np.sqrt(np.mean((pred_counts - gt_counts) ** 2))}


def _pair(v) -> Tuple[int, int]:
    return (int(v), int(v)) if isinstance(v, (int, float)) else tuple(int(x) for x in v)


def tile_grid(H: int, W: int, window: Tuple[int, int], stride: Tuple[int, int]) -> Tuple[int, int]:
    rows = int(np.ceil((H - window[0]) / stride[0]) + 1)
    cols = int(np.ceil((W - window[1]) / stride[1]) + 1)
    return rows, cols


def sliding_window_predict(model: nn.Module, image: Tensor, window_size: Union[int, Tuple[int, int]],
                           stride: Union[int, Tuple[int, int]], max_tiles_per_batch: int = 256,
                           shard: bool = False, group: Optional[object] = None) -> Tensor:
    """utils/eval_utils.py:26-96.  image [1, C, H, W] -> [1, Cp, H/r, W/r] (CPU tensor).

    shard=True (collective: every rank of `group` calls with the same image): each rank runs its
    contiguous share of the tiles and the predictions are all-gathered before the assembly."""
    assert len(image.shape) == 4, f"Image must be a 4D tensor (1, c, h, w), got {image.shape}"
    window, strd = _pair(window_size), _pair(stride)
    assert window[0] > 0 and window[1] > 0, f"Window size must be a positive integer tuple (h, w), got {window}"
    assert strd[0] > 0 and strd[1] > 0, f"Stride must be a positive integer tuple (h, w), got {strd}"
    assert strd[0] <= window[0] and strd[1] <= window[1], f"Stride must be smaller than window size, got {strd} and {window}"
    params = list(model.parameters())
    dev = params[0].device if params else (image.device if image.is_cuda else torch.device("cuda"))
    img = image.to(dev, torch.float32).contiguous()[0]
    C, H, W = img.shape
    rows, cols = tile_grid(H, W, window, strd)
    T = rows * cols
    reduction = getattr(model, "reduction", 1)
    world = dist.get_world_size(group) if shard and dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    t0, t1, per = shard_range(T, world, rank)
    L = _lib.lib()
    st = _lib.stream(dev)
    preds = None
    model.eval()
    with torch.no_grad(), _lib.on(dev):
        outs = []
        for b0 in range(t0, t1, max_tiles_per_batch):
            n = min(max_tiles_per_batch, t1 - b0)
            tiles = torch.empty(n, C, window[0], window[1], device=dev, dtype=torch.float32)
            _lib.check(L.ebc_tile_gather(_lib.ptr(img, dev), _lib.ptr(tiles), C, H, W, window[0], window[1], strd[0],
                                         strd[1], b0, n, st), "ebc_tile_gather")
            outs.append(model(tiles).float())
        if outs:
            preds = torch.cat(outs, 0)
        Cp = preds.shape[1] if preds is not None else 1
        ph, pw = window[0] // reduction, window[1] // reduction
        if world > 1:
            preds = gather_shards(preds, T, per, (Cp, ph, pw), dev, group)
        preds = preds.contiguous()
        out = torch.empty(Cp, H // reduction, W // reduction, device=dev)
        _lib.check(L.ebc_tile_assemble(_lib.ptr(preds, dev), _lib.ptr(out), Cp, H, W, window[0], window[1], strd[0],
                                       strd[1], reduction, st), "ebc_tile_assemble")
    return out.unsqueeze(0).cpu()


def evaluate(model: nn.Module, data_loader, device: torch.device, sliding_window: bool = False,
             window_size: Optional[int] = None, stride: Optional[int] = None) -> Dict[str, float]:
    """eval.py:11-40: per-image predicted count vs len(points); returns {"mae", "rmse"}."""
    model.eval()
    pred_counts, target_counts = [], []
    if sliding_window:
        assert window_size is not None, f"Window size must be provided when sliding_window is True, but got {window_size}"
        assert stride is not None, f"Stride must be provided when sliding_window is True, but got {stride}"
    for image, target_points, _ in data_loader:
        image = image.to(device)
        target_counts.append([len(p) for p in target_points])
        with torch.no_grad():
            if sliding_window:
                pred_density = sliding_window_predict(model, image, window_size, stride)
            else:
                pred_density = model(image)
            pred_counts.append(pred_density.sum(dim=(1, 2, 3)).cpu().numpy().tolist())
    pred_counts = np.array([x for s in pred_counts for x in s])
    target_counts = np.array([x for s in target_counts for x in s])
    return calculate_errors(pred_counts, target_counts)

"""Drop-in training epoch: `train(model, data_loader, loss_fn, optimizer, grad_scaler, device, rank, nprocs)`
(train.py:14-69), the reference trainer's per-epoch call (trainer.py:156).

Same contract and result: autocast under an enabled GradScaler (train.py:36-40), classification models
get (pred_class, pred_density) and regression models (`bins is None`) pred_density only, the scaler's
scale/step/update, and the epoch mean of every loss_info entry averaged over the ranks.  Two deliberate
changes for the GPU path:
  * the loss_info values stay on the device and are summed there; ONE packed all-reduce and ONE host
    read at the end of the epoch replace the reference's per-step five all-reduces and five .item()
    host synchronisations (train.py:62);
  * no per-step barrier (train.py:67): DDP's gradient all-reduce already keeps the ranks in step.
`amp_dtype` (extension, default fp16 as the reference) selects bf16 autocast, e.g. for clip_resnet50.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

from .losses import _INFO_DM

try:
    from tqdm import tqdm
except ImportError:                                   # pragma: no cover
    tqdm = None


def train(model: nn.Module, data_loader, loss_fn: nn.Module, optimizer: torch.optim.Optimizer,
          grad_scaler: Optional[torch.amp.GradScaler], device: torch.device, rank: int, nprocs: int,
          amp_dtype: torch.dtype = torch.float16, progress: bool = True
          ) -> Tuple[nn.Module, torch.optim.Optimizer, Optional[torch.amp.GradScaler], Dict[str, float]]:
    model.train()
    device = torch.device(device)
    ddp = nprocs > 1
    regression = (model.module.bins is None) if ddp else (model.bins is None)
    it = tqdm(data_loader) if (progress and rank == 0 and tqdm is not None) else data_loader
    keys, acc, steps = None, None, 0
    use_amp = grad_scaler is not None and grad_scaler.is_enabled()
    for image, target_points, target_density in it:
        image = image.to(device, non_blocking=True)
        target_points = [p.to(device, non_blocking=True) for p in target_points]
        target_density = target_density.to(device, non_blocking=True)
        with torch.set_grad_enabled(True), torch.autocast(device.type, dtype=amp_dtype, enabled=use_amp):
            if not regression:
                pred_class, pred_density = model(image)
                loss, loss_info = loss_fn(pred_class, pred_density, target_density, target_points)
            else:
                pred_density = model(image)
                loss, loss_info = loss_fn(pred_density, target_density, target_points)
        optimizer.zero_grad()
        if grad_scaler is not None:
            grad_scaler.scale(loss).backward()
            grad_scaler.step(optimizer)
            grad_scaler.update()
        else:
            loss.backward()
            optimizer.step()
        if keys is None:
            keys = list(loss_info.keys())
        terms = getattr(loss_fn, "last_terms", None)
        if terms is not None and keys == list(_INFO_DM):
            packed = terms                            # DACELoss's own [5] vector in keys' order: no stack launch
        else:
            packed = torch.stack([loss_info[k].detach().float().reshape(()) for k in keys])
        acc = packed if acc is None else acc + packed
        steps += 1
    if steps == 0:
        return model, optimizer, grad_scaler, {}
    if ddp:
        dist.all_reduce(acc, op=dist.ReduceOp.SUM)
        acc = acc / nprocs
    mean = (acc / steps).tolist()                     # the epoch's one host read
    return model, optimizer, grad_scaler, {k: float(v) for k, v in zip(keys, mean)}

"""Process-per-GPU data parallelism over RCCL (torch.distributed "nccl" = RCCL on ROCm).

Mirrors utils/ddp_utils.py (setup / cleanup / barrier / reduce_mean / init_seeds) and the DDP
wrapping of trainer.py:147, with two deliberate changes for MI355X:
  * the five per-step loss scalars are reduced in ONE packed all-reduce without a host sync
    (reference: five all-reduces + five `.item()`, train.py:62, collective C6);
  * no per-step barrier (reference train.py:67, C7): the gradient all-reduce already orders steps.
Rendezvous defaults to 127.0.0.1 (the container hostname may not resolve).
"""
from __future__ import annotations

import os
import random
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist
from torch import Tensor, nn

LOSS_KEYS = ("loss", "ot_loss", "tv_loss", "count_loss", "ce_loss")


def setup(local_rank: int, nprocs: int, backend: Optional[str] = None, port: int = 12355) -> None:
    """utils/ddp_utils.py:16-22."""
    if nprocs > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(port))
        backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend, rank=local_rank, world_size=nprocs)


def cleanup(ddp: bool = True) -> None:
    if ddp and dist.is_initialized():
        dist.destroy_process_group()


def barrier(ddp: bool = True) -> None:
    if ddp:
        dist.barrier()


def reduce_mean(tensor: Tensor, nprocs: int) -> Tensor:
    """utils/ddp_utils.py:9-13."""
    rt = tensor.clone()
    dist.all_reduce(rt, op=dist.ReduceOp.SUM)
    rt /= nprocs
    return rt


def init_seeds(seed: int, cuda_deterministic: bool = False) -> None:
    """utils/ddp_utils.py:30-39 (cudnn flags map to MIOpen on ROCm)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.backends.cudnn.deterministic = cuda_deterministic
    torch.backends.cudnn.benchmark = not cuda_deterministic


def reduce_loss_info(info: Dict[str, Tensor], nprocs: int, keys: Sequence[str] = LOSS_KEYS) -> Dict[str, Tensor]:
    """All five loss scalars in one packed all-reduce (mean over ranks), results stay on device."""
    keys = [k for k in keys if k in info]
    packed = torch.stack([info[k].detach().float().reshape(()) for k in keys])
    if nprocs > 1:
        dist.all_reduce(packed, op=dist.ReduceOp.SUM)
        packed /= nprocs
    return {k: packed[i] for i, k in enumerate(keys)}


def wrap_ddp(model: nn.Module, local_rank: int) -> nn.Module:
    """trainer.py:147: SyncBatchNorm for the decoder BN + DDP (bucketed gradient all-reduce, overlapped
    with the backward)."""
    model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
    return nn.parallel.DistributedDataParallel(model, device_ids=[local_rank], output_device=local_rank,
                                               bucket_cap_mb=25, gradient_as_bucket_view=True)


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int, int]:
    """Contiguous shard of `total` items for `rank`: (begin, end, per_rank_capacity)."""
    per = (total + world - 1) // world
    b = min(rank * per, total)
    return b, min(b + per, total), per


def gather_shards(local: Optional[Tensor], total: int, per: int, item_shape: Tuple[int, ...], device,
                  group=None) -> Tensor:
    """All-gather equal-capacity shards (zero padded) and return the first `total` items in order."""
    world = dist.get_world_size(group)
    buf = torch.zeros((per,) + tuple(item_shape), device=device)
    if local is not None and local.shape[0]:
        buf[: local.shape[0]] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat(parts, 0)[:total].contiguous()

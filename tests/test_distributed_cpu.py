"""world_size-2 gloo tests (CPU) of the N>1 path: packed loss all-reduce, tile sharding + gather,
and the DDP gradient contract of the DACE loss (mean over crops for CE/TV/count, SUM over crops for
the OT term, exactly as the reference under DDP)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ANCHORS_NWPU, BINS, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, world=2, *args):
    port = _free_port()
    mp.start_processes(_entry, args=(fn, world, port) + args, nprocs=world, start_method="spawn", join=True)


def _entry(rank, fn, world, port, *args):
    import sys
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.destroy_process_group()


def _packed_reduce(rank, world):
    from ebc_amd.distributed import reduce_loss_info, reduce_mean
    info = {k: torch.tensor(float(rank * 10 + i)) for i, k in enumerate(("loss", "ot_loss", "tv_loss", "count_loss", "ce_loss"))}
    packed = reduce_loss_info(info, world)
    for k, v in info.items():
        assert torch.allclose(packed[k], reduce_mean(v, world))


def test_packed_loss_reduce_matches_reference_reduce_mean():
    _run(_packed_reduce)


def _tile_gather(rank, world, T):
    from ebc_amd.distributed import gather_shards, shard_range
    b, e, per = shard_range(T, world, rank)
    local = torch.arange(b, e, dtype=torch.float32).view(-1, 1, 1, 1).expand(-1, 1, 2, 2).contiguous()
    full = gather_shards(local, T, per, (1, 2, 2), torch.device("cpu"))
    assert full.shape == (T, 1, 2, 2)
    assert torch.equal(full[:, 0, 0, 0], torch.arange(T, dtype=torch.float32))


@pytest.mark.parametrize("T", [140, 7, 1])
def test_tile_sharding_covers_every_tile_once(T):
    _run(_tile_gather, 2, T)


def _ddp_contract(rank, world, path):
    """DDP(mean over ranks) of per-rank DACE-loss gradients vs the single-process gradient."""
    from oracle import ref
    from ebc_amd import synthetic as syn
    g = np.random.Generator(np.random.PCG64(5))
    B = 4
    pcl = g.standard_normal((B, 5, 28, 28)).astype(np.float32)
    pde = (g.random((B, 1, 28, 28)) * 2).astype(np.float32)
    counts = [3, 0, 12, 7]
    pts = [(g.random((n, 2)) * 224).astype(np.float32) for n in counts]
    dens = np.stack([syn.point_map(p, 224, 224)[None] for p in pts])
    # single process, whole batch
    pc = torch.tensor(pcl, requires_grad=True); pd = torch.tensor(pde, requires_grad=True)
    loss, _ = ref.dace_loss(pc, pd, torch.from_numpy(dens), pts, BINS)
    loss.backward()
    # this rank's half, gradients averaged over ranks (what DDP does)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    qc = torch.tensor(pcl[sl], requires_grad=True); qd = torch.tensor(pde[sl], requires_grad=True)
    l2, _ = ref.dace_loss(qc, qd, torch.from_numpy(dens[sl]), pts[sl], BINS)
    l2.backward()
    gc = qc.grad.clone(); gd = qd.grad.clone()
    # per-crop CE/TV/count gradients are 1/B_rank-normalised: the mean over ranks equals the global
    # 1/B normalisation for equal shards.  pred_class only sees CE:
    full_c = torch.zeros(B, 5, 28, 28); full_c[sl] = gc / world
    dist.all_reduce(full_c)
    assert torch.allclose(full_c, pc.grad, rtol=1e-5, atol=1e-7)
    # the OT term is a SUM over crops (dm_loss.py:76), so under DDP its gradient is 1/world of the
    # single-process one: check the identity explicitly on pred_density.
    ot_single = np.zeros((B, 1, 28, 28), np.float32)
    for b, p in enumerate(pts):
        if len(p):
            ot_single[b, 0] = ref.ot_crop(p, pde[b, 0], 224)["ot_grad"].reshape(28, 28)
    full_d = torch.zeros(B, 1, 28, 28); full_d[sl] = gd / world
    dist.all_reduce(full_d)
    expect = pd.grad - 0.1 * torch.from_numpy(ot_single) * (1 - 1.0 / world)
    assert torch.allclose(full_d, expect, rtol=1e-4, atol=1e-6)


def test_ddp_gradient_contract_of_dace_loss():
    _run(_ddp_contract, 2, None)


# ------------------------------------------------------------------ drop-in train() (train.py:14-69)
class _TinyCounter(torch.nn.Module):
    """A stand-in CLIP-EBC-shaped model for the host logic of train(): (pred_class, pred_density)."""
    bins = [(0, 0), (1, 1)]

    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.conv = torch.nn.Conv2d(3, 3, 8, stride=8)

    def forward(self, x):
        y = self.conv(x)
        return y[:, :2], y[:, 2:].abs()


def _tiny_loss(pred_class, pred_density, target_density, target_points):
    n = torch.tensor([float(len(p)) for p in target_points])
    ce = pred_class.square().mean()
    cnt = (pred_density.sum(dim=(1, 2, 3)) - n).abs().mean()
    loss = ce + cnt
    return loss, {"loss": loss.detach(), "ce_loss": ce.detach(), "count_loss": cnt.detach()}


def _loader(rank, steps=3, B=2):
    g = torch.Generator().manual_seed(100 + rank)
    return [(torch.randn(B, 3, 16, 16, generator=g), [torch.rand(int(k), 2, generator=g) for k in torch.randint(0, 9, (B,), generator=g)],
             torch.zeros(B, 1, 16, 16)) for _ in range(steps)]


def _reference_epoch(model, loader, opt, rank, nprocs):
    """The reference's loop (train.py:30-69): per step five reduce_means + .item(), np.mean over steps."""
    from ebc_amd.distributed import reduce_mean
    per = {}
    for image, pts, dens in loader:
        pc, pd = model(image)
        loss, info = _tiny_loss(pc, pd, dens, pts)
        opt.zero_grad()
        loss.backward()
        opt.step()
        for k, v in info.items():
            per.setdefault(k, []).append(float(reduce_mean(v, nprocs)) if nprocs > 1 else float(v))
        if nprocs > 1:
            dist.barrier()
    return {k: float(np.mean(v)) for k, v in per.items()}


def _train_world2(rank, world):
    from ebc_amd.train import train
    a = torch.nn.parallel.DistributedDataParallel(_TinyCounter())
    b = torch.nn.parallel.DistributedDataParallel(_TinyCounter())
    oa = torch.optim.SGD(a.parameters(), lr=0.05)
    ob = torch.optim.SGD(b.parameters(), lr=0.05)
    _, _, _, got = train(a, _loader(rank), _tiny_loss, oa, None, torch.device("cpu"), rank, world, progress=False)
    want = _reference_epoch(b, _loader(rank), ob, rank, world)
    assert got.keys() == want.keys()
    for k in want:
        assert abs(got[k] - want[k]) <= 1e-6 * max(1.0, abs(want[k])), (k, got[k], want[k])
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-7)


def test_train_epoch_matches_reference_loop_world2():
    """One packed all-reduce at the end of the epoch == the reference's per-step reduce_mean + np.mean;
    the parameters after the epoch are the same as the reference loop's (DDP gradient averaging)."""
    _run(_train_world2)


def test_train_epoch_single_process():
    from ebc_amd.train import train
    a, b = _TinyCounter(), _TinyCounter()
    oa, ob = torch.optim.SGD(a.parameters(), lr=0.05), torch.optim.SGD(b.parameters(), lr=0.05)
    _, _, _, got = train(a, _loader(0), _tiny_loss, oa, None, torch.device("cpu"), 0, 1, progress=False)
    want = _reference_epoch(b, _loader(0), ob, 0, 1)
    for k in want:
        assert abs(got[k] - want[k]) <= 1e-6 * max(1.0, abs(want[k]))

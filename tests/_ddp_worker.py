"""Rank body of the world-2 DDP + SyncBatchNorm GPU test (tests/test_gpu_ddp.py).

Runs in a fresh process forked from the session's forkserver (started by conftest.py before anything
touched the GPU), so no process that initialised HIP ever execs.  Both ranks share cuda:0 over gloo
(a one-GPU box); rank r trains on its own slice of one crop batch, exactly as trainer.py:143-147 wraps
the model (SyncBatchNorm + DistributedDataParallel), and saves what the parent compares.
"""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for _p in (REPO, os.path.join(REPO, "clip-ebc_amd"), HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

BINS = [(0.0, 0.0), (1.0, 1.0), (2.0, 2.0), (3.0, 3.0), (4.0, float("inf"))]
ANCHORS = [0.0, 1.0, 2.0, 3.0, 4.21931]
LAYERS = 2
SPLIT = (2, 1)          # crops per rank: uneven, so SyncBN must all-reduce the per-rank counts


def batch():
    from ebc_amd import synthetic as syn
    return syn.synthetic_crops(sum(SPLIT), 224, seed=4040, counts=[30, 7, 120])


def build(device):
    import numpy as np
    import torch
    from ebc_amd.model import get_model
    txt = torch.from_numpy(np.load(os.path.join(HERE, "golden", "f6_text.npz"))["text_features_word"])
    return get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS, prompt_type="word", vit_layers=LAYERS, text_layers=1,
                     text_features=txt, weights_seed=0).to(device).train()


def rank_main(rank: int, world: int, port: int, out_dir: str) -> None:
    import torch
    import torch.distributed as dist
    from ebc_amd.distributed import wrap_ddp, reduce_loss_info
    from ebc_amd.losses import DACELoss
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    model = wrap_ddp(build(dev), 0)
    img, pts, dens = batch()
    b0 = sum(SPLIT[:rank])
    sl = slice(b0, b0 + SPLIT[rank])
    x = torch.from_numpy(img[sl]).to(dev)
    from ebc_amd.model import DecoderMaskTap
    DecoderMaskTap.capture = []                # this rank's decoder ReLU decisions (the parent replays them)
    logits, exp = model(x)
    (m1, m2, _, _), = DecoderMaskTap.capture
    DecoderMaskTap.capture = None
    loss, info = DACELoss(BINS, 8, count_loss="dmcount", input_size=224)(
        logits, exp, torch.from_numpy(dens[sl]).to(dev), [torch.from_numpy(p).to(dev) for p in pts[sl]])
    loss.backward()
    info = reduce_loss_info(info, world)
    torch.cuda.synchronize()
    m = model.module
    res = {k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.requires_grad}
    for k, b in m.named_buffers():
        if "running" in k or "num_batches" in k:
            res["buf:" + k] = b.detach().cpu()
    res.update({"info:" + k: v.detach().cpu() for k, v in info.items()})
    res["mask1"], res["mask2"] = m1.cpu(), m2.cpu()
    torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def eval_image():
    import numpy as np
    return np.random.Generator(np.random.PCG64(31)).standard_normal((1, 3, 500, 700)).astype("float32")


def eval_main(rank: int, world: int, port: int, out_dir: str) -> None:
    """Rank body of the eval-sharding test: (1) rank 0 alone calls sliding_window_predict while rank 1 waits in
    dist.barrier() -- the reference trainer's eval pattern (trainer.py:161-177,194); (2) both ranks call it with
    shard=True on the same image."""
    import torch
    import torch.distributed as dist
    from ebc_amd.eval_utils import sliding_window_predict
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    m = build(dev).eval()
    img = torch.from_numpy(eval_image()).to(dev)
    res = {}
    if rank == 0:
        res["rank0_only"] = sliding_window_predict(m, img, 224, 112)
    dist.barrier()
    res["sharded"] = sliding_window_predict(m, img, 224, 112, shard=True)
    torch.save(res, os.path.join(out_dir, f"eval_rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()

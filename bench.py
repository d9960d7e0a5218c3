"""Benchmark: train crops/s for clip_vit_b_16 + deep VPT(32) + DMCount at 224x224 on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--crops-per-gpu B] [--dtype fp16|bf16|fp32]

One step = forward (autocast, like the reference train.py:36-40) + DACE/DMCount loss (on-device
Sinkhorn) + backward + GradScaler/Adam step over the 11.3 M trainable parameters, on synthetic
crops pre-staged in HBM (BASELINE.md "Synthetic inputs").  N > 1: one process per GPU under
torch.distributed.run, DDP over RCCL with SyncBatchNorm as trainer.py:147; weak scaling (fixed
crops per GPU).  Rank 0 prints ONE JSON line (see README / DESIGN.md §Measurement).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BINS = [(0.0, 0.0), (1.0, 1.0), (2.0, 2.0), (3.0, 3.0), (4.0, float("inf"))]
ANCHORS_NWPU = [0.0, 1.0, 2.0, 3.0, 4.21931]     # configs/reduction_8.json ["4"]["nwpu"]["average"]
FLOP_PER_CROP = 135.63e9                          # 58.33 fwd + 77.30 bwd GFLOP
MFMA_PEAK_TF = {"fp16": 2500.0, "bf16": 2500.0, "fp32": 157.3}   # MI355X dense (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--crops-per-gpu", type=int, default=16)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "bf16", "fp32"])
    ap.add_argument("--pool", type=int, default=4, help="distinct synthetic batches cycled through")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-crops", type=int, default=8, help="crops per CPU-baseline step")
    ap.add_argument("--cpu-steps", type=int, default=12)
    ap.add_argument("--eval", action="store_true",
                    help="SURVEY §8(d) config 5 instead: sliding-window eval of 2048x3072 images (window = stride = 224, "
                         "140 tiles per image, tiles sharded over ranks); --steps images timed; --dtype fp32 is the "
                         "reference's own eval precision")
    ap.add_argument("--augment", action="store_true",
                    help="SURVEY §8f row f2 instead: the reference's training augmentation on device (RandomResizedCrop + "
                         "flip + RandomApply(jitter, blur, noise) + normalise + dot maps), 16 images x 2 crops per step")
    return ap.parse_args()


def make_batch(B, rank, step, device):
    """BASELINE.md synthetic crops: seed 1000 + rank*100003 + step, lognormal(ln 20, 1.2) points."""
    from ebc_amd import synthetic as syn
    img, pts, dens = syn.synthetic_crops(B, 224, seed=1000 + rank * 100003 + step)
    return (torch.from_numpy(img).to(device), [torch.from_numpy(p).to(device) for p in pts],
            torch.from_numpy(dens).to(device), [len(p) for p in pts])


def cpu_baseline(args, crops, steps):
    """The oracle (oracle/ref.py: torch-fp32 CPU restatement of the reference step) on host cores."""
    from oracle import ref
    from ebc_amd import synthetic as syn
    nthreads = torch.get_num_threads()
    sd = syn.full_state(0, layers=12, include_text=False)
    p = ref.params_from_state(sd)
    train = [v for k, v in p.items() if v.requires_grad]
    opt = torch.optim.Adam(train, lr=1e-4, weight_decay=1e-4)
    txt = torch.randn(5, 512, generator=torch.Generator().manual_seed(0))

    def step(s):
        img, pts, dens = syn.synthetic_crops(crops, 224, seed=5000 + s)
        logits, exp, _ = ref.forward(p, torch.from_numpy(img), txt, ANCHORS_NWPU, 12)
        loss, _ = ref.dace_loss(logits, exp, torch.from_numpy(dens), pts, BINS)
        opt.zero_grad()
        loss.backward()
        opt.step()

    step(0)                                                  # warm-up
    t0 = time.perf_counter()
    for s in range(steps):
        step(s + 1)
    dt = time.perf_counter() - t0
    return {"value": round(crops * steps / dt, 4), "unit": "crops/s", "cores": nthreads, "kind": "port",
            "sample": f"{steps} steps x {crops} crops (fwd+DACE/DMCount+bwd+Adam, fp32, 12 layers) of the oracle "
                      f"oracle/ref.py on {nthreads} host threads; {dt:.1f}s"}


def probe_kernels(dtype, device, reps=50):
    """Time the dominant encoder GEMM (MLP c_fc, M = 16*229) and the Sinkhorn loss kernel alone with
    HIP events on the current stream; returns roofline entries."""
    from ebc_amd import _lib
    L = _lib.lib()
    tdt = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32}[dtype]
    M, N, K = 16 * 229, 3072, 768
    A = torch.randn(M, K, device=device).to(tdt)
    Bw = (torch.randn(N, K, device=device) / 28).to(tdt)
    C = torch.empty(M, N, device=device, dtype=tdt)
    aux = torch.empty(M, N, device=device, dtype=tdt)
    bias = torch.zeros(N, device=device)
    code = _lib.dtype_code(tdt)

    def launch():
        _lib.check(L.ebc_gemm(code, 1, 0, _lib.ptr(A), _lib.ptr(Bw), _lib.ptr(C), _lib.ptr(bias), None,
                              _lib.ptr(aux), M, N, K, _lib.stream()), "probe gemm")
    for _ in range(5):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / reps * 1e-3
    flops = 2.0 * M * N * K
    return {"kernel": "gemm_nt_kernel<f16,GELU> (MLP c_fc 3664x3072x768, aux store)", "avg_us": t * 1e6,
            "achieved": flops / t / 1e12, "flops_per_launch": flops}


def setup(args, rank, world, local, device):
    """Model, loss, optimizer and the per-step closure (shared with tools/torch_prof.py)."""
    torch.manual_seed(42 + rank)
    from ebc_amd.model import get_model
    from ebc_amd.losses import DACELoss
    model = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", num_vpt=32,
                      vpt_drop=0.0, deep_vpt=True).to(device)
    model.train()
    if world > 1:
        from ebc_amd.distributed import wrap_ddp       # SyncBatchNorm + DDP, as trainer.py:147
        model = wrap_ddp(model, device.index)
    loss_fn = DACELoss(BINS, 8, weight_count_loss=1.0, count_loss="dmcount", input_size=224).to(device)
    params = [p for p in model.parameters() if p.requires_grad]
    try:
        opt = torch.optim.Adam(params, lr=1e-4, weight_decay=1e-4, fused=True)
    except Exception:
        opt = torch.optim.Adam(params, lr=1e-4, weight_decay=1e-4)
    amp_dtype = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": None}[args.dtype]
    scaler = torch.amp.GradScaler("cuda", enabled=args.dtype == "fp16")
    B = args.crops_per_gpu
    pool = [make_batch(B, rank, s, device) for s in range(args.pool)]
    info_buf = torch.zeros(5, device=device)

    def step(i):
        img, pts, dens, _ = pool[i % len(pool)]
        with torch.autocast("cuda", dtype=amp_dtype, enabled=amp_dtype is not None):
            logits, exp = model(img)
            loss, info = loss_fn(logits, exp, dens, pts)
        opt.zero_grad(set_to_none=True)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        # one packed all-reduce of the 5 loss_info scalars (reference: 5 separate + .item(), train.py:62)
        torch.stack([info[k] for k in ("loss", "ot_loss", "tv_loss", "count_loss", "ce_loss")], out=info_buf)
        if world > 1:
            dist.all_reduce(info_buf)
    return step


def run_augment(args, rank, device):
    """Row f2: crops/s of ebc_amd.transforms.CropAugment (host parameter draws + label arithmetic + the
    three augmentation launches + dot maps) for 16 NWPU-sized 1536x2048 images x num_crops 2 per step,
    images pre-staged in HBM; the CPU baseline runs the oracle (torch CPU: the reference's own ops) on the
    same crop plans."""
    from ebc_amd.transforms import CropAugment
    from oracle import augment_ref
    H, W, NI, NC = 1536, 2048, 16, 2
    g = torch.Generator().manual_seed(5 + rank)
    imgs = [torch.rand(3, H, W, generator=g).to(device) for _ in range(NI)]
    labels = [torch.rand(200, 2, generator=g) * torch.tensor([W, H], dtype=torch.float32) for _ in range(NI)]
    aug = CropAugment()                                     # trainer.py:40-52 defaults
    torch.manual_seed(rank)
    for _ in range(args.warmup):
        aug(imgs, labels, NC)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        aug(imgs, labels, NC)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # device-only share: the launches of one step between events
    plans = [aug.plan_crop(i, H, W, labels[i].clone())[0] for i in range(NI) for _ in range(NC)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        aug.apply(imgs, plans)
    e1.record()
    torch.cuda.synchronize()
    dev_ms = e0.elapsed_time(e1) / 10
    if rank == 0:
        cpu_imgs = [x.cpu() for x in imgs[:2]]
        sample = [p for p in plans if p.image < 2]
        t1 = time.perf_counter()
        augment_ref.apply_plans(cpu_imgs, sample, (224, 224))
        cpu_el = time.perf_counter() - t1
        crops = NI * NC * args.steps
        print(json.dumps({
            "metric": "train-augment crops/s (RandomResizedCrop+flip+jitter+blur+noise+normalise+dot maps, trainer defaults)",
            "value": round(crops / el, 2), "unit": "crops/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3), "higher_is_better": True, "vs_baseline": None, "dtype": "f32",
            "data": "synthetic 1536x2048 images in HBM, 200 points each",
            "config": {"workload": f"{NI} images x {NC} crops -> 224x224 (SURVEY §8f f2)"},
            "device_ms_per_step": round(dev_ms, 4),
            "cpu_baseline": {"value": round(len(sample) / cpu_el, 2), "unit": "crops/s", "cores": torch.get_num_threads(),
                             "kind": "port", "sample": f"{len(sample)} crops of the same plans through oracle/augment_ref.py "
                                                       f"(torch CPU ops the reference's workers run); {cpu_el:.2f}s"}}), flush=True)


def run_eval(args, rank, world, device):
    """Config 5: images/s and tiles/s of ebc_amd.eval_utils.sliding_window_predict (utils/eval_utils.py:26-96) on
    QNRF-shaped synthetic images; the timed region includes the tile gather, the forward, the cross-rank tile
    gather and the overlap assembly + D2H copy the reference's API returns."""
    from ebc_amd.eval_utils import sliding_window_predict, tile_grid
    from ebc_amd.model import get_model
    torch.manual_seed(42)
    model = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", num_vpt=32,
                      vpt_drop=0.0, deep_vpt=True).to(device).eval()
    H, W = 2048, 3072
    g = np.random.Generator(np.random.PCG64(7))                 # one image, its tiles sharded over the ranks
    mean = np.array([0.485, 0.456, 0.406], np.float32).reshape(1, 3, 1, 1)
    std = np.array([0.229, 0.224, 0.225], np.float32).reshape(1, 3, 1, 1)
    img = torch.from_numpy(((g.random((1, 3, H, W), dtype=np.float32) - mean) / std).astype(np.float32)).to(device)
    rows, cols = tile_grid(H, W, (224, 224), (224, 224))
    amp_dtype = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": None}[args.dtype]

    def one():
        with torch.autocast("cuda", dtype=amp_dtype, enabled=amp_dtype is not None):
            return sliding_window_predict(model, img, 224, 224)

    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    if rank == 0:
        tiles = rows * cols
        print(json.dumps({
            "metric": "eval tiles/s clip_vit_b_16 sliding window 2048x3072 (window 224, stride 224)",
            "value": round(tiles * args.steps / elapsed, 2), "unit": "tiles/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_image": round(elapsed / args.steps * 1e3, 3),
            "images_per_s": round(args.steps / elapsed, 3), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (uniform pixels, ImageNet-normalised)",
            "config": {"workload": f"SURVEY §8(d) config 5: {tiles} tiles per image sharded over {world} rank(s)",
                       "tiles_per_image": tiles, "density_map": list(out.shape)}}), flush=True)


def committed_traffic(dtype):
    """HBM bytes per launch of the probe kernel from the committed PMC passes (FETCH_SIZE x2 gfx950
    correction + WRITE_SIZE, profiles/r01_gemm_fc_traffic.json); None when no profile matches."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01_gemm_fc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if dtype != "fp16" or "EF16" not in rec.get("kernel", ""):
        return None
    return rec["traffic_bytes_per_launch"]


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EBC_BENCH_ONE_DEVICE=1 EBC_BENCH_BACKEND=gloo: rehearse the N-rank path with every rank on cuda:0
    # (a 1-GPU box); the measured numbers of such a run are not a scaling result
    dev_index = 0 if os.environ.get("EBC_BENCH_ONE_DEVICE") == "1" else local
    backend = os.environ.get("EBC_BENCH_BACKEND", "nccl")
    if world > 1:
        dist.init_process_group(backend, device_id=torch.device(f"cuda:{dev_index}") if backend == "nccl" else None)
    torch.cuda.set_device(dev_index)
    device = torch.device(f"cuda:{dev_index}")
    if args.augment:
        run_augment(args, rank, device)
        if world > 1:
            dist.destroy_process_group()
        return
    if args.eval:
        run_eval(args, rank, world, device)
        if world > 1:
            dist.destroy_process_group()
        return
    step = setup(args, rank, world, local, device)
    B = args.crops_per_gpu

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    crops = B * world * args.steps
    value = crops / elapsed
    ms = elapsed / args.steps * 1e3

    if rank == 0:
        probe = probe_kernels(args.dtype, device)
        peak = MFMA_PEAK_TF[args.dtype]
        out = {
            "metric": "train crops/sec clip_vit_b_16 224px @1/2/4/8 MI355X; MAE parity",
            "value": round(value, 3), "unit": "crops/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (BASELINE.md crops, pre-staged in HBM; synthetic random-init weights)",
            "config": {"workload": f"clip_vit_b_16 224x224 deep-VPT(32) + DACE/DMCount train step, "
                                   f"{B} crops/GPU, AMP {args.dtype} (BASELINE configs[2]" + (", DDP configs[3] shape" if world > 1 else "") + ")",
                       "global_batch": B * world, "seq_len": 229, "parallelism": f"dp{world}"},
            "roofline": {"bound": "mfma", "achieved": round(probe["achieved"], 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(probe["achieved"] / peak, 4), "traffic": committed_traffic(args.dtype),
                         "traffic_unit": "bytes/launch (rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE, profiles/r01_gemm_fc_traffic.json)",
                         "algorithmic_bytes": 55369728,
                         "kernel": probe["kernel"], "avg_us": round(probe["avg_us"], 2)},
            "step_roofline": {"flop_per_crop": FLOP_PER_CROP, "achieved_tflops": round(value / world * FLOP_PER_CROP / 1e12, 2),
                              "frac": round(value / world * FLOP_PER_CROP / 1e12 / peak, 4)},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, args.cpu_crops, args.cpu_steps)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

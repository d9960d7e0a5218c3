"""Generate the golden parity fixtures by running the REFERENCE (Yiming-M/CLIP-EBC) in this container.

Run here only (it reads /root/reference, which does not exist on the GPU box):

    python tests/golden/make_golden.py

What it imports from the reference, and how:
  * `losses/` (DACELoss, DMLoss, sinkhorn) - imported as a package, it only needs torch.
  * the CLIP-EBC ViT path - `import models` would download CLIP weights on import
    (`models/clip/_clip/__init__.py:31-36`), so stub parent packages are registered in
    `sys.modules` and only the needed files are loaded by path: `models/utils.py`,
    `models/clip/utils.py`, `models/clip/_clip/{blocks,image_encoder,text_encoder,simple_tokenizer}.py`,
    `models/clip/model.py`.  `tokenize` is restated from `_clip/utils.py:209-249` (that file
    imports torchvision, absent here); `ftfy.fix_text` is stubbed as identity (prompts are ASCII).
  * `utils/eval_utils.py` loaded by path (its package `__init__` imports torchvision).

Weights are the deterministic synthetic ones of `ebc_amd.synthetic` (regenerable on the GPU
box); inputs are seeded.  Only inputs that cannot be regenerated cheaply and the outputs
are written, as compressed .npz files next to this script.
"""
from __future__ import annotations

import importlib.util
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
sys.dont_write_bytecode = True          # never write __pycache__ into the (read-only) reference tree
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
from ebc_amd import synthetic as syn  # noqa: E402

BINS = [(0.0, 0.0), (1.0, 1.0), (2.0, 2.0), (3.0, 3.0), (4.0, float("inf"))]
ANCHORS_NWPU = [0.0, 1.0, 2.0, 3.0, 4.21931]   # configs/reduction_8.json ["4"]["nwpu"]


def _load(name: str, path: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def _stub_pkg(name: str, path: str):
    m = types.ModuleType(name)
    m.__path__ = [path]
    sys.modules[name] = m
    return m


def load_reference():
    sys.modules.setdefault("ftfy", types.SimpleNamespace(fix_text=lambda s: s))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import losses  # the reference's own package
    from losses.bregman_pytorch import sinkhorn
    models = _stub_pkg("models", f"{REF}/models")
    mclip = _stub_pkg("models.clip", f"{REF}/models/clip")
    _clip = _stub_pkg("models.clip._clip", f"{REF}/models/clip/_clip")
    _load("models.utils", f"{REF}/models/utils.py")
    _load("models.clip.utils", f"{REF}/models/clip/utils.py")
    _load("models.clip._clip.blocks", f"{REF}/models/clip/_clip/blocks.py")
    ie = _load("models.clip._clip.image_encoder", f"{REF}/models/clip/_clip/image_encoder.py")
    te = _load("models.clip._clip.text_encoder", f"{REF}/models/clip/_clip/text_encoder.py")
    st = _load("models.clip._clip.simple_tokenizer", f"{REF}/models/clip/_clip/simple_tokenizer.py")
    tok = st.SimpleTokenizer()

    def tokenize(texts, context_length=77):
        # restated from models/clip/_clip/utils.py:209-249
        if isinstance(texts, str):
            texts = [texts]
        sot, eot = tok.encoder["<|startoftext|>"], tok.encoder["<|endoftext|>"]
        out = torch.zeros(len(texts), context_length, dtype=torch.int)
        for i, t in enumerate(texts):
            ids = [sot] + tok.encode(t) + [eot]
            out[i, :len(ids)] = torch.tensor(ids)
        return out

    state = {"vit_layers": 12}
    _clip.tokenize = tokenize
    _clip.vit_b_16_img = lambda features_only=True, input_size=224, **kw: ie.VisionTransformer(
        input_size, 16, 512, 768, state["vit_layers"], 12, features_only=features_only)
    _clip.vit_b_16_txt = lambda: te.CLIPTextEncoder(512, 77, 49408, 512, 8, 12)
    # clip_image_encoder_resnet50.json / clip_text_encoder_resnet50.json values (models/clip/_clip/__init__.py:73-148):
    # layers (3,4,6,3), width 64, embed 1024, heads 32, resolution 224; text 512 wide, 8 heads, 12 layers
    _clip.resnet50_img = lambda features_only=True, out_indices=None, reduction=32, **kw: ie.ModifiedResNet(
        (3, 4, 6, 3), 1024, 224, 64, 32, features_only=features_only, out_indices=out_indices, reduction=reduction)
    _clip.resnet50_txt = lambda: te.CLIPTextEncoder(1024, 77, 49408, 512, 8, 12)
    model_mod = _load("models.clip.model", f"{REF}/models/clip/model.py")
    eval_utils = _load("ref_eval_utils", f"{REF}/utils/eval_utils.py")
    return types.SimpleNamespace(losses=losses, sinkhorn=sinkhorn, model_mod=model_mod, state=state,
                                 tokenize=tokenize, eval_utils=eval_utils)


def build_ref_model(ref, layers: int, prompt_type: str = "word", anchors=ANCHORS_NWPU, seed: int = 0,
                    deep_vpt: bool = True):
    ref.state["vit_layers"] = layers
    torch.manual_seed(0)
    m = ref.model_mod._clip_ebc("vit_b_16", BINS, anchors, reduction=8, prompt_type=prompt_type,
                                input_size=224, num_vpt=32, deep_vpt=deep_vpt, vpt_drop=0.0)
    sd = syn.full_state(seed, layers=layers)
    if not deep_vpt:                             # shallow VPT: vpt_0 only (models/clip/model.py:72-75)
        sd = {k: v for k, v in sd.items() if not (k.startswith("vpt_") and k != "vpt_0")}
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith("num_batches_tracked") for k in missing) or not missing, missing
    m._extract_text_features()
    return m


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", path, f"{os.path.getsize(path) / 1024:.0f} KiB")


def pack_points(points):
    offs = np.zeros(len(points) + 1, np.int32)
    offs[1:] = np.cumsum([len(p) for p in points])
    flat = np.concatenate([p.reshape(-1, 2) for p in points]).astype(np.float32) if offs[-1] else np.zeros((0, 2), np.float32)
    return flat, offs


def loss_case(ref, size: int, counts, seed: int, reduction: int = 8, p_limit: int = 200 * 784):
    """F1: DACE(dmcount) loss + Sinkhorn internals on a ragged crop batch (any input_size % reduction == 0;
    transport plans P kept for crops with n * g^2 <= p_limit)."""
    g = np.random.Generator(np.random.PCG64(seed))
    B = len(counts)
    h = size // reduction
    points = [(g.random((n, 2)) * size).astype(np.float32) for n in counts]
    density = np.stack([syn.point_map(p, size, size)[None] for p in points])
    pred_class = g.standard_normal((B, 5, h, h)).astype(np.float32)
    pred_density = (g.random((B, 1, h, h)) * 1.5).astype(np.float32)
    pc = torch.tensor(pred_class, requires_grad=True)
    pd = torch.tensor(pred_density, requires_grad=True)
    loss_fn = ref.losses.DACELoss(BINS, reduction, weight_count_loss=1.0, count_loss="dmcount", input_size=size)
    loss, info = loss_fn(pc, pd, torch.from_numpy(density), [torch.from_numpy(p) for p in points])
    loss.backward()
    out = dict(size=size, reduction=reduction, counts=np.asarray(counts), pred_class=pred_class, pred_density=pred_density,
               grad_pred_class=pc.grad.numpy(), grad_pred_density=pd.grad.numpy())
    flat, offs = pack_points(points)
    out["points"], out["offsets"] = flat, offs
    for k, v in info.items():
        out["info_" + k] = v.detach().numpy().reshape(())
    # sinkhorn internals per crop, with OTLoss's exact inputs (dm_loss.py:51-64)
    ot = loss_fn.count_loss_fn.ot_loss
    cood = ot.cood
    pdt = torch.from_numpy(pred_density)
    normed = pdt / (pdt.view(B, -1).sum(1).view(-1, 1, 1, 1) + 1e-8)
    betas, us, vs, errs, grads, wds = [], [], [], [], [], []
    for b, p in enumerate(points):
        if len(p) == 0:
            betas.append(np.zeros(h * h, np.float32)); us.append(np.zeros(0, np.float32))
            vs.append(np.zeros(h * h, np.float32)); errs.append(np.zeros(10, np.float32) - 1)
            grads.append(np.zeros(h * h, np.float32)); wds.append(0.0)
            continue
        pt = torch.from_numpy(p)
        x = pt[:, 0].unsqueeze(1); y = pt[:, 1].unsqueeze(1)
        xd = -2 * torch.matmul(x, cood) + x * x + cood * cood
        yd = -2 * torch.matmul(y, cood) + y * y + cood * cood
        dist = (yd.unsqueeze(2) + xd.unsqueeze(1)).view(len(p), -1)
        a = torch.ones(len(p)) / len(p)
        P, log = ref.sinkhorn(a, normed[b][0].view(-1), dist, 10.0, maxIter=100, log=True)
        betas.append(log["beta"].numpy()); us.append(log["u"].numpy()); vs.append(log["v"].numpy())
        e = np.full(10, -1.0, np.float32); e[:len(log["err"])] = log["err"]; errs.append(e)
        sd = pdt[b][0].view(-1); sc = sd.sum()
        grad = sc / (sc * sc + 1e-8) * log["beta"] - (sd * log["beta"]).sum() / (sc * sc + 1e-8)
        grads.append(grad.numpy()); wds.append(float(torch.sum(dist * P)))
        if len(p) * h * h <= p_limit:
            out[f"P_{b}"] = P.numpy()
    out.update(beta=np.stack(betas), v=np.stack(vs), err=np.stack(errs), ot_grad=np.stack(grads), wd=np.asarray(wds))
    out["u_flat"] = np.concatenate(us) if us else np.zeros(0, np.float32)
    return out


LOSS_GRIDS = [(224, 16, [0, 5, 40, 300, 2], 303), (224, 32, [17, 0, 120], 304), (448, 16, [60, 1, 800], 305),
              (448, 32, [9, 250], 306), (384, 8, [33, 0, 500, 4], 307), (512, 8, [70, 3], 308)]


def loss_grids(ref):
    """F1g: the loss at the other geometries the reference allows (reduction 16 / 32, other crop sizes):
    density grids 14, 7, 28, 14, 48 and 64."""
    for size, red, counts, seed in LOSS_GRIDS:
        save(f"f1g_loss_{size}_r{red}.npz", **loss_case(ref, size, counts, seed, reduction=red, p_limit=40000))


def _capture_sinkhorn(ref):
    """Wrap the reference's sinkhorn as dm_loss.py calls it: record every call's log and the
    iteration its NaN/Inf rollback warning names (bregman_pytorch.py:111-115)."""
    import contextlib
    import io
    dm = sys.modules["losses.dm_loss"]
    calls = []
    orig = dm.sinkhorn

    def wrapped(*a, **k):
        f = io.StringIO()
        with contextlib.redirect_stdout(f):
            r = orig(*a, **k)
        msg = f.getvalue().strip()
        calls.append((r, int(msg.split()[-1]) if msg else 0))
        return r
    dm.sinkhorn = wrapped
    return calls, lambda: setattr(dm, "sinkhorn", orig)


def sinkhorn_case(ref):
    """F1b: the reference `sinkhorn` on general dense problems (losses/bregman_pytorch.py:11-144): early
    stop on stopThr, the NaN/Inf rollback at iteration 1 (a negative cost: K = inf) and 2 (marginals of
    mass 1 vs 1e24), log=False (err never updated: every iteration runs), a DMCount-shaped crop and one
    whose K exceeds LDS.  Inputs are stored (they are small); `roll` = the iteration of the warning."""
    import contextlib
    import io
    out = {}
    cases = []
    g = torch.Generator().manual_seed(4242)
    # 0: converges before maxIter (loose stopThr)
    C = torch.rand(9, 30, generator=g) * 20
    a = torch.rand(9, generator=g); a /= a.sum(); b = torch.rand(30, generator=g); b /= b.sum()
    cases.append((a, b, C, 5.0, 1000, 1e-4, True))
    # 1: a negative cost -> K = inf -> NaN at iteration 1
    C = torch.rand(5, 16, generator=g) * 5; C[1, 3] = -2000.0
    a = torch.ones(5) / 5; b = torch.rand(16, generator=g); b /= b.sum()
    cases.append((a, b, C, 1.0, 50, 1e-9, True))
    # 2: |b| = 1e24 vs |a| = 1: v overflows at iteration 2
    C = torch.rand(7, 20, generator=torch.Generator().manual_seed(1)) * 4
    a = torch.ones(7) / 7; b = torch.rand(20, generator=torch.Generator().manual_seed(2)); b = b / b.sum() * 1e24
    cases.append((a, b, C, 0.5, 100, 1e-9, True))
    # 3: log=False: err stays 1, all maxIter iterations run
    C = torch.rand(12, 50, generator=g) * 30
    a = torch.rand(12, generator=g); a /= a.sum(); b = torch.rand(50, generator=g); b /= b.sum()
    cases.append((a, b, C, 3.0, 37, 1e-9, False))
    # 4, 5: DMCount-shaped (pixel costs at 224, reduction 8, reg 10): 47 points (K in LDS), 300 points (K global)
    cood = torch.arange(0, 224, step=8, dtype=torch.float32).unsqueeze(0) + 4.0
    for n in (47, 300):
        pts = torch.rand(n, 2, generator=g) * 224
        x = pts[:, 0].unsqueeze(1); y = pts[:, 1].unsqueeze(1)
        xd = -2 * torch.matmul(x, cood) + x * x + cood * cood
        yd = -2 * torch.matmul(y, cood) + y * y + cood * cood
        C = (yd.unsqueeze(2) + xd.unsqueeze(1)).view(n, -1)
        b = torch.rand(784, generator=g); b /= b.sum()
        cases.append((torch.ones(n) / n, b, C, 10.0, 100, 1e-9, True))
    for i, (a, b, C, reg, it, thr, log) in enumerate(cases):
        f = io.StringIO()
        with contextlib.redirect_stdout(f):
            r = ref.sinkhorn(a, b, C, reg, maxIter=it, stopThr=thr, log=log)
        msg = f.getvalue().strip()
        P, lg = (r if log else (r, None))
        out[f"a_{i}"], out[f"b_{i}"], out[f"C_{i}"] = a.numpy(), b.numpy(), C.numpy()
        out[f"cfg_{i}"] = np.asarray([reg, it, thr, float(log)], np.float64)
        out[f"P_{i}"] = P.numpy()
        out[f"roll_{i}"] = np.asarray(int(msg.split()[-1]) if msg else 0)
        if log:
            for k in ("u", "v", "alpha", "beta"):
                out[f"{k}_{i}"] = lg[k].numpy()
            out[f"err_{i}"] = np.asarray(lg["err"], np.float32)
    out["n_cases"] = np.asarray(len(cases))
    return out


def loss_extra_case(ref):
    """F1c: DACE/DMCount beyond the default geometry: reduction 16 at 448 (grid 28, cell pitch 16) and
    norm_cood=True (coordinates in [-1, 1]: dense K); per-crop beta and any rollback iteration recorded
    through the reference's own sinkhorn.  (A NaN density cannot reach the rollback there: sinkhorn
    asserts b >= 0 first, bregman_pytorch.py:81.)"""
    out = {}
    calls, restore = _capture_sinkhorn(ref)
    specs = [("r16", 448, 16, False, [0, 30, 300, 4], 303), ("norm", 224, 8, True, [12, 0, 150], 304)]
    for tag, size, red, norm, counts, seed in specs:
        g = np.random.Generator(np.random.PCG64(seed))
        B, h = len(counts), size // red
        points = [(g.random((n, 2)) * size).astype(np.float32) for n in counts]
        density = np.stack([syn.point_map(p, size, size)[None] for p in points])
        pred_class = g.standard_normal((B, 5, h, h)).astype(np.float32)
        pred_density = (g.random((B, 1, h, h)) * 1.5).astype(np.float32)
        pc = torch.tensor(pred_class, requires_grad=True)
        pd = torch.tensor(pred_density, requires_grad=True)
        loss_fn = ref.losses.DACELoss(BINS, red, weight_count_loss=1.0, count_loss="dmcount", input_size=size,
                                      norm_cood=norm)
        del calls[:]
        loss, info = loss_fn(pc, pd, torch.from_numpy(density), [torch.from_numpy(p) for p in points])
        loss.backward()
        flat, offs = pack_points(points)
        beta = np.zeros((B, h * h), np.float32)
        roll = np.zeros(B, np.int32)
        k = 0
        for b, p in enumerate(points):
            if len(p):
                (P, lg), rl = calls[k]
                beta[b] = lg["beta"].numpy()
                roll[b] = rl
                k += 1
        out.update({f"{tag}_size": size, f"{tag}_red": red, f"{tag}_norm": int(norm), f"{tag}_counts": np.asarray(counts),
                    f"{tag}_points": flat, f"{tag}_offsets": offs, f"{tag}_pred_class": pred_class,
                    f"{tag}_pred_density": pred_density, f"{tag}_grad_pred_class": pc.grad.numpy(),
                    f"{tag}_grad_pred_density": pd.grad.numpy(), f"{tag}_beta": beta, f"{tag}_roll": roll})
        for kk, v in info.items():
            out[f"{tag}_info_{kk}"] = v.detach().numpy().reshape(())
    restore()
    return out


def head_case(ref, seed: int = 5):
    """F2: projection + similarity head on a given decoder output."""
    m = build_ref_model(ref, layers=1)
    m._forward_vpt = lambda x: x
    m.reduction = m.encoder_reduction
    m.image_decoder = torch.nn.Identity()
    m.train()
    g = np.random.Generator(np.random.PCG64(seed))
    X = np.maximum(g.standard_normal((2, 768, 28, 28)), 0).astype(np.float32)
    R1 = g.standard_normal((2, 5, 28, 28)).astype(np.float32)
    R2 = g.standard_normal((2, 1, 28, 28)).astype(np.float32)
    xt = torch.tensor(X, requires_grad=True)
    logits, exp = m(xt)
    L = (logits * torch.from_numpy(R1)).sum() + (exp * torch.from_numpy(R2)).sum()
    L.backward()
    return dict(seed=seed, logits=logits.detach().numpy(), exp=exp.detach().numpy(),
                grad_x_sub=xt.grad.numpy()[:, ::7, ::3, ::3], grad_x_norm=np.linalg.norm(xt.grad.numpy()),
                grad_proj_w_sub=m.projection.weight.grad.numpy()[::3, ::3], grad_proj_b=m.projection.bias.grad.numpy(),
                grad_logit_scale=m.logit_scale.grad.numpy(), text_features=m.text_features.numpy())


def e2e_case(ref, layers: int, seed: int = 7, B: int = 2, counts=(37, 5), deep_vpt: bool = True):
    """F3/F4 (F9: deep_vpt=False, the prompt rows carried from block to block, models/clip/model.py:174-178):
    full CLIP-EBC forward + DACE loss + backward on synthetic crops."""
    m = build_ref_model(ref, layers=layers, deep_vpt=deep_vpt)
    nv = layers if deep_vpt else 1
    img, points, density = syn.synthetic_crops(B, 224, seed=seed, counts=list(counts))
    x = torch.from_numpy(img)
    feats = {}
    h = m.image_encoder.ln_post.register_forward_hook(lambda mod, i, o: feats.__setitem__("ln_post", o.detach()))
    m.train()
    logits, exp = m(x)
    h.remove()
    loss_fn = ref.losses.DACELoss(BINS, 8, weight_count_loss=1.0, count_loss="dmcount", input_size=224)
    loss, info = loss_fn(logits, exp, torch.from_numpy(density), [torch.from_numpy(p) for p in points])
    loss.backward()
    out = dict(layers=layers, seed=seed, counts=np.asarray(counts), logits=logits.detach().numpy(),
               exp=exp.detach().numpy(), enc_out_sub=feats["ln_post"].numpy()[:, 1::3, ::2],
               grad_vpt_sub=np.stack([getattr(m, f"vpt_{i}").grad.numpy() for i in range(nv)])[:, :, ::4],
               grad_vpt_norm=np.asarray([np.linalg.norm(getattr(m, f"vpt_{i}").grad.numpy()) for i in range(nv)]),
               deep_vpt=deep_vpt,
               grad_proj_w_sub=m.projection.weight.grad.numpy()[::3, ::3], grad_proj_b=m.projection.bias.grad.numpy(),
               grad_logit_scale=m.logit_scale.grad.numpy(),
               grad_dec_conv1_sub=m.image_decoder[0].conv1.weight.grad.numpy()[::5, ::5],
               grad_dec_conv2_sub=m.image_decoder[0].conv2.weight.grad.numpy()[::5, ::5],
               grad_dec_bn1_w=m.image_decoder[0].bn1.weight.grad.numpy(),
               grad_dec_bn2_b=m.image_decoder[0].bn2.bias.grad.numpy())
    for k, v in info.items():
        out["info_" + k] = v.detach().numpy().reshape(())
    m.eval()
    with torch.no_grad():
        out["exp_eval"] = m(x).numpy()
    return out


ANCHORS_SHA = [0.0, 1.0, 2.0, 3.0, 4.29992]     # configs/reduction_8.json ["4"]["sha"]


def resnet_case(ref, seed: int = 9, B: int = 2, size: int = 448, counts=(60, 3)):
    """F7: clip_resnet50 (config 2 geometry: 448 crops, reduction 8, word prompts, SHA anchors) forward + DACE
    loss + backward in fp32, on the synthetic ResNet-50 weights (ebc_amd.synthetic.resnet50_full_state(0))."""
    torch.manual_seed(0)
    m = ref.model_mod._clip_ebc("resnet50", BINS, ANCHORS_SHA, reduction=8, prompt_type="word", input_size=size)
    sd = syn.resnet50_full_state(0)
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=False)
    assert not unexpected, unexpected
    assert not missing, missing
    m._extract_text_features()
    img, points, density = syn.synthetic_crops(B, size, seed=seed, counts=list(counts))
    x = torch.from_numpy(img)
    feats = {}
    h = m.image_encoder.layer4.register_forward_hook(lambda mod, i, o: feats.__setitem__("enc", o.detach()))
    m.train()
    logits, exp = m(x)
    h.remove()
    loss_fn = ref.losses.DACELoss(BINS, 8, weight_count_loss=1.0, count_loss="dmcount", input_size=size)
    loss, info = loss_fn(logits, exp, torch.from_numpy(density), [torch.from_numpy(p) for p in points])
    loss.backward()
    dec = m.image_decoder[0]
    enc = m.image_encoder
    out = dict(seed=seed, counts=np.asarray(counts), size=size, logits=logits.detach().numpy(),
               exp=exp.detach().numpy(), enc_out_sub=feats["enc"].numpy()[:, ::7, ::3, ::3],
               text_features=m.text_features.numpy(),
               grad_proj_w_sub=m.projection.weight.grad.numpy()[::5, ::7], grad_proj_b=m.projection.bias.grad.numpy(),
               grad_logit_scale=m.logit_scale.grad.numpy(),
               grad_dec_conv1_sub=dec.conv1.weight.grad.numpy()[::9, ::9],
               grad_dec_conv2_sub=dec.conv2.weight.grad.numpy()[::17, ::17],
               grad_dec_conv3_sub=dec.conv3.weight.grad.numpy()[::9, ::9],
               grad_dec_bn1_w=dec.bn1.weight.grad.numpy(), grad_dec_bn2_b=dec.bn2.bias.grad.numpy(),
               grad_dec_bn3_w=dec.bn3.weight.grad.numpy(), grad_dec_bn3_b=dec.bn3.bias.grad.numpy(),
               grad_enc_conv1=enc.conv1.weight.grad.numpy(),
               grad_enc_l4_conv3_sub=enc.layer4[2].conv3.weight.grad.numpy()[::11, ::7],
               grad_enc_l1_bn1_w=enc.layer1[0].bn1.weight.grad.numpy(),
               dec_bn2_running_mean=dec.bn2.running_mean.numpy(), dec_bn3_running_var=dec.bn3.running_var.numpy(),
               state_keys=np.asarray(sorted(m.state_dict().keys())),
               trainable_keys=np.asarray(sorted(k for k, p in m.named_parameters() if p.requires_grad)))
    for k, v in info.items():
        out["info_" + k] = v.detach().numpy().reshape(())
    m.eval()
    with torch.no_grad():
        out["exp_eval"] = m(x).numpy()
    return out


def vgg_case(ref, seed: int = 11, B: int = 2, size: int = 448, counts=(25, 140)):
    """F8: BASELINE configs[0] (vgg19_ae, 448 crops, reduction 8, SHA anchors, DMCount, batch 2 on the CPU):
    the reference's own VGG (models/encoder_decoder/vgg.py:13-41, features = make_vgg_layers(cfg E)) under its
    Classifier (models/model.py:37-75), on ebc_amd.synthetic.vgg19_ae_state(0) (the ImageNet weights are a
    download)."""
    _stub_pkg("models.encoder_decoder", f"{REF}/models/encoder_decoder")
    enc = types.ModuleType("models.encoder")                       # timm-backed encoders: not needed here
    enc._timm_encoder = None
    sys.modules["models.encoder"] = enc
    vgg = _load("models.encoder_decoder.vgg", f"{REF}/models/encoder_decoder/vgg.py")
    mm = _load("models.model", f"{REF}/models/model.py")
    mu = sys.modules["models.utils"]
    torch.manual_seed(0)
    m = mm.Classifier(vgg.VGG(mu.make_vgg_layers(mu.vgg_cfgs["E"]), reduction=8), BINS, ANCHORS_SHA)
    sd = syn.vgg19_ae_state(0)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=True)
    img, points, density = syn.synthetic_crops(B, size, seed=seed, counts=list(counts))
    x = torch.from_numpy(img)
    m.train()
    logits, exp = m(x)
    loss_fn = ref.losses.DACELoss(BINS, 8, weight_count_loss=1.0, count_loss="dmcount", input_size=size)
    loss, info = loss_fn(logits, exp, torch.from_numpy(density), [torch.from_numpy(p) for p in points])
    loss.backward()
    f = m.backbone.features
    out = dict(seed=seed, counts=np.asarray(counts), size=size, logits=logits.detach().numpy(), exp=exp.detach().numpy(),
               state_keys=np.asarray(sorted(m.state_dict().keys())),
               grad_cls_w=m.classifier.weight.grad.numpy(), grad_cls_b=m.classifier.bias.grad.numpy(),
               grad_reg0_sub=m.backbone.reg_layer[0].weight.grad.numpy()[::7, ::9],
               grad_reg2_b=m.backbone.reg_layer[2].bias.grad.numpy(),
               grad_f0_w=f[0].weight.grad.numpy(), grad_f34_sub=f[34].weight.grad.numpy()[::9, ::11],
               grad_f34_b=f[34].bias.grad.numpy())
    for k, v in info.items():
        out["info_" + k] = v.detach().numpy().reshape(())
    m.eval()
    with torch.no_grad():
        out["exp_eval"] = m(x).numpy()
    return out


def sliding_case(ref):
    """F5: sliding-window tiling + overlap averaging with a stub model (utils/eval_utils.py:26-96)."""
    class Stub(torch.nn.Module):
        reduction = 8
        def forward(self, x):
            return torch.nn.functional.avg_pool2d(x.mean(1, keepdim=True).abs(), 8)
    out = {}
    for i, (H, W, win, stride) in enumerate([(500, 700, 224, 224), (500, 700, 224, 112), (224, 448, 224, 224), (232, 240, 224, 112)]):
        # image regenerable: PCG64(11 + i) standard normal [1,3,H,W]
        img = np.random.Generator(np.random.PCG64(11 + i)).standard_normal((1, 3, H, W)).astype(np.float32)
        pred = ref.eval_utils.sliding_window_predict(Stub(), torch.from_numpy(img), win, stride)
        out[f"pred_{i}"] = pred.numpy()
        out[f"cfg_{i}"] = np.asarray([H, W, win, stride])
    return out


def text_case(ref):
    """F6: prompt tokens and text features (synthetic text-tower weights, seed 0)."""
    mc = ref.model_mod
    prompts_w = [sys.modules["models.clip.utils"].format_count(b[0] if b[0] == b[1] else b, "word") for b in BINS]
    prompts_n = [sys.modules["models.clip.utils"].format_count(b[0] if b[0] == b[1] else b, "number") for b in BINS]
    m = build_ref_model(ref, layers=1, prompt_type="word")
    mn = build_ref_model(ref, layers=1, prompt_type="number")
    return dict(prompts_word=np.asarray(prompts_w), prompts_number=np.asarray(prompts_n),
                tokens_word=ref.tokenize(prompts_w).numpy(), tokens_number=ref.tokenize(prompts_n).numpy(),
                text_features_word=m.text_features.numpy(), text_features_number=mn.text_features.numpy())


def prompt_table(ref):
    """CLIP BPE ids of the standard count prompts (data asset for ebc_amd/text.py; the product
    has no tokenizer of its own: clip-ebc_amd/ebc_amd/data/prompt_tokens.json)."""
    import json
    fc = sys.modules["models.clip.utils"].format_count
    prompts = set()
    for t in ("word", "number"):
        for n in range(0, 101):
            prompts.add(fc(n, t))
            prompts.add(fc((n, float("inf")), t))
    prompts = sorted(prompts)
    toks = ref.tokenize(prompts)
    table = {p: [int(x) for x in toks[i].tolist() if x != 0] for i, p in enumerate(prompts)}
    path = os.path.join(REPO, "clip-ebc_amd", "ebc_amd", "data", "prompt_tokens.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(table, f, separators=(",", ":"), sort_keys=True)
    print("wrote", path, len(table), "prompts")


TOKENIZER_TEXTS = [
    "There are more than one hundred and twenty-five people.", "There is 0 person.", "  Crowd   of\tpeople\n  ",
    "A photo of 3,141 pedestrians at 5:30pm!", "CAFÉ crowd: naïve façade, Zürich — 東京 😀", "it's they'll we've I'd",
    "&amp; &lt;tag&gt; html &quot;entities&quot;", "numbers 1234567890 and x1.5e-3", "",
    "a " * 100,
]


def tokenizer_case(ref):
    """F6b: the reference tokenizer (simple_tokenizer.py + tokenize, restated above) on assorted texts,
    including a long one truncated to the context (truncate=True semantics checked separately)."""
    st = sys.modules["models.clip._clip.simple_tokenizer"]
    tok = st.SimpleTokenizer()
    ids = [tok.encode(t) for t in TOKENIZER_TEXTS]
    flat = np.concatenate([np.asarray(i, np.int64) for i in ids]) if any(ids) else np.zeros(0, np.int64)
    offs = np.zeros(len(ids) + 1, np.int64)
    offs[1:] = np.cumsum([len(i) for i in ids])
    return dict(texts=np.asarray(TOKENIZER_TEXTS), ids=flat, offsets=offs)


def bpe_merges():
    """Data asset for ebc_amd/tokenizer.py: the 48894 BPE merges CLIP uses (lines 1..48894 of the reference's
    models/clip/_clip/bpe_simple_vocab_16e6.txt.gz, simple_tokenizer.py's `merges[1:49152-256-2+1]`)."""
    import gzip
    with gzip.open(f"{REF}/models/clip/_clip/bpe_simple_vocab_16e6.txt.gz", "rt", encoding="utf-8") as f:
        lines = f.read().split("\n")
    merges = lines[1:49152 - 256 - 2 + 1]
    path = os.path.join(REPO, "clip-ebc_amd", "ebc_amd", "data", "clip_bpe_merges.txt.gz")
    with gzip.open(path, "wt", encoding="utf-8", compresslevel=9) as f:
        f.write("\n".join(merges) + "\n")
    print("wrote", path, len(merges), "merges", f"{os.path.getsize(path) / 1024:.0f} KiB")


def main():
    torch.set_num_threads(8)
    ref = load_reference()
    if "--only" in sys.argv:                     # e.g. --only f1b,f1c: regenerate just those fixtures
        want = sys.argv[sys.argv.index("--only") + 1].split(",")
        if "f1b" in want:
            save("f1b_sinkhorn.npz", **sinkhorn_case(ref))
        if "f1c" in want:
            save("f1c_loss_extra.npz", **loss_extra_case(ref))
        if "bpe" in want:
            bpe_merges()
        if "f6b" in want:
            save("f6b_tokens.npz", **tokenizer_case(ref))
        if "f7" in want:
            save("f7_resnet50.npz", **resnet_case(ref))
        if "f8" in want:
            save("f8_vgg19_ae.npz", **vgg_case(ref))
        if "f1g" in want:
            loss_grids(ref)
        if "f9" in want:
            save("f9_shallow_vpt_l12.npz", **e2e_case(ref, layers=12, seed=19, counts=(80, 2), deep_vpt=False))
        return
    prompt_table(ref)
    bpe_merges()
    if "--tokens-only" in sys.argv:
        return
    save("f1b_sinkhorn.npz", **sinkhorn_case(ref))
    save("f1c_loss_extra.npz", **loss_extra_case(ref))
    save("f6_text.npz", **text_case(ref))
    save("f6b_tokens.npz", **tokenizer_case(ref))
    save("f1_loss_224.npz", **loss_case(ref, 224, [0, 1, 3, 10, 47, 200, 1000, 25], seed=101))
    save("f1_loss_448.npz", **loss_case(ref, 448, [5, 0, 150, 2000], seed=202))
    save("f2_head.npz", **head_case(ref))
    save("f5_sliding.npz", **sliding_case(ref))
    save("f4_e2e_l2.npz", **e2e_case(ref, layers=2))
    save("f3_e2e_l12.npz", **e2e_case(ref, layers=12))
    save("f7_resnet50.npz", **resnet_case(ref))
    save("f8_vgg19_ae.npz", **vgg_case(ref))
    save("f9_shallow_vpt_l12.npz", **e2e_case(ref, layers=12, seed=19, counts=(80, 2), deep_vpt=False))
    loss_grids(ref)


if __name__ == "__main__":
    main()

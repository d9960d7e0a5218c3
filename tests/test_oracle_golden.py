"""Pin the CPU oracle (oracle/) against the golden fixtures produced by running the reference.

These run on CPU (`-m "not gpu"`).  Tolerances: the reference and the oracle are both fp32 with
different summation orders; the C Sinkhorn accumulates in double.  Forward outputs agree to
~1e-6 relative; gradients are compared in relative L2 norm because the BatchNorm backward of the
decoder cancels a near-constant count-loss gradient (fp32 vs fp64 of the reference itself differs by
~2e-3 max-relative there, see DESIGN.md "Parity tolerances").
"""
import numpy as np
import pytest
import torch

from conftest import ANCHORS_NWPU, BINS, golden, rel_l2, rel_max, split_points
from oracle import ref
from ebc_amd import synthetic as syn


F1G = ["f1g_loss_224_r16.npz", "f1g_loss_224_r32.npz", "f1g_loss_448_r16.npz", "f1g_loss_448_r32.npz",
       "f1g_loss_384_r8.npz", "f1g_loss_512_r8.npz"]


def _red(d):
    return int(d["reduction"]) if "reduction" in d.files else 8


def ref_iters(err):
    """Iterations bregman_pytorch.py:102-126 ran, from its err log (a check every 10; stop at err <= 1e-9)."""
    e = err[err >= 0]
    hit = np.nonzero(e <= 1e-9)[0]
    return 10 * (int(hit[0]) + 1) if len(hit) else 100


@pytest.mark.parametrize("fixture", ["f1_loss_224.npz", "f1_loss_448.npz"] + F1G)
def test_sinkhorn_oracle_matches_reference(fixture):
    d = golden(fixture)
    size = int(d["size"])
    offs = d["offsets"]
    u_ref = d["u_flat"]
    for b, p in enumerate(split_points(d)):
        if len(p) == 0:
            continue
        r = ref.ot_crop(p, d["pred_density"][b, 0], size, _red(d))
        assert rel_max(r["beta"], d["beta"][b]) < 2e-6
        assert rel_max(r["v"], d["v"][b]) < 2e-5
        assert rel_max(r["ot_grad"], d["ot_grad"][b]) < 2e-6
        assert rel_max(r["u"], u_ref[offs[b]:offs[b + 1]]) < 2e-5
        ne = len(r["err"])
        np.testing.assert_allclose(r["err"], d["err"][b][:ne], rtol=1e-4)
        assert abs(r["wd"] - d["wd"][b]) <= 1e-5 * abs(d["wd"][b]) + 1e-6
        assert r["iters"] == ref_iters(d["err"][b]) and not r["rolled_back"]


def test_sinkhorn_oracle_plan_small():
    """P = u K v for crops with n <= 200 (bregman_pytorch.py:140)."""
    d = golden("f1_loss_224.npz")
    lib_pts = split_points(d)
    for b, p in enumerate(lib_pts):
        key = f"P_{b}"
        if key not in d.files or len(p) == 0:
            continue
        r = ref.ot_crop(p, d["pred_density"][b, 0], 224)
        g = 28
        cood = np.arange(0, 224, 8, dtype=np.float32) + 4
        x = p[:, :1]; y = p[:, 1:]
        xd = -2 * (x * cood) + x * x + cood * cood
        yd = -2 * (y * cood) + y * y + cood * cood
        K = np.exp((yd[:, :, None] + xd[:, None, :]).reshape(len(p), -1) / -10.0)
        P = r["u"][:, None] * K * r["v"][None, :]
        assert rel_l2(P, d[key]) < 1e-5


@pytest.mark.parametrize("fixture", ["f1_loss_224.npz", "f1_loss_448.npz"] + F1G)
def test_dace_loss_oracle_matches_reference(fixture):
    d = golden(fixture)
    size = int(d["size"])
    pts = split_points(d)
    dens = np.stack([syn.point_map(p, size, size)[None] for p in pts])
    pc = torch.tensor(d["pred_class"], requires_grad=True)
    pd = torch.tensor(d["pred_density"], requires_grad=True)
    loss, info = ref.dace_loss(pc, pd, torch.from_numpy(dens), pts, BINS, reduction=_red(d), input_size=size)
    loss.backward()
    for k in ("loss", "tv_loss", "count_loss", "ce_loss"):
        assert abs(float(info[k]) - float(d["info_" + k])) <= 1e-5 * abs(float(d["info_" + k])) + 1e-4, k
    assert abs(float(info["ot_loss"])) < 1e-3 and abs(float(d["info_ot_loss"])) < 1e-3   # ~0 by construction
    assert rel_max(pc.grad.numpy(), d["grad_pred_class"]) < 1e-5
    assert rel_max(pd.grad.numpy(), d["grad_pred_density"]) < 1e-5


def test_head_oracle_matches_reference():
    d = golden("f2_head.npz")
    g = np.random.Generator(np.random.PCG64(int(d["seed"])))
    X = np.maximum(g.standard_normal((2, 768, 28, 28)), 0).astype(np.float32)
    R1 = g.standard_normal((2, 5, 28, 28)).astype(np.float32)
    R2 = g.standard_normal((2, 1, 28, 28)).astype(np.float32)
    p = ref.params_from_state(syn.trainable_state(0, layers=1))
    xt = torch.tensor(X, requires_grad=True)
    logits, exp = ref.head(p, xt, torch.from_numpy(d["text_features"]), ANCHORS_NWPU)
    ((logits * torch.from_numpy(R1)).sum() + (exp * torch.from_numpy(R2)).sum()).backward()
    assert rel_max(logits.detach().numpy(), d["logits"]) < 1e-5
    assert rel_max(exp.detach().numpy(), d["exp"]) < 1e-5
    assert rel_l2(xt.grad.numpy()[:, ::7, ::3, ::3], d["grad_x_sub"]) < 1e-5
    assert rel_l2(p["projection.weight"].grad.numpy()[::3, ::3], d["grad_proj_w_sub"]) < 1e-5
    assert rel_l2(p["projection.bias"].grad.numpy(), d["grad_proj_b"]) < 1e-5
    assert abs(float(p["logit_scale"].grad) - float(d["grad_logit_scale"])) < 1e-4 * abs(float(d["grad_logit_scale"]))


@pytest.mark.parametrize("fixture", ["f4_e2e_l2.npz", "f3_e2e_l12.npz", "f9_shallow_vpt_l12.npz"])
def test_e2e_oracle_matches_reference(fixture):
    d = golden(fixture)
    L = int(d["layers"])
    deep = bool(d["deep_vpt"]) if "deep_vpt" in d else True
    nv = L if deep else 1
    txt = torch.from_numpy(golden("f6_text.npz")["text_features_word"])
    sd = syn.full_state(0, layers=L, include_text=False)
    if not deep:                                    # shallow VPT: vpt_0 only
        sd = {k: v for k, v in sd.items() if not (k.startswith("vpt_") and k != "vpt_0")}
    p = ref.params_from_state(sd)
    img, pts, dens = syn.synthetic_crops(2, 224, seed=int(d["seed"]), counts=list(d["counts"]))
    logits, exp, feats = ref.forward(p, torch.from_numpy(img), txt, ANCHORS_NWPU, L, deep_vpt=deep)
    loss, info = ref.dace_loss(logits, exp, torch.from_numpy(dens), pts, BINS)
    loss.backward()
    assert rel_max(logits.detach().numpy(), d["logits"]) < 1e-5
    assert rel_max(exp.detach().numpy(), d["exp"]) < 1e-5
    enc = feats.detach().permute(0, 2, 3, 1).reshape(2, 196, 768).numpy()[:, ::3, ::2]
    assert rel_max(enc, d["enc_out_sub"]) < 1e-5
    for k in ("loss", "tv_loss", "count_loss", "ce_loss"):
        assert abs(float(info[k]) - float(d["info_" + k])) <= 1e-5 * abs(float(d["info_" + k])), k
    gv = np.stack([p[f"vpt_{i}"].grad.numpy() for i in range(nv)])
    assert rel_l2(gv[:, :, ::4], d["grad_vpt_sub"]) < 5e-4   # reference fp32 vs fp64: 2e-4
    assert rel_l2(p["projection.weight"].grad.numpy()[::3, ::3], d["grad_proj_w_sub"]) < 1e-4
    assert rel_l2(p["image_decoder.0.conv1.weight"].grad.numpy()[::5, ::5], d["grad_dec_conv1_sub"]) < 5e-3
    assert abs(float(p["logit_scale"].grad) - float(d["grad_logit_scale"])) < 1e-4 * abs(float(d["grad_logit_scale"]))


def test_sliding_window_fixture_shapes():
    """F5 fixture sanity (the assembler itself is tested in test_eval.py)."""
    d = golden("f5_sliding.npz")
    for i in range(4):
        H, W, win, stride = d[f"cfg_{i}"]
        assert d[f"pred_{i}"].shape == (1, 1, H // 8, W // 8)


# ------------------------------------------------------------------ F1b / F1c (general sinkhorn, geometry)
def plan_close(P, Pref, tol):
    """Same non-finite pattern (a negative cost makes K = inf: P holds inf / nan there), finite parts close."""
    P, Pref = np.asarray(P, np.float64), np.asarray(Pref, np.float64)
    assert np.array_equal(np.isnan(P), np.isnan(Pref)) and np.array_equal(np.isinf(P), np.isinf(Pref))
    m = np.isfinite(Pref)
    return rel_l2(P[m], Pref[m]) < tol


def _f1b_case(d, i):
    reg, it, thr, log = (float(x) for x in d[f"cfg_{i}"])
    return d[f"a_{i}"], d[f"b_{i}"], d[f"C_{i}"], reg, int(it), thr, bool(log)


def test_dense_sinkhorn_oracle_matches_reference():
    """oracle.sinkhorn (C) vs the reference's own sinkhorn on F1b: early stop, rollback at iterations 1
    and 2 (the returned u, v are the pre-failure pair), log=False, DMCount-shaped crops."""
    d = golden("f1b_sinkhorn.npz")
    for i in range(int(d["n_cases"])):
        a, b, C, reg, it, thr, log = _f1b_case(d, i)
        r = ref.sinkhorn(a, b, C, reg, it, thr, log=log)
        assert r["roll"] == int(d[f"roll_{i}"]), (i, r["roll"])
        assert plan_close(r["P"], d[f"P_{i}"], 1e-5), i
        if log:
            for k in ("u", "v", "alpha", "beta"):
                assert rel_max(r[k], d[f"{k}_{i}"]) < 5e-5, (i, k)
            np.testing.assert_allclose(r["err"], d[f"err_{i}"], rtol=1e-3, atol=1e-12)


@pytest.mark.parametrize("tag", ["r16", "norm"])
def test_dace_loss_oracle_matches_reference_extra_geometry(tag):
    """Reduction 16 at 448 (cell pitch 16) and norm_cood=True (F1c)."""
    d = golden("f1c_loss_extra.npz")
    size, red, norm = int(d[f"{tag}_size"]), int(d[f"{tag}_red"]), bool(d[f"{tag}_norm"])
    offs, flat = d[f"{tag}_offsets"], d[f"{tag}_points"]
    pts = [flat[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    dens = np.stack([syn.point_map(p, size, size)[None] for p in pts])
    pc = torch.tensor(d[f"{tag}_pred_class"], requires_grad=True)
    pd = torch.tensor(d[f"{tag}_pred_density"], requires_grad=True)
    loss, info = ref.dace_loss(pc, pd, torch.from_numpy(dens), pts, BINS, reduction=red, input_size=size,
                               norm_cood=norm)
    loss.backward()
    for k in ("loss", "tv_loss", "count_loss", "ce_loss"):
        ref_v = float(d[f"{tag}_info_{k}"])
        assert abs(float(info[k]) - ref_v) <= 1e-5 * abs(ref_v) + 1e-5, (k, float(info[k]), ref_v)
    assert rel_max(pc.grad.numpy(), d[f"{tag}_grad_pred_class"]) < 1e-5
    assert rel_l2(pd.grad.numpy(), d[f"{tag}_grad_pred_density"]) < 1e-4
    for b, p in enumerate(pts):
        if len(p):
            r = ref.ot_crop(p, d[f"{tag}_pred_density"][b, 0], size, red, norm_cood=norm)
            assert rel_max(r["beta"], d[f"{tag}_beta"][b]) < 1e-4, (tag, b)
            assert not r["rolled_back"] and int(d[f"{tag}_roll"][b]) == 0


def test_resnet50_oracle_matches_reference():
    """F7: the oracle's functional clip_resnet50 restatement (oracle/ref.py resnet_forward) against the
    reference's own fp32 outputs on the same synthetic weights and crops."""
    import torch
    from ebc_amd import synthetic as syn
    from oracle import ref
    d = golden("f7_resnet50.npz")
    p = ref.resnet_params_from_state(syn.resnet50_full_state(0, include_text=False))
    img, pts, dens = syn.synthetic_crops(2, int(d["size"]), seed=int(d["seed"]), counts=list(d["counts"]))
    logits, exp, feats = ref.resnet_forward(p, torch.from_numpy(img), torch.from_numpy(d["text_features"]),
                                            [0.0, 1.0, 2.0, 3.0, 4.29992])
    assert rel_l2(feats.detach().numpy()[:, ::7, ::3, ::3], d["enc_out_sub"]) < 1e-4
    assert rel_l2(logits.detach().numpy(), d["logits"]) < 1e-4
    loss, info = ref.dace_loss(logits, exp, torch.from_numpy(dens), pts, BINS, input_size=int(d["size"]))
    assert abs(loss.item() - float(d["info_loss"])) < 1e-4 * abs(float(d["info_loss"]))
    loss.backward()
    assert rel_l2(p["image_decoder.0.conv3.weight"].grad.numpy()[::9, ::9], d["grad_dec_conv3_sub"]) < 1e-3
    assert rel_l2(p["image_encoder.conv1.weight"].grad.numpy(), d["grad_enc_conv1"]) < 1e-3

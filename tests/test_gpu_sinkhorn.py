"""GPU parity of the Sinkhorn pieces: the general `sinkhorn()` (ebc_sinkhorn) against the reference's
own outputs (F1b: early stop, NaN/Inf rollback at iterations 1 and 2, log=False, DMCount-shaped crops with
K in LDS and in global memory), and the fused loss kernel's internals (beta, iteration status, err of
the last check) against F1 / F1c and the C oracle, including reduction 16, norm_cood and a rollback."""
import io
import contextlib

import numpy as np
import pytest
import torch

from conftest import BINS, golden, rel_l2, rel_max, split_points
from oracle import ref
from ebc_amd import synthetic as syn

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _plan_close(P, Pref, tol):
    P, Pref = np.asarray(P, np.float64), np.asarray(Pref, np.float64)
    assert np.array_equal(np.isnan(P), np.isnan(Pref)) and np.array_equal(np.isinf(P), np.isinf(Pref))
    m = np.isfinite(Pref)
    return rel_l2(P[m], Pref[m]) < tol


@pytest.mark.parametrize("i", range(6))
def test_sinkhorn_matches_reference_f1b(i):
    from ebc_amd.losses import sinkhorn
    d = golden("f1b_sinkhorn.npz")
    reg, it, thr, log = (float(x) for x in d[f"cfg_{i}"])
    a, b, C = (torch.from_numpy(d[f"{k}_{i}"]).to(DEV) for k in "abC")
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        r = sinkhorn(a, b, C, reg, maxIter=int(it), stopThr=thr, log=bool(log))
    roll = int(d[f"roll_{i}"])
    msg = out.getvalue().strip()
    assert (msg == f"Warning: numerical errors at iteration {roll}") if roll else msg == "", msg
    P, lg = r if log else (r, None)
    # tolerance: K and the products round differently from torch's CPU matmul (fp32, ~1e-7 per op)
    assert _plan_close(P.cpu().numpy(), d[f"P_{i}"], 2e-5)
    if log:
        for k in ("u", "v", "alpha", "beta"):
            assert rel_max(lg[k].cpu().numpy(), d[f"{k}_{i}"]) < 1e-4, k
        assert len(lg["err"]) == len(d[f"err_{i}"])
        np.testing.assert_allclose(lg["err"], d[f"err_{i}"], rtol=2e-3, atol=1e-12)


def test_sinkhorn_without_log_runs_every_iteration():
    """log=False: err is never updated (bregman_pytorch.py:117), so maxIter iterations run even when a
    loose stopThr would stop the logged run early; P equals the logged run's P at the same iteration."""
    from ebc_amd.losses import sinkhorn
    d = golden("f1b_sinkhorn.npz")
    a, b, C = (torch.from_numpy(d[f"{k}_0"]).to(DEV) for k in "abC")
    P_log, lg = sinkhorn(a, b, C, 5.0, maxIter=10, stopThr=1e-4, log=True)     # stops at the first check
    P_nolog = sinkhorn(a, b, C, 5.0, maxIter=10, stopThr=1e-4, log=False)
    np.testing.assert_array_equal(P_log.cpu().numpy(), P_nolog.cpu().numpy())
    o = ref.sinkhorn(d["a_0"], d["b_0"], d["C_0"], 5.0, 25, 1e-4, log=False)
    P25 = sinkhorn(a, b, C, 5.0, maxIter=25, stopThr=1e-4, log=False)
    assert o["iters"] == 25 and rel_l2(P25.cpu().numpy(), o["P"]) < 2e-5


def _dace(pc, pd, dens, pts, size, red=8, norm=False, keep=True):
    from ebc_amd.losses import DACELoss
    fn = DACELoss(BINS, red, weight_count_loss=1.0, count_loss="dmcount", input_size=size, norm_cood=norm,
                  keep_internals=keep)
    pct = torch.tensor(pc, device=DEV, requires_grad=True)
    pdt = torch.tensor(pd, device=DEV, requires_grad=True)
    loss, info = fn(pct, pdt, torch.from_numpy(dens).to(DEV), [torch.from_numpy(p).to(DEV) for p in pts])
    loss.backward()
    torch.cuda.synchronize()
    return fn, {k: float(v) for k, v in info.items()}, pct.grad.cpu().numpy(), pdt.grad.cpu().numpy()


F1G = ["f1g_loss_224_r16.npz", "f1g_loss_224_r32.npz", "f1g_loss_448_r16.npz", "f1g_loss_448_r32.npz",
       "f1g_loss_384_r8.npz", "f1g_loss_512_r8.npz"]


def _ref_iters(err):
    e = err[err >= 0]
    hit = np.nonzero(e <= 1e-9)[0]
    return 10 * (int(hit[0]) + 1) if len(hit) else 100


@pytest.mark.parametrize("fixture", ["f1_loss_224.npz", "f1_loss_448.npz"] + F1G)
def test_fused_kernel_internals_match_reference(fixture):
    """beta, the iteration count (the reference's, from its err log: 100 unless an err check reaches 1e-9) and
    the last err check of every crop, as the reference's sinkhorn log holds them (F1, F1g)."""
    d = golden(fixture)
    size = int(d["size"])
    red = int(d["reduction"]) if "reduction" in d.files else 8
    pts = split_points(d)
    dens = np.stack([syn.point_map(p, size, size)[None] for p in pts])
    fn, _, _, _ = _dace(d["pred_class"], d["pred_density"], dens, pts, size, red=red)
    it = fn.count_loss_fn.internals
    beta, status, err_last = it.beta.cpu().numpy(), it.status.cpu().numpy(), it.err_last.cpu().numpy()
    for b, p in enumerate(pts):
        if len(p) == 0:
            assert status[b] == 0 and not beta[b].any()
            continue
        assert status[b] == _ref_iters(d["err"][b]), (b, status[b])
        assert rel_max(beta[b], d["beta"][b]) < 1e-4, b
        e_ref = d["err"][b][d["err"][b] >= 0][-1]
        assert abs(err_last[b] - e_ref) <= 2e-3 * e_ref + 1e-12, (b, err_last[b], e_ref)
        assert abs(float(it.wd[b]) - float(d["wd"][b])) <= 1e-4 * abs(float(d["wd"][b])) + 1e-4


@pytest.mark.parametrize("tag", ["r16", "norm"])
def test_fused_kernel_extra_geometry_matches_reference(tag):
    """Reduction 16 at 448 (grid 28, cell pitch 16) and norm_cood=True (dense K: the windowed paths fall
    back to the dense one), against the reference's outputs (F1c)."""
    d = golden("f1c_loss_extra.npz")
    size, red, norm = int(d[f"{tag}_size"]), int(d[f"{tag}_red"]), bool(d[f"{tag}_norm"])
    offs, flat = d[f"{tag}_offsets"], d[f"{tag}_points"]
    pts = [flat[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
    dens = np.stack([syn.point_map(p, size, size)[None] for p in pts])
    fn, info, gc, gd = _dace(d[f"{tag}_pred_class"], d[f"{tag}_pred_density"], dens, pts, size, red, norm)
    for k in ("loss", "tv_loss", "count_loss", "ce_loss"):
        r = float(d[f"{tag}_info_{k}"])
        assert abs(info[k] - r) <= 2e-5 * abs(r) + 1e-4, (k, info[k], r)
    assert rel_max(gc, d[f"{tag}_grad_pred_class"]) < 1e-5
    assert rel_l2(gd, d[f"{tag}_grad_pred_density"]) < 1e-4
    beta = fn.count_loss_fn.internals.beta.cpu().numpy()
    for b, p in enumerate(pts):
        if len(p):
            assert rel_max(beta[b], d[f"{tag}_beta"][b]) < 2e-4, (tag, b)


def test_fused_kernel_rollback_on_nan_crop():
    """A NaN in one crop's density: its Sinkhorn fails at iteration 1 and keeps the initial (u, v)
    (bregman_pytorch.py:111-115), status = -1 and beta = reg * log(1/784 + 1e-16); the C oracle runs the
    same loop.  (The reference itself asserts b >= 0 first, :81, so no reference fixture exists for this.)
    The other crops are unaffected."""
    g = np.random.Generator(np.random.PCG64(77))
    counts = [15, 30, 8]
    pts = [(g.random((n, 2)) * 224).astype(np.float32) for n in counts]
    dens = np.stack([syn.point_map(p, 224, 224)[None] for p in pts])
    pc = g.standard_normal((3, 5, 28, 28)).astype(np.float32)
    pd = (g.random((3, 1, 28, 28)) * 1.5).astype(np.float32)
    pd_nan = pd.copy()
    pd_nan[1, 0, 3, 5] = np.nan
    fn, _, _, gd = _dace(pc, pd_nan, dens, pts, 224)
    it = fn.count_loss_fn.internals
    status, beta = it.status.cpu().numpy(), it.beta.cpu().numpy()
    assert status[1] == -1 and status[0] == 100 and status[2] == 100
    o = ref.ot_crop(pts[1], pd_nan[1, 0], 224)
    assert o["rolled_back"] and o["iters"] == 1
    np.testing.assert_allclose(beta[1], o["beta"], rtol=1e-6)
    np.testing.assert_allclose(beta[1], 10.0 * np.log(np.float32(1 / 784) + 1e-16), rtol=1e-6)
    fn2, _, _, gd2 = _dace(pc, pd, dens, pts, 224)
    for b in (0, 2):
        np.testing.assert_allclose(beta[b], fn2.count_loss_fn.internals.beta.cpu().numpy()[b], rtol=1e-6)


def test_otloss_matches_oracle():
    """OTLoss.forward (dm_loss.py:38-79): loss, wd, ot_obj_values and the gradient w.r.t. pred_density."""
    from ebc_amd.losses import OTLoss
    g = np.random.Generator(np.random.PCG64(78))
    counts = [0, 12, 140, 3]
    pts = [(g.random((n, 2)) * 224).astype(np.float32) for n in counts]
    pd = (g.random((4, 1, 28, 28)) * 1.5).astype(np.float32)
    pdt = torch.tensor(pd, device=DEV, requires_grad=True)
    cnt = pdt.detach().view(4, -1).sum(1).view(-1, 1, 1, 1)
    loss, wd, obj = OTLoss(224, 8, False)(pdt, pdt.detach() / (cnt + 1e-8), [torch.from_numpy(p).to(DEV) for p in pts])
    loss.backward()
    o_loss, o_wd, o_obj, o_grad = 0.0, 0.0, 0.0, np.zeros_like(pd)
    for b, p in enumerate(pts):
        if len(p):
            r = ref.ot_crop(p, pd[b, 0], 224)
            o_loss += r["loss"]; o_wd += r["wd"]; o_obj += r["ot_obj"]; o_grad[b, 0] = r["ot_grad"].reshape(28, 28)
    assert abs(float(loss) - o_loss) <= 1e-4 * max(1.0, abs(o_loss))
    assert abs(wd - o_wd) <= 1e-4 * abs(o_wd)
    assert abs(float(obj) - o_obj) <= 1e-4 * abs(o_obj) + 1e-4
    assert rel_l2(pdt.grad.cpu().numpy(), o_grad) < 1e-4
    # a differently normalised marginal is refused (the kernel forms it from pred_density itself)
    with pytest.raises(ValueError):
        OTLoss(224, 8, False)(pdt, pdt.detach() / (2 * cnt + 1e-8), [torch.from_numpy(p).to(DEV) for p in pts])

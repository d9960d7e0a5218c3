"""GPU parity: fused DACE/DMCount kernel vs the golden fixtures and the CPU oracle."""
import numpy as np
import pytest
import torch

from conftest import BINS, golden, rel_l2, rel_max, split_points
from oracle import ref
from ebc_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _run(pred_class, pred_density, target_density, points, size, count_loss="dmcount", reduced=False, red=8):
    from ebc_amd.losses import DACELoss
    dev = torch.device("cuda:0")
    fn = DACELoss(BINS, red, weight_count_loss=1.0, count_loss=count_loss, input_size=size)
    pc = torch.tensor(pred_class, device=dev, requires_grad=True)
    pd = torch.tensor(pred_density, device=dev, requires_grad=True)
    td = torch.from_numpy(target_density).to(dev)
    if reduced:
        td = ref.reshape_density(td, red)
    loss, info = fn(pc, pd, td, [torch.from_numpy(p).to(dev) for p in points])
    loss.backward()
    torch.cuda.synchronize()
    return float(loss), {k: float(v) for k, v in info.items()}, pc.grad.cpu().numpy(), pd.grad.cpu().numpy()


F1G = ["f1g_loss_224_r16.npz", "f1g_loss_224_r32.npz", "f1g_loss_448_r16.npz", "f1g_loss_448_r32.npz",
       "f1g_loss_384_r8.npz", "f1g_loss_512_r8.npz"]


@pytest.mark.parametrize("fixture", ["f1_loss_224.npz", "f1_loss_448.npz"] + F1G)
def test_dace_kernel_matches_reference_fixture(fixture):
    """Every density grid the reference allows up to 64 (reduction 8 / 16 / 32; grids 7, 14, 28, 48, 56, 64 run
    on padded LDS grids 8 / 16 / 28 / 48 / 56 / 64 with dead cells)."""
    d = golden(fixture)
    size = int(d["size"])
    red = int(d["reduction"]) if "reduction" in d.files else 8
    pts = split_points(d)
    dens = np.stack([syn.point_map(p, size, size)[None] for p in pts])
    loss, info, gc, gd = _run(d["pred_class"], d["pred_density"], dens, pts, size, red=red)
    for k in ("loss", "tv_loss", "count_loss", "ce_loss"):
        assert abs(info[k] - float(d["info_" + k])) <= 2e-5 * abs(float(d["info_" + k])) + 1e-4, (k, info[k])
    assert abs(info["ot_loss"]) < 1e-3
    assert rel_max(gc, d["grad_pred_class"]) < 1e-5
    # OT gradient through the separable kernel: K rounding differs from exp(C/-reg) by ~ulp(C)/reg
    assert rel_max(gd, d["grad_pred_density"]) < 1e-4
    assert rel_l2(gd, d["grad_pred_density"]) < 2e-5


def _random_batch(B, size, seed, counts=None):
    g = np.random.Generator(np.random.PCG64(seed))
    h = size // 8
    if counts is None:
        counts = np.clip(np.floor(g.lognormal(np.log(20.0), 1.2, B)), 0, 2048).astype(int).tolist()
    pts = [(g.random((n, 2)) * size).astype(np.float32) for n in counts]
    dens = np.stack([syn.point_map(p, size, size)[None] for p in pts])
    pcl = g.standard_normal((B, 5, h, h)).astype(np.float32)
    pde = (g.random((B, 1, h, h)) * 2.0).astype(np.float32)
    return pcl, pde, dens, pts


def _oracle(pcl, pde, dens, pts, size, count_loss="dmcount"):
    pc = torch.tensor(pcl, requires_grad=True)
    pd = torch.tensor(pde, requires_grad=True)
    if count_loss == "dmcount":
        loss, info = ref.dace_loss(pc, pd, torch.from_numpy(dens), pts, BINS, input_size=size)
    else:
        td = ref.reshape_density(torch.from_numpy(dens), 8)
        ce = torch.nn.functional.cross_entropy(pc, ref.bin_count(td, BINS), reduction="none").sum(dim=(-1, -2)).mean()
        diff = pd - td
        cnt = (diff.abs() if count_loss == "mae" else diff * diff).sum(dim=(-1, -2, -3)).mean()
        loss = ce + cnt
        info = {"loss": loss, "ce_loss": ce, f"{count_loss}_loss": cnt}
    loss.backward()
    return float(loss), {k: float(v) for k, v in info.items()}, pc.grad.numpy(), pd.grad.numpy()


@pytest.mark.parametrize("size,counts", [
    (224, None),                                  # lognormal ragged batch, 16 crops
    (224, [0, 0, 0, 0]),                          # empty crops: OT skipped (dm_loss.py:49)
    (224, [600, 1, 2048, 473, 474, 475, 3]),      # above the full-row LDS capacity (468 points)
    (224, [1202, 1203, 582, 583, 5]),             # g = 28 LDS capacities: compact rows 1202, full rows 582
    (448, [0, 130, 127, 129, 900, 2]),            # g = 56
    (448, [722, 723, 183, 184]),                  # g = 56 LDS capacities: compact rows 722, full rows 183
])
def test_dace_kernel_matches_oracle(size, counts):
    B = 16 if counts is None else len(counts)
    pcl, pde, dens, pts = _random_batch(B, size, seed=3 + size, counts=counts)
    loss, info, gc, gd = _run(pcl, pde, dens, pts, size)
    oloss, oinfo, ogc, ogd = _oracle(pcl, pde, dens, pts, size)
    for k in ("loss", "tv_loss", "count_loss", "ce_loss"):
        assert abs(info[k] - oinfo[k]) <= 2e-5 * abs(oinfo[k]) + 1e-4, (k, info[k], oinfo[k])
    assert rel_max(gc, ogc) < 1e-5
    assert rel_l2(gd, ogd) < 2e-5


@pytest.mark.parametrize("mode", ["mae", "mse"])
def test_dace_kernel_count_modes(mode):
    pcl, pde, dens, pts = _random_batch(6, 224, seed=9)
    loss, info, gc, gd = _run(pcl, pde, dens, pts, 224, count_loss=mode)
    oloss, oinfo, ogc, ogd = _oracle(pcl, pde, dens, pts, 224, count_loss=mode)
    assert abs(loss - oloss) <= 1e-5 * abs(oloss)
    assert abs(info[f"{mode}_loss"] - oinfo[f"{mode}_loss"]) <= 1e-5 * abs(oinfo[f"{mode}_loss"])
    assert rel_max(gc, ogc) < 1e-5 and rel_max(gd, ogd) < 1e-5


def test_dace_kernel_reduced_target_and_dmloss():
    from ebc_amd.losses import DMLoss
    pcl, pde, dens, pts = _random_batch(5, 224, seed=12)
    a = _run(pcl, pde, dens, pts, 224)
    b = _run(pcl, pde, dens, pts, 224, reduced=True)
    assert a[0] == pytest.approx(b[0], rel=1e-6)
    np.testing.assert_allclose(a[3], b[3], rtol=1e-6, atol=1e-9)
    dev = torch.device("cuda:0")
    pd = torch.tensor(pde, device=dev, requires_grad=True)
    loss, info = DMLoss(224, 8)(pd, torch.from_numpy(dens).to(dev), [torch.from_numpy(p).to(dev) for p in pts])
    assert float(loss) == pytest.approx(a[1]["loss"] - a[1]["ce_loss"], rel=1e-5)


def test_dace_kernel_host_and_device_label_metadata_agree():
    """Up to 64 crops the crop offsets / order travel as kernel arguments (ebc_dace_loss_h); 70 crops take the device
    tensors (ebc_dace_loss).  Each crop runs in its own workgroup on the same arithmetic, so the per-crop statistics
    (CE, TV, count, OT, Wasserstein distance, iterations) of the 70-crop batch equal those of its two 35-crop halves
    bit for bit; packed label views (one buffer, the second half) give the same as separate tensors."""
    from ebc_amd.losses import DACELoss
    dev = torch.device("cuda:0")
    B, size = 70, 224
    img, pts, dens = syn.synthetic_crops(B, size, seed=123)
    g = torch.Generator().manual_seed(9)
    pc = torch.randn(B, len(BINS), 28, 28, generator=g).to(dev)
    pd = torch.rand(B, 1, 28, 28, generator=g).to(dev)
    td = torch.from_numpy(dens).to(dev)
    fn = DACELoss(BINS, 8, count_loss="dmcount", input_size=size)

    def run(sl, packed=False):
        a, b = pc[sl].clone().requires_grad_(), pd[sl].clone().requires_grad_()
        if packed:
            buf = torch.from_numpy(np.concatenate([p.reshape(-1, 2) for p in pts[sl]], 0).astype(np.float32)).to(dev)
            views, o = [], 0
            for p in pts[sl]:
                views.append(buf[o:o + len(p)])
                o += len(p)
        else:
            views = [torch.from_numpy(p).to(dev) for p in pts[sl]]
        loss, _ = fn(a, b, td[sl], views)
        loss.backward()
        return fn.last_stats.clone(), a.grad.clone(), b.grad.clone()
    full = run(slice(0, B))
    halves = [run(slice(0, 35)), run(slice(35, B), packed=True)]
    st = torch.cat([h[0] for h in halves])
    assert torch.equal(full[0][:, :6], st[:, :6])          # per-crop ce, tv*n, count, ot, wd, iterations

"""GPU: training-crop augmentation (ebc_augment_crops / ebc_point_map) against the
CPU oracle (oracle/augment_ref.py): crop + antialiased bicubic resize pinned by torch's own
F.interpolate (what the reference's TF.resize calls), flip / noise / normalise exact, ColorJitter and
GaussianBlur against the restated torchvision algorithms (parity unpinned against torchvision itself:
it is not importable here).  Tolerances: 2e-5 absolute on [0, 1] pixels for the resize paths
(f32 tap order), 1e-4 absolute after normalisation (values up to ~2.6) with jitter and blur."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _images(shapes, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.rand(3, h, w, generator=g) for h, w in shapes]


def _plans(aug, shapes, n_per, seed):
    torch.manual_seed(seed)
    plans, labels = [], []
    for i, (h, w) in enumerate(shapes):
        for _ in range(n_per):
            lab = torch.rand(50, 2) * torch.tensor([w, h], dtype=torch.float32)
            p, l = aug.plan_crop(i, h, w, lab)
            plans.append(p)
            labels.append(l)
    return plans, labels


@pytest.mark.parametrize("scale", [(1.0, 1.0), (0.75, 1.25), (1.0, 2.0)])
def test_crop_resize_flip_matches_torch_interpolate(scale):
    from ebc_amd.transforms import CropAugment
    from oracle import augment_ref as ref
    shapes = [(300, 400), (512, 700), (230, 260)]
    aug = CropAugment(224, *scale, jitter_prob=0.0, blur_prob=0.0, noise_prob=0.0)
    imgs = _images(shapes, 1)
    plans, _ = _plans(aug, shapes, 3, seed=5)
    out = aug.apply([x.cuda() for x in imgs], plans, normalize=False).cpu()
    exp = ref.apply_plans(imgs, plans, (224, 224), normalize=False)
    assert out.shape == exp.shape == (9, 3, 224, 224)
    assert any(p.flip for p in plans) and not all(p.flip for p in plans)
    assert (out - exp).abs().max().item() < 2e-5


def test_small_image_pre_resize_branch():
    """RandomResizedCrop's resize-then-crop branch (crop larger than the image, transforms.py:155-162)."""
    from ebc_amd.transforms import CropAugment
    from oracle import augment_ref as ref
    shapes = [(200, 180), (150, 400)]
    aug = CropAugment(224, 1.0, 2.0, jitter_prob=0.0, blur_prob=0.0, noise_prob=0.0)
    imgs = _images(shapes, 2)
    plans, labels = _plans(aug, shapes, 2, seed=7)
    assert all(p.pre_resize is not None for p in plans)
    out = aug.apply([x.cuda() for x in imgs], plans, normalize=False).cpu()
    exp = ref.apply_plans(imgs, plans, (224, 224), normalize=False)
    assert (out - exp).abs().max().item() < 2e-5
    for l in labels:
        assert len(l) == 0 or (float(l.min()) >= 0 and float(l.max()) <= 223)


@pytest.mark.parametrize("probs,hue", [((1.0, 0.0, 0.0), 0.0), ((0.0, 1.0, 0.0), 0.0), ((0.0, 0.0, 1.0), 0.0),
                                       ((1.0, 1.0, 1.0), 0.0), ((0.2, 0.2, 0.5), 0.0), ((1.0, 0.0, 0.0), 0.3),
                                       ((1.0, 1.0, 1.0), 0.1)])
def test_full_pipeline_matches_oracle(probs, hue):
    from ebc_amd.transforms import CropAugment
    from oracle import augment_ref as ref
    shapes = [(480, 640), (300, 300), (768, 1024)]
    aug = CropAugment(224, 1.0, 2.0, brightness=0.4, contrast=0.4, saturation=0.4, hue=hue, saltiness=0.02,
                      spiciness=0.02, jitter_prob=probs[0], blur_prob=probs[1], noise_prob=probs[2])
    imgs = _images(shapes, 3)
    plans, _ = _plans(aug, shapes, 4, seed=11)
    out = aug.apply([x.cuda() for x in imgs], plans).cpu()
    exp = ref.apply_plans(imgs, plans, (224, 224), saltiness=0.02, spiciness=0.02)
    if probs[0] == 1.0:
        assert all(len(p.jitter) == (4 if hue else 3) for p in plans)
    if probs[2] == 1.0:                                    # the noise really fires (both salt and pepper)
        raw = aug.apply([x.cuda() for x in imgs], plans, normalize=False).cpu()
        assert (raw == 1.0).any() and (raw == 0.0).any()
    assert torch.isfinite(out).all()
    assert (out - exp).abs().max().item() < 1e-4


def test_density_map_matches_reference():
    from ebc_amd.transforms import generate_density_map
    from oracle import augment_ref as ref
    g = torch.Generator().manual_seed(4)
    pts = [torch.rand(n, 2, generator=g) * 230 - 3 for n in (0, 1, 37, 500)]
    pts.append(torch.tensor([[5.0, 6.0], [5.9, 6.2], [223.99, 0.0], [0.0, 223.5]]))   # duplicates, borders
    out = generate_density_map(pts, 224, 224).cpu()
    exp = torch.stack([ref.density_map(p, 224, 224) for p in pts])
    assert torch.equal(out, exp)


def test_crowd_batch_end_to_end():
    """CropAugment(...)(images, labels, num_crops=2) = Crowd.__getitem__ x B + collate_fn shapes and targets."""
    from ebc_amd.transforms import CropAugment
    from oracle import augment_ref as ref
    shapes = [(768, 1024), (600, 800)]
    imgs = [x.cuda() for x in _images(shapes, 9)]
    g = torch.Generator().manual_seed(1)
    labels = [torch.rand(300, 2, generator=g) * torch.tensor([w, h], dtype=torch.float32) for h, w in shapes]
    torch.manual_seed(0)
    x, points, dens = CropAugment()(imgs, labels, num_crops=2)
    assert x.shape == (4, 3, 224, 224) and dens.shape == (4, 1, 224, 224) and len(points) == 4
    assert torch.isfinite(x).all()
    for p, d in zip(points, dens.cpu()):
        assert torch.equal(d, ref.density_map(p, 224, 224))


@pytest.mark.parametrize("hue", [0.0, 0.2])
def test_reference_rng_stream_end_to_end(hue):
    """CropAugment(noise_rng="reference")(images, labels, num_crops) over a multi-crop stream with noisy crops
    in the middle equals the restated reference transform run crop after crop from the same seed
    (oracle/augment_ref.reference_crop: transforms.py:133-262 with rand_like for the noise): labels exact,
    dot maps exact, normalised pixels within 1e-4 (jitter / blur f32 order), and the generator ends in the same
    state -- the stream is the reference's draw for draw after every noisy crop."""
    from ebc_amd.transforms import CropAugment
    from oracle import augment_ref as ref
    shapes = [(300, 400), (200, 180), (480, 640)]
    kw = dict(min_scale=1.0, max_scale=2.0, brightness=0.4, contrast=0.4, saturation=0.4, saltiness=0.02,
              spiciness=0.02, jitter_prob=0.5, blur_prob=0.3, noise_prob=0.5, hue=hue)
    g = torch.Generator().manual_seed(17)
    imgs = [torch.rand(3, h, w, generator=g) for h, w in shapes]
    labs = [torch.rand(40, 2, generator=g) * torch.tensor([w, h], dtype=torch.float32) for h, w in shapes]
    torch.manual_seed(23)
    exp, exp_lab = [], []
    for img, lab in zip(imgs, labs):
        for _ in range(3):
            o, l = ref.reference_crop(img, lab, 224, (1.0, 2.0), 0.4, 0.4, 0.4, 5, 0.02, 0.02, (0.5, 0.3, 0.5), hue=hue)
            exp.append(ref.normalize(o))
            exp_lab.append(l)
    nxt_ref = torch.rand(1).item()
    torch.manual_seed(23)
    x, points, dens = CropAugment(224, noise_rng="reference", **kw)([t.cuda() for t in imgs], labs, num_crops=3)
    nxt = torch.rand(1).item()
    assert nxt == nxt_ref
    x = x.cpu()
    assert x.shape == (9, 3, 224, 224)
    for k in range(9):
        assert torch.equal(points[k], exp_lab[k]), k
        assert torch.equal(dens[k].cpu(), ref.density_map(exp_lab[k], 224, 224)), k
        assert (x[k] - exp[k]).abs().max().item() < 1e-4, k

"""CPU: the host half of the GPU augmentation (parameter draws and label arithmetic of
ebc_amd.transforms.CropAugment.plan_crop, datasets/transforms.py:9-43,133-187) and the oracle's
counter-based uniforms (the same hash the device kernel uses)."""
import numpy as np
import torch


def _hash_py(seed, i):
    h = (seed ^ ((i * 0x9E3779B9) & 0xFFFFFFFF)) & 0xFFFFFFFF
    h ^= h >> 16; h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13; h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return (h >> 8) / 16777216.0


def test_hash_uniform_matches_scalar_definition():
    from oracle.augment_ref import hash_uniform
    u = hash_uniform(123456789, 5000)
    assert all(abs(float(u[i]) - _hash_py(123456789, i)) == 0.0 for i in range(0, 5000, 37))
    assert 0.45 < float(u.mean()) < 0.55 and float(u.min()) >= 0 and float(u.max()) < 1


def test_whole_image_crop_scales_labels():
    from ebc_amd.transforms import CropAugment
    aug = CropAugment(224, 2.0, 2.0, jitter_prob=0, blur_prob=0, noise_prob=0, flip_prob=0.0)
    lab = torch.tensor([[0.0, 0.0], [100.0, 300.0], [447.0, 447.5]])
    plan, out = aug.plan_crop(0, 448, 448, lab.clone())
    assert (plan.top, plan.left, plan.crop_h, plan.crop_w, plan.pre_resize) == (0, 0, 448, 448, None)
    assert torch.equal(out, torch.tensor([[0.0, 0.0], [50.0, 150.0], [223.0, 223.0]]))   # x*224/448 clamped to 223


def test_small_image_pre_resize_labels_and_flip():
    from ebc_amd.transforms import CropAugment
    torch.manual_seed(3)
    aug = CropAugment(224, 1.0, 1.0, jitter_prob=0, blur_prob=0, noise_prob=0, flip_prob=1.0)
    lab = torch.tensor([[10.0, 20.0], [99.0, 50.0]])
    plan, out = aug.plan_crop(0, 100, 120, lab.clone())
    assert plan.pre_resize == (int(100 * 2.24) + 1, int(120 * 2.24) + 1) and plan.flip
    x = lab[:, 0] * plan.pre_resize[1] / 120 - plan.left
    y = lab[:, 1] * plan.pre_resize[0] / 100 - plan.top
    keep = (x >= 0) & (x < 224) & (y >= 0) & (y < 224)
    exp_x = (223 - x[keep]).clamp(0, 223)
    assert torch.equal(out[:, 0], exp_x) and torch.equal(out[:, 1], y[keep])


def test_draw_order_is_the_references():
    """One crop consumes: uniform (scale), randint, randint, rand (flip), rand (jitter) [+ randperm(4) +
    3 uniforms], rand (blur), rand (noise) [+ one seed draw]."""
    from ebc_amd.transforms import CropAugment
    aug = CropAugment(224, 1.0, 2.0, jitter_prob=1.0, blur_prob=0.0, noise_prob=0.0)
    torch.manual_seed(9)
    aug.plan_crop(0, 500, 600, torch.zeros(0, 2))
    after = torch.rand(1).item()
    torch.manual_seed(9)
    torch.empty(1).uniform_(1.0, 2.0); torch.randint(0, 10, (1,)); torch.randint(0, 10, (1,))
    torch.rand(1); torch.rand(1); torch.randperm(4)
    for _ in range(3):
        torch.empty(1).uniform_(0.9, 1.1)
    torch.rand(1); torch.rand(1)
    assert torch.rand(1).item() == after


def test_rand_like_is_rand_of_the_shape():
    """PepperSaltNoise draws torch.rand_like(image) (transforms.py:252); the host half draws torch.rand of the
    crop's shape: the same generator call, the same values."""
    torch.manual_seed(5)
    a = torch.rand_like(torch.empty(3, 224, 224))
    torch.manual_seed(5)
    assert torch.equal(a, torch.rand(3, 224, 224))


def _stream(aug_kw, shapes, n_per, seed, ref_mode):
    """(plans, labels, next draw) of CropAugment.plan_crop, or (images, labels, next draw) of the oracle's
    restated reference transform, over the same seeded multi-crop stream."""
    from ebc_amd.transforms import CropAugment
    from oracle import augment_ref as ref
    g = torch.Generator().manual_seed(17)
    imgs = [torch.rand(3, h, w, generator=g) for h, w in shapes]
    labs = [torch.rand(40, 2, generator=g) * torch.tensor([w, h], dtype=torch.float32) for h, w in shapes]
    torch.manual_seed(seed)
    outs, labels = [], []
    if ref_mode:
        for img, lab in zip(imgs, labs):
            for _ in range(n_per):
                o, l = ref.reference_crop(img, lab, 224, (aug_kw["min_scale"], aug_kw["max_scale"]),
                                          aug_kw["brightness"], aug_kw["contrast"], aug_kw["saturation"], 5,
                                          aug_kw["saltiness"], aug_kw["spiciness"],
                                          (aug_kw["jitter_prob"], aug_kw["blur_prob"], aug_kw["noise_prob"]),
                                          hue=aug_kw.get("hue", 0.0))
                outs.append(o)
                labels.append(l)
    else:
        aug = CropAugment(224, noise_rng="reference", **aug_kw)
        for i, (img, lab) in enumerate(zip(imgs, labs)):
            for _ in range(n_per):
                p, l = aug.plan_crop(i, img.shape[1], img.shape[2], lab.clone())
                outs.append(p)
                labels.append(l)
    return imgs, outs, labels, torch.rand(1).item()


AUG_KW = dict(min_scale=1.0, max_scale=2.0, brightness=0.4, contrast=0.4, saturation=0.4, saltiness=0.02,
              spiciness=0.02, jitter_prob=0.5, blur_prob=0.3, noise_prob=0.5)
SHAPES = [(300, 400), (200, 180), (480, 640)]


def test_reference_rng_stream_is_the_references():
    """noise_rng="reference": a multi-crop stream with noisy crops in the middle consumes the reference's draws
    one for one -- every crop's labels, pixels (oracle pixel path on the drawn plans) and the generator state
    after the stream equal the restated reference transform's (oracle/augment_ref.reference_crop)."""
    from oracle import augment_ref as ref
    imgs, plans, lab_a, nxt_a = _stream(AUG_KW, SHAPES, 3, 23, False)
    _, ref_imgs, lab_b, nxt_b = _stream(AUG_KW, SHAPES, 3, 23, True)
    noisy = [k for k, p in enumerate(plans) if p.noise]
    assert noisy and noisy[0] < len(plans) - 1, "the seed must give a noisy crop before the last one"
    assert nxt_a == nxt_b
    for a, b in zip(lab_a, lab_b):
        assert torch.equal(a, b)
    got = ref.apply_plans(imgs, plans, (224, 224), saltiness=0.02, spiciness=0.02, normalize=False)
    for k in range(len(plans)):
        assert (got[k] - ref_imgs[k]).abs().max().item() < 1e-5, k


def test_reference_rng_stream_with_hue():
    """ColorJitter with hue != 0 (the reference ColorJitter's class default is 0.2, datasets/transforms.py:206):
    get_params draws the hue factor after the saturation factor and applies it at fn_idx 3; the stream and the
    pixels (oracle pixel path on the drawn plans) equal the restated reference transform's."""
    from oracle import augment_ref as ref
    kw = dict(AUG_KW, hue=0.2, jitter_prob=0.9)
    imgs, plans, lab_a, nxt_a = _stream(kw, SHAPES, 3, 31, False)
    _, ref_imgs, lab_b, nxt_b = _stream(kw, SHAPES, 3, 31, True)
    assert any(op == 4 for p in plans for op, _ in p.jitter)
    assert nxt_a == nxt_b
    got = ref.apply_plans(imgs, plans, (224, 224), saltiness=0.02, spiciness=0.02, normalize=False)
    for k in range(len(plans)):
        assert (got[k] - ref_imgs[k]).abs().max().item() < 1e-5, k


def test_hue_leaves_the_noise_field_channels_last():
    """The reference's rand_like follows its image's layout: channels-last after adjust_hue (einsum), contiguous
    again after GaussianBlur -- the layout CropAugment(noise_rng="reference") draws its field in."""
    from oracle import augment_ref as ref
    x = torch.rand(3, 24, 20)
    y = ref.jitter(ref.adjust_hue(x, 0.1), 1, 1.05)
    assert y.stride() == (1, 60, 3)
    assert ref.gaussian_blur(y, 5, 1.0, 1.0).is_contiguous()
    torch.manual_seed(2)
    a = torch.rand_like(y)
    torch.manual_seed(2)
    assert torch.equal(a, torch.rand(24, 20, 3).permute(2, 0, 1))


def test_adjust_hue_restatement_properties():
    """torchvision adjust_hue restated (oracle): hue 0 keeps the image, a third of a turn maps the primaries
    red -> green -> blue, and +f then -f returns the image (to f32 rounding)."""
    from oracle import augment_ref as ref
    g = torch.Generator().manual_seed(3)
    img = torch.rand(3, 17, 19, generator=g)
    assert (ref.adjust_hue(img, 0.0) - img).abs().max().item() < 1e-6
    prim = torch.eye(3).reshape(3, 3, 1)                   # pixel k = primary k
    out = ref.adjust_hue(prim, 1.0 / 3.0)
    assert torch.allclose(out, torch.roll(torch.eye(3), 1, dims=0).reshape(3, 3, 1), atol=1e-6)   # [channel, pixel]
    back = ref.adjust_hue(ref.adjust_hue(img, 0.23), -0.23)
    assert (back - img).abs().max().item() < 1e-5

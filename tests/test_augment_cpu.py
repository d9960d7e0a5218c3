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

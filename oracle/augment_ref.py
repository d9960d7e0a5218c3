"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

CPU restatement of the reference's training-crop pixel pipeline, applied to the per-crop parameters
that `ebc_amd.transforms.CropAugment.plan_crop` drew.  Pinning:
  * crop + resize: `TF.resize(..., BICUBIC, antialias=True)` on a float tensor is torch's
    `F.interpolate(mode="bicubic", antialias=True)` (the reference's dependency, called here directly),
    `_crop` is a slice (datasets/transforms.py:9-43,133-171) -- pinned by torch itself;
  * flip, normalise: exact (transforms.py:174-187, datasets/crowd.py:64,162);
  * ColorJitter / GaussianBlur: torchvision's functional algorithms restated (adjust_brightness /
    adjust_contrast / adjust_saturation / adjust_hue with _rgb2hsv / _hsv2rgb / rgb_to_grayscale / _blend,
    gaussian_blur with reflect padding
    and the outer-product kernel); torchvision is not importable here, so these two are
    "parity unpinned" against the library itself (the restatement follows its published code);
  * PepperSaltNoise: the reference's two `torch.where`s (transforms.py:242-255) over the plan's host-drawn
    field (noise_rng="reference") or the same counter-based uniforms the device draws (`hash_uniform`).
`reference_crop` restates the whole train transform of one crop -- its torch RNG calls in the reference's
order (RandomResizedCrop :133-171, RandomHorizontalFlip :174-187, RandomApply :226-239 over torchvision
ColorJitter.get_params / GaussianBlur / PepperSaltNoise's rand_like :252) and the label arithmetic -- so a
whole multi-crop stream can be compared draw for draw with CropAugment(noise_rng="reference").
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch
import torch.nn.functional as F

MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def hash_uniform(seed: int, n: int) -> np.ndarray:
    """murmur3-finalised (seed ^ idx * 0x9E3779B9) -> 24-bit uniforms, as the device kernel."""
    idx = np.arange(n, dtype=np.uint64)
    h = (np.uint64(seed) ^ ((idx * np.uint64(0x9E3779B9)) & np.uint64(0xFFFFFFFF))) & np.uint64(0xFFFFFFFF)
    m = np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & m
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & m
    h ^= h >> np.uint64(16)
    return ((h >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)).astype(np.float32)


def resize(img: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """datasets/transforms.py:_resize pixels (TF.resize bicubic, antialias) for [3, H, W]."""
    if img.shape[-2:] == (h, w):
        return img
    return F.interpolate(img[None], size=(h, w), mode="bicubic", align_corners=False, antialias=True)[0]


def _gray(img):
    r, g, b = img.unbind(dim=-3)
    return (0.2989 * r + 0.587 * g + 0.114 * b).unsqueeze(dim=-3)


def _blend(a, b, ratio):
    return (ratio * a + (1.0 - ratio) * b).clamp(0, 1.0)


def _rgb2hsv(img):
    """torchvision.transforms._functional_tensor._rgb2hsv."""
    r, g, b = img.unbind(dim=-3)
    maxc = torch.max(img, dim=-3).values
    minc = torch.min(img, dim=-3).values
    eqc = maxc == minc
    cr = maxc - minc
    ones = torch.ones_like(maxc)
    s = cr / torch.where(eqc, ones, maxc)
    cr_divisor = torch.where(eqc, ones, cr)
    rc = (maxc - r) / cr_divisor
    gc = (maxc - g) / cr_divisor
    bc = (maxc - b) / cr_divisor
    hr = (maxc == r) * (bc - gc)
    hg = ((maxc == g) & (maxc != r)) * (2.0 + rc - bc)
    hb = ((maxc != g) & (maxc != r)) * (4.0 + gc - rc)
    h = hr + hg + hb
    h = torch.fmod((h / 6.0 + 1.0), 1.0)
    return torch.stack((h, s, maxc), dim=-3)


def _hsv2rgb(img):
    """torchvision.transforms._functional_tensor._hsv2rgb."""
    h, s, v = img.unbind(dim=-3)
    i = torch.floor(h * 6.0)
    f = (h * 6.0) - i
    i = i.to(dtype=torch.int32)
    p = torch.clamp((v * (1.0 - s)), 0.0, 1.0)
    q = torch.clamp((v * (1.0 - s * f)), 0.0, 1.0)
    t = torch.clamp((v * (1.0 - s * (1.0 - f))), 0.0, 1.0)
    i = i % 6
    mask = i.unsqueeze(dim=-3) == torch.arange(6, device=i.device).view(-1, 1, 1)
    a1 = torch.stack((v, q, p, p, t, v), dim=-3)
    a2 = torch.stack((t, v, v, q, p, p), dim=-3)
    a3 = torch.stack((p, p, t, v, v, q), dim=-3)
    a4 = torch.stack((a1, a2, a3), dim=-4)
    return torch.einsum("...ijk, ...xijk -> ...xjk", mask.to(dtype=img.dtype), a4)


def adjust_hue(img, hue_factor: float):
    """torchvision F.adjust_hue on a float [3, H, W] image."""
    if not (-0.5 <= hue_factor <= 0.5):
        raise ValueError(f"hue_factor ({hue_factor}) is not in [-0.5, 0.5].")
    hsv = _rgb2hsv(img)
    h, s, v = hsv.unbind(dim=-3)
    h = (h + hue_factor) % 1.0
    return _hsv2rgb(torch.stack((h, s, v), dim=-3))


def jitter(img, op, f):
    """torchvision adjust_brightness (1) / adjust_contrast (2) / adjust_saturation (3) / adjust_hue (4) on float
    images."""
    if op == 4:
        return adjust_hue(img, f)
    if op == 1:
        return _blend(img, torch.zeros_like(img), f)
    if op == 2:
        mean = torch.mean(_gray(img), dim=(-3, -2, -1), keepdim=True)
        return _blend(img, mean, f)
    return _blend(img, _gray(img), f)


def gaussian_blur(img, k: int, sx: float, sy: float):
    """torchvision gaussian_blur(img, [k, k], [sx, sy]) for a float [3, H, W] tensor."""
    def k1(s):
        half = (k - 1) * 0.5
        x = torch.linspace(-half, half, steps=k)
        pdf = torch.exp(-0.5 * (x / s).pow(2))
        return pdf / pdf.sum()
    kern = k1(sy)[:, None] * k1(sx)[None, :]
    kern = kern.expand(3, 1, k, k)
    x = F.pad(img[None], [k // 2, k // 2, k // 2, k // 2], mode="reflect")
    return F.conv2d(x, kern, groups=3)[0]


def apply_plans(images: Sequence[torch.Tensor], plans, size, saltiness=1e-3, spiciness=1e-3, kernel_size=5,
                sigma=(0.1, 5.0), normalize=True) -> torch.Tensor:
    out = []
    for p in plans:
        img = images[p.image].float()
        if p.pre_resize is not None:
            img = resize(img, *p.pre_resize)
        img = img[:, p.top:p.top + p.crop_h, p.left:p.left + p.crop_w]
        img = resize(img, size[0], size[1])
        if p.flip:
            img = img.flip(-1)
        for op, f in p.jitter:
            img = jitter(img, op, f)
        if p.blur:
            img = gaussian_blur(img, kernel_size, sigma[0], sigma[1])
        if p.noise:
            if getattr(p, "noise_field", None) is not None:
                u = p.noise_field
            else:
                u = torch.from_numpy(hash_uniform(p.seed, img.numel())).reshape(img.shape)
            img = torch.where(u < saltiness, 1.0, img)
            img = torch.where(u > 1 - spiciness, 0.0, img)
        if normalize:
            img = (img - torch.tensor(MEAN)[:, None, None]) / torch.tensor(STD)[:, None, None]
        out.append(img)
    return torch.stack(out)


def density_map(label: torch.Tensor, h: int, w: int) -> torch.Tensor:
    """datasets/utils.py:generate_density_map (:11-28), sigma = None."""
    d = torch.zeros((1, h, w), dtype=torch.float32)
    if len(label) > 0:
        lab = label.long()
        lab[:, 0] = lab[:, 0].clamp(min=0, max=w - 1)
        lab[:, 1] = lab[:, 1].clamp(min=0, max=h - 1)
        d[0, lab[:, 1], lab[:, 0]] = 1.0
    return d


def _resize_pair(img, label, h, w):
    """datasets/transforms.py:_resize (:28-43)."""
    ih, iw = img.shape[-2:]
    if ih == h and iw == w:
        return img, label
    img = resize(img, h, w)
    if len(label) > 0:
        label[:, 0] = label[:, 0] * w / iw
        label[:, 1] = label[:, 1] * h / ih
        label[:, 0] = label[:, 0].clamp(min=0, max=w - 1)
        label[:, 1] = label[:, 1].clamp(min=0, max=h - 1)
    return img, label


def _crop_pair(img, label, top, left, h, w):
    """datasets/transforms.py:_crop (:9-25)."""
    img = img[:, top:top + h, left:left + w]
    if len(label) > 0:
        label[:, 0] -= left
        label[:, 1] -= top
        m = (label[:, 0] >= 0) & (label[:, 0] < w) & (label[:, 1] >= 0) & (label[:, 1] < h)
        label = label[m]
    return img, label


def _jitter_range(v):
    """torchvision ColorJitter._check_input for a scalar: (max(1 - v, 0), 1 + v), None when (1, 1)."""
    lo, hi = max(1.0 - v, 0.0), 1.0 + v
    return None if lo == hi == 1.0 else (lo, hi)


def reference_crop(image, label, size=224, scale=(1.0, 2.0), brightness=0.1, contrast=0.1, saturation=0.1,
                   kernel_size=5, saltiness=1e-3, spiciness=1e-3, probs=(0.2, 0.2, 0.5), flip_prob=0.5,
                   sigma=(0.1, 5.0), hue=0.0):
    """One crop of the train transform (utils/data_utils.py:15-24) with the reference's RNG calls, unnormalised."""
    img, label = image.float().clone(), label.float().clone()
    # RandomResizedCrop (transforms.py:147-171)
    s = torch.empty(1).uniform_(scale[0], scale[1]).item()
    ch, cw = int(size * s), int(size * s)
    ih, iw = img.shape[-2:]
    if ch <= ih and cw <= iw:
        top = torch.randint(0, ih - ch + 1, (1,)).item()
        left = torch.randint(0, iw - cw + 1, (1,)).item()
    else:
        ratio = max(ch / ih, cw / iw)
        rh, rw = int(ih * ratio) + 1, int(iw * ratio) + 1
        img, label = _resize_pair(img, label, rh, rw)
        top = torch.randint(0, rh - ch + 1, (1,)).item()
        left = torch.randint(0, rw - cw + 1, (1,)).item()
    img, label = _crop_pair(img, label, top, left, ch, cw)
    img, label = _resize_pair(img, label, size, size)
    # RandomHorizontalFlip (:179-187)
    if torch.rand(1) < flip_prob:
        img = img.flip(-1)
        if len(label) > 0:
            label[:, 0] = img.shape[-1] - 1 - label[:, 0]
            label[:, 0] = label[:, 0].clamp(min=0, max=img.shape[-1] - 1)
    # RandomApply (:233-239): ColorJitter, GaussianBlur, PepperSaltNoise
    if torch.rand(1) < probs[0]:
        rb, rc, rs = _jitter_range(brightness), _jitter_range(contrast), _jitter_range(saturation)
        fn_idx = torch.randperm(4)          # torchvision ColorJitter.get_params
        b = None if rb is None else float(torch.empty(1).uniform_(rb[0], rb[1]))
        c = None if rc is None else float(torch.empty(1).uniform_(rc[0], rc[1]))
        sa = None if rs is None else float(torch.empty(1).uniform_(rs[0], rs[1]))
        hf = None if hue == 0.0 else float(torch.empty(1).uniform_(-hue, hue))
        for fn in fn_idx.tolist():
            if fn == 0 and b is not None:
                img = jitter(img, 1, b)
            elif fn == 1 and c is not None:
                img = jitter(img, 2, c)
            elif fn == 2 and sa is not None:
                img = jitter(img, 3, sa)
            elif fn == 3 and hf is not None:
                img = jitter(img, 4, hf)
    if torch.rand(1) < probs[1]:
        img = gaussian_blur(img, kernel_size, sigma[0], sigma[1])
    if torch.rand(1) < probs[2]:
        noise = torch.rand_like(img)
        img = torch.where(noise < saltiness, 1.0, img)
        img = torch.where(noise > 1 - spiciness, 0.0, img)
    return img, label


def normalize(img):
    """datasets/crowd.py:64,162 Normalize(ImageNet mean / std)."""
    return (img - torch.tensor(MEAN)[:, None, None]) / torch.tensor(STD)[:, None, None]

"""Training-crop augmentation on the GPU.

The reference builds every training crop on the CPU inside DataLoader workers
(`utils/data_utils.py:14-26` composes `datasets/transforms.py` and `datasets/crowd.py:134-175`
normalises and makes the dot maps; with 8 GPUs `num_workers = 4 // nprocs` is 0, so the training
process itself does it).  Here the host only draws the random parameters -- with the reference's own
torch RNG calls, in the reference's order -- and transforms the point labels (tiny, exact same float32
arithmetic), and the pixel work of a whole batch runs in three launches (`ebc_augment_crops`:
crop + antialiased-bicubic resize, flip, colour jitter, blur, salt-and-pepper, normalise) plus one for
the dot maps (`ebc_point_map`).

Surface (mirrors the reference):
  * `CropAugment(...)` -- the train-split `Compose([RandomResizedCrop, RandomHorizontalFlip,
    RandomApply([ColorJitter, GaussianBlur, PepperSaltNoise])])` of `get_dataloader`
    (utils/data_utils.py:15-24) with the trainer's argument names and defaults (trainer.py:40-52);
    `__call__(images, labels, num_crops)` returns what `Crowd.__getitem__` + `collate_fn`
    (datasets/crowd.py:134-175, datasets/utils.py:32-47) return: images `[B*num_crops, 3, S, S]`
    (normalised), the per-crop point lists and the dot maps `[B*num_crops, 1, S, S]`.
  * `plan_crop(...)` -- one crop's parameters and labels (the host half; used by the tests' oracle).
  * `generate_density_map(points, H, W)` -- datasets/utils.py:11-28 with sigma=None, batched.

The salt-and-pepper uniforms come from one of two sources (`noise_rng`):
  * "device" (default): a counter-based hash on device seeded by ONE host draw -- no 600 KB host draw and
    upload per noisy crop, but the host RNG stream (and with it every later crop's parameters) diverges
    from the reference's after the first noisy crop;
  * "reference": the host draws the field with the reference's own call, `torch.rand_like(image)` on the
    [3, S, S] crop (datasets/transforms.py:252), at its place in the stream, and uploads it: the whole
    stream -- every crop's window, flip, jitter factors and noise -- is the reference's draw for draw.
ColorJitter's hue (torchvision adjust_hue: RGB -> HSV, hue shift, HSV -> RGB) runs per pixel on device; the trainer's
default is hue = 0 (trainer.py:46), the reference's ColorJitter class default 0.2 (datasets/transforms.py:206).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from . import _lib

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # datasets/crowd.py:64
IMAGENET_STD = (0.229, 0.224, 0.225)
JIT_BRIGHTNESS, JIT_CONTRAST, JIT_SATURATION, JIT_HUE = 1, 2, 3, 4


@dataclass
class CropPlan:
    """One output crop: source window, optional pre-resize, and the pixel ops (in reference order)."""
    image: int                               # index of the source image
    top: int
    left: int
    crop_h: int
    crop_w: int
    pre_resize: Optional[Tuple[int, int]]    # RandomResizedCrop resizes the whole image first when it is smaller than the crop
    flip: bool
    jitter: List[Tuple[int, float]] = field(default_factory=list)   # (JIT_*, factor) in application order
    blur: bool = False
    noise: bool = False
    seed: int = 0
    noise_field: Optional[Tensor] = None     # [3, S, S] uniforms drawn by the host (noise_rng="reference")


def _check_jitter(value: float, name: str, center: float = 1.0, clip_first_on_zero: bool = True):
    """torchvision ColorJitter._check_input for a scalar argument: [center - v, center + v] or None."""
    if value < 0:
        raise ValueError(f"If {name} is a single number, it must be non negative.")
    lo, hi = center - value, center + value
    if clip_first_on_zero:
        lo = max(lo, 0.0)
    return None if lo == hi == center else (lo, hi)


def _resize_label(label: Tensor, in_h: int, in_w: int, h: int, w: int) -> Tensor:
    # datasets/transforms.py:_resize (:28-43): float32 arithmetic on the CPU label tensor
    if len(label) > 0 and (in_h != h or in_w != w):
        label[:, 0] = label[:, 0] * w / in_w
        label[:, 1] = label[:, 1] * h / in_h
        label[:, 0] = label[:, 0].clamp(min=0, max=w - 1)
        label[:, 1] = label[:, 1].clamp(min=0, max=h - 1)
    return label


def _crop_label(label: Tensor, top: int, left: int, h: int, w: int) -> Tensor:
    # datasets/transforms.py:_crop (:9-25)
    if len(label) > 0:
        label[:, 0] -= left
        label[:, 1] -= top
        mask = (label[:, 0] >= 0) & (label[:, 0] < w) & (label[:, 1] >= 0) & (label[:, 1] < h)
        label = label[mask]
    return label


def _upload(descs, dev) -> Tensor:
    """Descriptor array -> device, through pinned memory (async; the caching host allocator keeps the
    pinned block alive until the copy has run)."""
    host = torch.frombuffer(bytearray(bytes(descs)), dtype=torch.uint8).pin_memory()
    return host.to(dev, non_blocking=True)


class CropAugment:
    """The reference's training transform on the GPU (see module docstring)."""

    def __init__(self, input_size: int = 224, min_scale: float = 1.0, max_scale: float = 2.0,
                 brightness: float = 0.1, contrast: float = 0.1, saturation: float = 0.1, hue: float = 0.0,
                 kernel_size: int = 5, saltiness: float = 1e-3, spiciness: float = 1e-3,
                 jitter_prob: float = 0.2, blur_prob: float = 0.2, noise_prob: float = 0.5, flip_prob: float = 0.5,
                 blur_sigma: Tuple[float, float] = (0.1, 5.0), mean=IMAGENET_MEAN, std=IMAGENET_STD,
                 noise_rng: str = "device"):
        if noise_rng not in ("device", "reference"):
            raise ValueError(f"noise_rng must be 'device' or 'reference', got {noise_rng!r}")
        self.noise_rng = noise_rng
        if not 0 < min_scale <= max_scale:
            raise ValueError(f"scale should satisfy 0 < scale[0] <= scale[1], got {(min_scale, max_scale)}.")
        if not 0.0 <= hue <= 0.5:
            raise ValueError(f"hue values should be between (-0.5, 0.5), got {hue}")     # torchvision _check_input
        if kernel_size % 2 == 0 or not 1 <= kernel_size <= 31:
            raise ValueError("kernel_size must be odd and <= 31")
        self.size = (input_size, input_size)
        self.scale = (min_scale, max_scale)
        self.bright = _check_jitter(brightness, "brightness")
        self.contr = _check_jitter(contrast, "contrast")
        self.satur = _check_jitter(saturation, "saturation")
        self.hue = None if hue == 0.0 else (-hue, hue)
        self.saltiness, self.spiciness = saltiness, spiciness
        self.p = (jitter_prob, blur_prob, noise_prob)
        self.flip_prob = flip_prob
        self.const = _lib.EbcAugConst((ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*std), kernel_size,
                                      float(blur_sigma[0]), float(blur_sigma[1]))

    # ---------------------------------------------------------------- host half: parameters + labels
    def plan_crop(self, image_index: int, in_h: int, in_w: int, label: Tensor) -> Tuple[CropPlan, Tensor]:
        """Draw one crop's parameters with the reference's RNG calls, in its order, and move its label.

        RandomResizedCrop (datasets/transforms.py:133-171), RandomHorizontalFlip (:174-187), RandomApply
        (:226-239) over ColorJitter (torchvision ColorJitter.get_params: randperm(4), then one uniform per
        enabled factor), GaussianBlur (no draw) and PepperSaltNoise (one seed draw, or with
        noise_rng="reference" the reference's `torch.rand_like(image)` field, transforms.py:252)."""
        out_h, out_w = self.size
        scale = torch.empty(1).uniform_(self.scale[0], self.scale[1]).item()
        crop_h, crop_w = int(out_h * scale), int(out_w * scale)
        pre = None
        H, W = in_h, in_w
        if not (crop_h <= H and crop_w <= W):
            ratio = max(crop_h / H, crop_w / W)
            pre = (int(H * ratio) + 1, int(W * ratio) + 1)
            label = _resize_label(label, H, W, pre[0], pre[1])
            H, W = pre
        top = torch.randint(0, H - crop_h + 1, (1,)).item()
        left = torch.randint(0, W - crop_w + 1, (1,)).item()
        label = _crop_label(label, top, left, crop_h, crop_w)
        label = _resize_label(label, crop_h, crop_w, out_h, out_w)
        plan = CropPlan(image_index, top, left, crop_h, crop_w, pre, False)
        if torch.rand(1) < self.flip_prob:
            plan.flip = True
            if len(label) > 0:
                label[:, 0] = out_w - 1 - label[:, 0]
                label[:, 0] = label[:, 0].clamp(min=0, max=out_w - 1)
        if torch.rand(1) < self.p[0]:
            fn_idx = torch.randperm(4)
            b = None if self.bright is None else float(torch.empty(1).uniform_(*self.bright))
            c = None if self.contr is None else float(torch.empty(1).uniform_(*self.contr))
            s = None if self.satur is None else float(torch.empty(1).uniform_(*self.satur))
            h = None if self.hue is None else float(torch.empty(1).uniform_(*self.hue))
            for fn in fn_idx.tolist():
                if fn == 0 and b is not None:
                    plan.jitter.append((JIT_BRIGHTNESS, b))
                elif fn == 1 and c is not None:
                    plan.jitter.append((JIT_CONTRAST, c))
                elif fn == 2 and s is not None:
                    plan.jitter.append((JIT_SATURATION, s))
                elif fn == 3 and h is not None:
                    plan.jitter.append((JIT_HUE, h))
        if torch.rand(1) < self.p[1]:
            plan.blur = True
        if torch.rand(1) < self.p[2]:
            plan.noise = True
            if self.noise_rng == "reference":
                # rand_like of the float32 [3, out_h, out_w] crop: the same generator call as torch.rand of that shape,
                # in the crop's memory order -- torchvision's adjust_hue ends in an einsum that leaves the image
                # channels-last (strides (1, 3 W, 3)), the later jitter ops keep that layout and GaussianBlur's conv
                # makes it contiguous again, so after a hue op with no blur the uniforms land in (y, x, c) order
                if not plan.blur and any(op == JIT_HUE for op, _ in plan.jitter):
                    plan.noise_field = torch.rand(out_h, out_w, 3).permute(2, 0, 1).contiguous()
                else:
                    plan.noise_field = torch.rand(3, out_h, out_w)
            else:
                plan.seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item())
        return plan, label

    # ---------------------------------------------------------------- device half
    def apply(self, images: Sequence[Tensor], plans: Sequence[CropPlan], normalize: bool = True) -> Tensor:
        """Run the pixel work of `plans` on `images` ([3, H, W] f32 in [0, 1] on the device)."""
        L = _lib.lib()
        dev = images[0].device
        out_h, out_w = self.size
        n = len(plans)
        out = torch.empty(n, 3, out_h, out_w, device=dev)
        if n == 0:
            return out
        # whole-image pre-resizes (RandomResizedCrop's small-image branch) first, as their own crops
        srcs = list(images)
        pre_plans, pre_index = [], {}
        for k, p in enumerate(plans):
            if p.pre_resize is not None:
                pre_index[k] = len(srcs) + len(pre_plans)
                img = images[p.image]
                pre_plans.append((img, p.pre_resize))
        pre_out = []
        if pre_plans:
            for img, (h, w) in pre_plans:
                pre_out.append(self._resize_whole(img, h, w))
            srcs = srcs + pre_out
        for t in srcs:
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.dim() == 3 and t.shape[0] == 3):
                raise ValueError("images must be contiguous [3, H, W] float32 device tensors")
        base = min(t.data_ptr() for t in srcs)
        descs = (_lib.EbcCropDesc * n)()
        tmp = 0
        max_ch = 0
        fields = []
        for k, p in enumerate(plans):
            src = srcs[pre_index.get(k, p.image)]
            off = src.data_ptr() - base
            assert off % 4 == 0
            d = descs[k]
            d.src_off, d.out_off, d.tmp_off = off // 4, k * 3 * out_h * out_w, tmp
            d.src_h, d.src_w = src.shape[1], src.shape[2]
            d.top, d.left, d.crop_h, d.crop_w, d.out_h, d.out_w = p.top, p.left, p.crop_h, p.crop_w, out_h, out_w
            if p.top + p.crop_h > d.src_h or p.left + p.crop_w > d.src_w or p.top < 0 or p.left < 0:
                raise ValueError(f"crop window outside its image: {p}")
            d.flip = int(p.flip)
            ops, f = 0, {JIT_BRIGHTNESS: 1.0, JIT_CONTRAST: 1.0, JIT_SATURATION: 1.0, JIT_HUE: 0.0}
            for slot, (op, v) in enumerate(p.jitter):
                ops |= op << (3 * slot)
                f[op] = v
            d.jitter_ops = ops
            d.brightness, d.contrast, d.saturation = f[JIT_BRIGHTNESS], f[JIT_CONTRAST], f[JIT_SATURATION]
            d.hue = f[JIT_HUE]
            d.blur, d.noise = int(p.blur), int(p.noise)
            d.saltiness, d.spiciness, d.seed = self.saltiness, self.spiciness, p.seed & 0xFFFFFFFF
            d.noise_off = -1
            if p.noise and p.noise_field is not None:
                if tuple(p.noise_field.shape) != (3, out_h, out_w) or p.noise_field.dtype != torch.float32:
                    raise ValueError(f"noise_field must be float32 [3, {out_h}, {out_w}], got {p.noise_field.shape}")
                d.noise_off = len(fields) * 3 * out_h * out_w
                fields.append(p.noise_field)
            d.normalize = int(normalize)
            tmp += 3 * max(p.crop_h, out_h) * out_w
            max_ch = max(max_ch, p.crop_h)
        ws = torch.empty(tmp, device=dev)
        ddesc = _upload(descs, dev)
        noise = None
        if fields:
            noise = torch.stack(fields).pin_memory().to(dev, non_blocking=True)
        src_base = ctypes.c_void_p(base)
        _lib.check(L.ebc_augment_crops(src_base, _lib.ptr(ddesc), n, max_ch, out_h, _lib.ptr(out), _lib.ptr(ws),
                                       _lib.ptr(noise), self.const, _lib.stream(dev)),
                   "ebc_augment_crops")
        return out     # temporaries are released stream-ordered (caching allocator), after the launches

    def _resize_whole(self, img: Tensor, h: int, w: int) -> Tensor:
        """_resize of the whole image (transforms.py:28-43) -- the pre-resize of RandomResizedCrop."""
        L = _lib.lib()
        img = img.contiguous()
        out = torch.empty(1, 3, h, w, device=img.device)
        d = (_lib.EbcCropDesc * 1)()
        d[0].src_off, d[0].out_off, d[0].tmp_off, d[0].noise_off = 0, 0, 0, -1
        d[0].src_h, d[0].src_w = img.shape[1], img.shape[2]
        d[0].top, d[0].left, d[0].crop_h, d[0].crop_w, d[0].out_h, d[0].out_w = 0, 0, img.shape[1], img.shape[2], h, w
        ws = torch.empty(3 * max(img.shape[1], h) * w, device=img.device)
        ddesc = _upload(d, img.device)
        _lib.check(L.ebc_augment_crops(_lib.ptr(img), _lib.ptr(ddesc), 1, img.shape[1], h, _lib.ptr(out), _lib.ptr(ws),
                                       None, self.const, _lib.stream(img)), "ebc_augment_crops (pre-resize)")
        return out[0]

    def __call__(self, images: Sequence[Tensor], labels: Sequence[Tensor], num_crops: int = 1):
        """Crowd.__getitem__ for each image (num_crops crops) + collate_fn: (images, points, densities)."""
        plans, points = [], []
        for i, (img, lab) in enumerate(zip(images, labels)):
            for _ in range(num_crops):
                p, l = self.plan_crop(i, img.shape[-2], img.shape[-1], lab.clone().float())
                plans.append(p)
                points.append(l)
        imgs = self.apply(images, plans)
        dens = generate_density_map(points, self.size[0], self.size[1], device=imgs.device)
        return imgs, points, dens


def generate_density_map(points: Sequence[Tensor], height: int, width: int, device=None) -> Tensor:
    """datasets/utils.py:11-28 (sigma=None) for a list of [n, 2] (x, y) labels -> [B, 1, H, W] on the device."""
    L = _lib.lib()
    dev = torch.device("cuda") if device is None else device
    B = len(points)
    counts = [int(p.shape[0]) for p in points]
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    packed = torch.cat([p.reshape(-1, 2).float().cpu() for p in points], 0) if offs[-1] else torch.zeros(1, 2)
    dpts = packed.contiguous().pin_memory().to(dev, non_blocking=True)
    doffs = torch.tensor(offs, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
    out = torch.empty(B, 1, height, width, device=dev)
    _lib.check(L.ebc_point_map(_lib.ptr(dpts), _lib.ptr(doffs), B, height, width, max(counts, default=0), _lib.ptr(out),
                               _lib.stream(dev)), "ebc_point_map")
    return out

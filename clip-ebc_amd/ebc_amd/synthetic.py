"""Deterministic synthetic weights and crops for CLIP-EBC (ViT-B/16 + deep VPT; CLIP ResNet-50, config 2).

There are no CLIP checkpoints offline (the reference downloads them on import,
`models/clip/_clip/__init__.py:31-36`), so parity and benchmarking run on weights
generated here from a seed.  Every tensor is drawn from its own
`numpy.random.Generator(PCG64([seed, crc32(key)]))`, so a key's values do not depend
on which other keys exist or on their order; the GPU box regenerates exactly the same
arrays as this container.

Key names are the reference's `CLIP_EBC.state_dict()` keys:
`image_encoder.*`, `vpt_{l}`, `image_decoder.0.*`, `projection.*`, `text_encoder.*`,
`logit_scale`.

Synthetic crops follow BASELINE.md: pixels U[0,1) normalised by the ImageNet mean/std
(`datasets/crowd.py:64`), point counts lognormal(ln 20, 1.2) clipped to [0, 2048],
coordinates U[0, S)^2, density = point map (`datasets/utils.py:11-28`, sigma=None).
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, List, Tuple

import numpy as np

WIDTH = 768          # ViT-B/16 width
HEADS = 12
PATCH = 16
EMBED = 512          # CLIP joint embedding
TEXT_WIDTH = 512
TEXT_HEADS = 8
TEXT_CTX = 77
VOCAB = 49408
NUM_VPT = 32
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed, zlib.crc32(key.encode())]))


def _normal(seed, key, shape, std, mean=0.0):
    return (mean + std * _rng(seed, key).standard_normal(shape)).astype(np.float32)


def _uniform(seed, key, shape, lo, hi):
    return _rng(seed, key).uniform(lo, hi, shape).astype(np.float32)


def _block(sd, seed, prefix, width):
    s = 1.0 / math.sqrt(width)
    sd[prefix + "attn.in_proj_weight"] = _normal(seed, prefix + "attn.in_proj_weight", (3 * width, width), s)
    sd[prefix + "attn.in_proj_bias"] = _normal(seed, prefix + "attn.in_proj_bias", (3 * width,), 0.02)
    sd[prefix + "attn.out_proj.weight"] = _normal(seed, prefix + "attn.out_proj.weight", (width, width), 0.5 * s)
    sd[prefix + "attn.out_proj.bias"] = _normal(seed, prefix + "attn.out_proj.bias", (width,), 0.02)
    for ln in ("ln_1", "ln_2"):
        sd[prefix + ln + ".weight"] = _normal(seed, prefix + ln + ".weight", (width,), 0.05, 1.0)
        sd[prefix + ln + ".bias"] = _normal(seed, prefix + ln + ".bias", (width,), 0.05)
    sd[prefix + "mlp.c_fc.weight"] = _normal(seed, prefix + "mlp.c_fc.weight", (4 * width, width), s)
    sd[prefix + "mlp.c_fc.bias"] = _normal(seed, prefix + "mlp.c_fc.bias", (4 * width,), 0.02)
    sd[prefix + "mlp.c_proj.weight"] = _normal(seed, prefix + "mlp.c_proj.weight", (width, 4 * width), 0.5 / math.sqrt(4 * width))
    sd[prefix + "mlp.c_proj.bias"] = _normal(seed, prefix + "mlp.c_proj.bias", (width,), 0.02)


def vit_state(seed: int = 0, layers: int = 12, input_size: int = 224) -> Dict[str, np.ndarray]:
    """Frozen CLIP ViT-B/16 visual tower (`image_encoder.py:118-161`), features_only."""
    g = input_size // PATCH
    sd: Dict[str, np.ndarray] = {}
    p = "image_encoder."
    sd[p + "conv1.weight"] = _normal(seed, p + "conv1.weight", (WIDTH, 3, PATCH, PATCH), 1.0 / math.sqrt(3 * PATCH * PATCH))
    sd[p + "class_embedding"] = _normal(seed, p + "class_embedding", (WIDTH,), WIDTH ** -0.5)
    sd[p + "positional_embedding"] = _normal(seed, p + "positional_embedding", (g * g + 1, WIDTH), WIDTH ** -0.5)
    for ln in ("ln_pre", "ln_post"):
        sd[p + ln + ".weight"] = _normal(seed, p + ln + ".weight", (WIDTH,), 0.05, 1.0)
        sd[p + ln + ".bias"] = _normal(seed, p + ln + ".bias", (WIDTH,), 0.05)
    for i in range(layers):
        _block(sd, seed, f"{p}transformer.resblocks.{i}.", WIDTH)
    return sd


def outlier_stats(sd: Dict[str, np.ndarray], seed: int = 0, n_channels: int = 6, dc: float = 3.0) -> Dict[str, np.ndarray]:
    """A copy of a ViT state dict (vit_state / full_state) with residual-stream statistics closer to a pretrained
    CLIP tower's than the benign init above: a handful of 'massive activation' channels (ln_pre gamma at 30..100x,
    random sign, and every block's out-proj / c_proj bias pushing them further by 2..8 per block), a common offset
    `dc` on every channel (ln_pre beta: the rows' mean, which the fold's one-pass variance E[x^2] - mean^2 must
    survive) and the LayerNorm gammas spread log-uniformly over 0.1..10.  Rows then carry per-channel ranges of ~100x and a mean offset from
    the outliers: the stress case of the folded LayerNorm (gemm.hip EPI_LN normalises f16 rows after the product;
    VERDICT r04 item 6)."""
    out = dict(sd)
    g = _rng(seed, "outlier_stats")
    ch = g.choice(WIDTH, n_channels, replace=False)
    sign = np.where(g.random(n_channels) < 0.5, -1.0, 1.0).astype(np.float32)
    p = "image_encoder."
    w = out[p + "ln_pre.weight"].copy()
    w[ch] = sign * g.uniform(30.0, 100.0, n_channels).astype(np.float32)
    out[p + "ln_pre.weight"] = w
    out[p + "ln_pre.bias"] = out[p + "ln_pre.bias"] + np.float32(dc)
    i = 0
    while f"{p}transformer.resblocks.{i}.ln_1.weight" in out:
        q = f"{p}transformer.resblocks.{i}."
        for ln in ("ln_1", "ln_2"):
            out[q + ln + ".weight"] = np.exp(g.uniform(math.log(0.1), math.log(10.0), WIDTH)).astype(np.float32)
        for b in ("attn.out_proj.bias", "mlp.c_proj.bias"):
            v = out[q + b].copy()
            v[ch] += sign * g.uniform(2.0, 8.0, n_channels).astype(np.float32)
            out[q + b] = v
        i += 1
    return out


def text_state(seed: int = 0, layers: int = 12, embed: int = EMBED) -> Dict[str, np.ndarray]:
    """Frozen CLIP text tower (`text_encoder.py:7-53`)."""
    sd: Dict[str, np.ndarray] = {}
    p = "text_encoder."
    sd[p + "token_embedding.weight"] = _normal(seed, p + "token_embedding.weight", (VOCAB, TEXT_WIDTH), 0.02)
    sd[p + "positional_embedding"] = _normal(seed, p + "positional_embedding", (TEXT_CTX, TEXT_WIDTH), 0.01)
    for i in range(layers):
        _block(sd, seed, f"{p}transformer.resblocks.{i}.", TEXT_WIDTH)
    sd[p + "ln_final.weight"] = _normal(seed, p + "ln_final.weight", (TEXT_WIDTH,), 0.05, 1.0)
    sd[p + "ln_final.bias"] = _normal(seed, p + "ln_final.bias", (TEXT_WIDTH,), 0.05)
    sd[p + "text_projection"] = _normal(seed, p + "text_projection", (TEXT_WIDTH, embed), TEXT_WIDTH ** -0.5)
    return sd


def trainable_state(seed: int = 0, layers: int = 12, deep_vpt: bool = True) -> Dict[str, np.ndarray]:
    """VPT tokens, BasicBlock decoder, projection, logit_scale.

    Init laws follow the reference: VPT U(+-sqrt(6/(3*16+768))) (`models/clip/model.py:70-75`),
    conv kaiming_normal(fan_out, relu) and BN (1, 0) (`models/utils.py:366-379`),
    logit_scale = ln(1/0.07) (`models/clip/model.py:117`).
    """
    sd: Dict[str, np.ndarray] = {}
    val = math.sqrt(6.0 / float(3 * PATCH + WIDTH))
    for i in range(layers if deep_vpt else 1):
        sd[f"vpt_{i}"] = _uniform(seed, f"vpt_{i}", (NUM_VPT, WIDTH), -val, val)
    d = "image_decoder.0."
    std = math.sqrt(2.0 / (WIDTH * 9))
    for c, bn in (("conv1", "bn1"), ("conv2", "bn2")):
        sd[d + c + ".weight"] = _normal(seed, d + c + ".weight", (WIDTH, WIDTH, 3, 3), std)
        sd[d + bn + ".weight"] = np.ones(WIDTH, np.float32)
        sd[d + bn + ".bias"] = np.zeros(WIDTH, np.float32)
        sd[d + bn + ".running_mean"] = np.zeros(WIDTH, np.float32)
        sd[d + bn + ".running_var"] = np.ones(WIDTH, np.float32)
        sd[d + bn + ".num_batches_tracked"] = np.zeros((), np.int64)
    sd["projection.weight"] = _normal(seed, "projection.weight", (EMBED, WIDTH, 1, 1), math.sqrt(2.0 / EMBED))
    sd["projection.bias"] = np.zeros(EMBED, np.float32)
    sd["logit_scale"] = np.array(math.log(1 / 0.07), np.float32)
    return sd


def full_state(seed: int = 0, layers: int = 12, text_layers: int = 12, input_size: int = 224,
               include_text: bool = True) -> Dict[str, np.ndarray]:
    sd = vit_state(seed, layers, input_size)
    sd.update(trainable_state(seed, layers))
    if include_text:
        sd.update(text_state(seed, text_layers))
    return sd


# ----------------------------------------------------------------------------- CLIP ResNet-50 (config 2)
RN50_LAYERS = (3, 4, 6, 3)
RN50_WIDTH = 64
RN50_EMBED = 1024          # clip_resnet50 joint embedding (models/clip/model.py:16)
RN50_CHANNELS = 2048       # layer4 output = decoder cfg [2048] (models/clip/model.py:237-238)


def _bn(sd, seed, key, n, gamma_mean=1.0):
    sd[key + ".weight"] = _normal(seed, key + ".weight", (n,), 0.05, gamma_mean)
    sd[key + ".bias"] = _normal(seed, key + ".bias", (n,), 0.05)
    sd[key + ".running_mean"] = np.zeros(n, np.float32)
    sd[key + ".running_var"] = np.ones(n, np.float32)
    sd[key + ".num_batches_tracked"] = np.zeros((), np.int64)


def _conv(sd, seed, key, cout, cin, k):
    sd[key + ".weight"] = _normal(seed, key + ".weight", (cout, cin, k, k), math.sqrt(2.0 / (cin * k * k)))


def resnet50_state(seed: int = 0, layers=RN50_LAYERS, width: int = RN50_WIDTH) -> Dict[str, np.ndarray]:
    """CLIP ModifiedResNet image tower, features_only (`image_encoder.py:10-77`, blocks.py:56-101): He-normal
    convs, BatchNorm gamma ~1 (the residual branch's bn3 at 0.25 so 16 stacked blocks stay well scaled)."""
    sd: Dict[str, np.ndarray] = {}
    p = "image_encoder."
    _conv(sd, seed, p + "conv1", width // 2, 3, 3); _bn(sd, seed, p + "bn1", width // 2)
    _conv(sd, seed, p + "conv2", width // 2, width // 2, 3); _bn(sd, seed, p + "bn2", width // 2)
    _conv(sd, seed, p + "conv3", width, width // 2, 3); _bn(sd, seed, p + "bn3", width)
    inplanes = width
    for li, nblocks in enumerate(layers):
        planes = width * (2 ** li)
        for bi in range(nblocks):
            q = f"{p}layer{li + 1}.{bi}."
            _conv(sd, seed, q + "conv1", planes, inplanes, 1); _bn(sd, seed, q + "bn1", planes)
            _conv(sd, seed, q + "conv2", planes, planes, 3); _bn(sd, seed, q + "bn2", planes)
            _conv(sd, seed, q + "conv3", planes * 4, planes, 1); _bn(sd, seed, q + "bn3", planes * 4, 0.25)
            if bi == 0:
                _conv(sd, seed, q + "downsample.0", planes * 4, inplanes, 1); _bn(sd, seed, q + "downsample.1", planes * 4)
            inplanes = planes * 4
    return sd


def resnet50_trainable_state(seed: int = 0) -> Dict[str, np.ndarray]:
    """Decoder Bottleneck(2048, 2048, expansion=1) and projection 2048 -> 1024 with the reference's init laws:
    kaiming_normal(fan_out, relu) convs, BN (1, 0) (`models/utils.py:366-379`), logit_scale = ln(1/0.07)."""
    sd: Dict[str, np.ndarray] = {}
    d = "image_decoder.0."
    C = RN50_CHANNELS
    for c, bn, k in (("conv1", "bn1", 1), ("conv2", "bn2", 3), ("conv3", "bn3", 1)):
        sd[d + c + ".weight"] = _normal(seed, d + c + ".weight", (C, C, k, k), math.sqrt(2.0 / (C * k * k)))
        sd[d + bn + ".weight"] = np.ones(C, np.float32)
        sd[d + bn + ".bias"] = np.zeros(C, np.float32)
        sd[d + bn + ".running_mean"] = np.zeros(C, np.float32)
        sd[d + bn + ".running_var"] = np.ones(C, np.float32)
        sd[d + bn + ".num_batches_tracked"] = np.zeros((), np.int64)
    sd["projection.weight"] = _normal(seed, "projection.weight", (RN50_EMBED, C, 1, 1), math.sqrt(2.0 / RN50_EMBED))
    sd["projection.bias"] = np.zeros(RN50_EMBED, np.float32)
    sd["logit_scale"] = np.array(math.log(1 / 0.07), np.float32)
    return sd


def resnet50_full_state(seed: int = 0, text_layers: int = 12, include_text: bool = True) -> Dict[str, np.ndarray]:
    sd = resnet50_state(seed)
    sd.update(resnet50_trainable_state(seed))
    if include_text:
        sd.update(text_state(seed, text_layers, embed=RN50_EMBED))
    return sd


def crop_rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(seed))


def synthetic_crops(batch: int, size: int = 224, seed: int = 1000, max_points: int = 2048,
                    counts: List[int] | None = None) -> Tuple[np.ndarray, List[np.ndarray], np.ndarray]:
    """Return (images [B,3,S,S] f32 normalised, points list of [n_i,2] (x,y) f32, density [B,1,S,S])."""
    g = crop_rng(seed)
    img = g.random((batch, 3, size, size), dtype=np.float32)
    mean = np.asarray(IMAGENET_MEAN, np.float32).reshape(1, 3, 1, 1)
    std = np.asarray(IMAGENET_STD, np.float32).reshape(1, 3, 1, 1)
    img = (img - mean) / std
    if counts is None:
        counts = np.clip(np.floor(g.lognormal(math.log(20.0), 1.2, batch)), 0, max_points).astype(int).tolist()
    points = [(g.random((n, 2)) * size).astype(np.float32) for n in counts]
    density = np.zeros((batch, 1, size, size), np.float32)
    for b, p in enumerate(points):
        density[b, 0] = point_map(p, size, size)
    return img.astype(np.float32), points, density


def point_map(points: np.ndarray, height: int, width: int) -> np.ndarray:
    """Dot-annotation map: 1.0 at each (clamped, truncated) point (`datasets/utils.py:11-22`)."""
    m = np.zeros((height, width), np.float32)
    if len(points):
        p = points.astype(np.int64)  # .long() truncates toward zero
        x = np.clip(p[:, 0], 0, width - 1)
        y = np.clip(p[:, 1], 0, height - 1)
        m[y, x] = 1.0
    return m


# ----------------------------------------------------------------------------- vgg19_ae (config 1)
def vgg19_ae_state(seed: int = 0, n_bins=5) -> Dict[str, np.ndarray]:
    """VGG-19 features (He-normal convs, small biases: the ImageNet weights are a download), the reg_layer and
    the classifier (n_bins) / regressor (n_bins None) with the reference's `_init_weights` laws
    (kaiming_normal fan_out, zero bias; models/utils.py:366-379)."""
    from .vgg import VGG_CFG_E
    sd: Dict[str, np.ndarray] = {}
    idx, cin = 0, 3
    for v in VGG_CFG_E:
        if v == "M":
            idx += 1
            continue
        k = f"backbone.features.{idx}"
        sd[k + ".weight"] = _normal(seed, k + ".weight", (v, cin, 3, 3), math.sqrt(2.0 / (cin * 9)))
        sd[k + ".bias"] = _normal(seed, k + ".bias", (v,), 0.01)
        idx += 2
        cin = v
    for i, (co, ci) in ((0, (256, 512)), (2, (128, 256))):
        k = f"backbone.reg_layer.{i}"
        sd[k + ".weight"] = _normal(seed, k + ".weight", (co, ci, 3, 3), math.sqrt(2.0 / (co * 9)))
        sd[k + ".bias"] = np.zeros(co, np.float32)
    if n_bins is None:
        sd["regressor.0.weight"] = _normal(seed, "regressor.0.weight", (1, 128, 1, 1), math.sqrt(2.0))
        sd["regressor.0.bias"] = np.zeros(1, np.float32)
    else:
        sd["classifier.weight"] = _normal(seed, "classifier.weight", (n_bins, 128, 1, 1), math.sqrt(2.0 / n_bins))
        sd["classifier.bias"] = np.zeros(n_bins, np.float32)
    return sd

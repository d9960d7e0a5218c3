"""BASELINE configs[0]: `vgg19_ae` (the DM-Count VGG-19 encoder-decoder) behind `get_model`, with the EBC
classification head.

Reference surface (BASELINE configs[0]):
  * `models/encoder_decoder/vgg.py:13-41` VGG(features = make_vgg_layers(cfg "E"), reduction): features
    (16 conv3x3+ReLU, 4 max-pools -> stride 16), bilinear x(16 / reduction), reg_layer conv3x3 512->256->128
    + ReLU; `encoder_reduction` 16, `channels` 128.  `vgg19_ae` = `vgg19` there
    (`models/encoder_decoder/__init__.py:4`).
  * `models/model.py:37-75` Classifier: 1x1 conv 128 -> len(bins) (channels <= 512), softmax over the bins,
    `exp = sum_n p_n anchor_n`; train mode returns (logits, exp), eval mode exp.  `models/model.py:17-34`
    Regressor (bins is None): 1x1 conv 128 -> 1 + ReLU.
  * `models/utils.py:405-420` make_vgg_layers, `:366-379` _init_weights (reg_layer / classifier).

The network is plain PyTorch-ROCm (MIOpen convolutions, channels_last on the GPU); its training step's loss
is the HIP DACE/DMCount kernel (ebc_amd.losses).  The ImageNet VGG-19 weights are a download
(`vgg.py:44-45`), unavailable offline: `weights_seed` draws synthetic ones (ebc_amd.synthetic.vgg19_ae_state).
"""
from __future__ import annotations

from typing import Any, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.nn.functional as F
from torch import Tensor, nn

VGG_CFG_E = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512]


def make_vgg_layers(cfg: List[Union[str, int]], in_channels: int = 3) -> nn.Sequential:
    """models/utils.py:405-420 (batch_norm=False, dilation=1)."""
    layers: List[nn.Module] = []
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(in_channels, int(v), kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            in_channels = int(v)
    return nn.Sequential(*layers)


class VGGEncoderDecoder(nn.Module):
    """models/encoder_decoder/vgg.py:13-41."""

    def __init__(self, features: nn.Module, reduction: Optional[int] = None) -> None:
        super().__init__()
        self.features = features
        self.reg_layer = nn.Sequential(nn.Conv2d(512, 256, kernel_size=3, padding=1), nn.ReLU(inplace=True),
                                       nn.Conv2d(256, 128, kernel_size=3, padding=1), nn.ReLU(inplace=True))
        self.encoder_reduction = 16
        self.reduction = self.encoder_reduction if reduction is None else reduction
        self.channels = 128

    def forward(self, x: Tensor) -> Tensor:
        x = self.features(x)
        if self.encoder_reduction != self.reduction:
            x = F.interpolate(x, scale_factor=self.encoder_reduction / self.reduction, mode="bilinear")
        return self.reg_layer(x)


class Classifier(nn.Module):
    """models/model.py:37-75 (the EBC blockwise classification head on a non-CLIP backbone)."""

    def __init__(self, backbone: nn.Module, bins: List[Tuple[float, float]], anchor_points: List[float]) -> None:
        super().__init__()
        self.backbone = backbone
        self.reduction = backbone.reduction
        assert len(bins) == len(anchor_points), \
            f"Expected bins and anchor_points to have the same length, got {len(bins)} and {len(anchor_points)}"
        assert all(len(b) == 2 for b in bins), f"Expected bins to be a list of tuples of length 2, got {bins}"
        assert all(b[0] <= p <= b[1] for b, p in zip(bins, anchor_points)), \
            f"Expected anchor_points to be within the range of the corresponding bin, got {bins} and {anchor_points}"
        self.bins = bins
        self.anchor_points = torch.tensor(anchor_points, dtype=torch.float32, requires_grad=False).view(1, -1, 1, 1)
        if backbone.channels > 512:
            self.classifier = nn.Sequential(nn.Conv2d(backbone.channels, 512, kernel_size=1), nn.ReLU(inplace=True),
                                            nn.Conv2d(512, len(self.bins), kernel_size=1))
        else:
            self.classifier = nn.Conv2d(backbone.channels, len(self.bins), kernel_size=1)

    def forward(self, x: Tensor) -> Union[Tensor, Tuple[Tensor, Tensor]]:
        x = self.classifier(self.backbone(x))
        probs = x.softmax(dim=1)
        exp = (probs * self.anchor_points.to(x.device)).sum(dim=1, keepdim=True)
        return (x, exp) if self.training else exp


class Regressor(nn.Module):
    """models/model.py:17-34 (bins is None: a density regressor)."""

    def __init__(self, backbone: nn.Module) -> None:
        super().__init__()
        self.backbone = backbone
        self.reduction = backbone.reduction
        self.regressor = nn.Sequential(nn.Conv2d(backbone.channels, 1, kernel_size=1), nn.ReLU(inplace=True))
        self.bins = None
        self.anchor_points = None

    def forward(self, x: Tensor) -> Tensor:
        return self.regressor(self.backbone(x))


def vgg19_ae(reduction: int = 8) -> VGGEncoderDecoder:
    return VGGEncoderDecoder(make_vgg_layers(VGG_CFG_E), reduction=reduction)


def build(backbone: str, input_size: int, reduction: int, bins=None, anchor_points=None,
          weights_seed: Optional[int] = None, **kw: Any) -> nn.Module:
    """models/model.py:94-111 (`_regressor` / `_classifier`) for the vgg19_ae backbone."""
    if backbone != "vgg19_ae":
        raise NotImplementedError(f"{backbone}: of the non-CLIP backbones only vgg19_ae (BASELINE configs[0]) is built")
    bb = vgg19_ae(reduction=reduction)
    if bins is None and anchor_points is None:
        m: nn.Module = Regressor(bb)
    else:
        assert bins is not None and anchor_points is not None, \
            f"Expected bins and anchor_points to be both None or not None, got {bins} and {anchor_points}"
        m = Classifier(bb, bins, anchor_points)
    if weights_seed is not None:
        from .synthetic import vgg19_ae_state
        sd = vgg19_ae_state(weights_seed, n_bins=None if bins is None else len(bins))
        own = m.state_dict()
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items() if k in own}, strict=True)
    return m

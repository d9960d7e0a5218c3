"""clip_resnet50 (config 2) host-side parity, CPU only: the drop-in model's state_dict / trainable-parameter
layout, the PyTorch ModifiedResNet encoder's layer4 output and the 1024-wide text features, all against the
reference's own outputs on the same synthetic weights (tests/golden/f7_resnet50.npz, make_golden.py
resnet_case).  The decoder + head run on the HIP path: tests/test_gpu_resnet.py."""
import numpy as np
import pytest
import torch

from conftest import BINS, golden, rel_l2

ANCHORS_SHA = [0.0, 1.0, 2.0, 3.0, 4.29992]


@pytest.fixture(scope="module")
def model():
    from ebc_amd.model import get_model
    return get_model("clip_resnet50", 448, 8, BINS, ANCHORS_SHA, prompt_type="word", weights_seed=0)


def test_state_dict_keys_match_reference(model):
    d = golden("f7_resnet50.npz")
    assert sorted(model.state_dict().keys()) == list(d["state_keys"])
    assert sorted(k for k, p in model.named_parameters() if p.requires_grad) == list(d["trainable_keys"])


def test_geometry(model):
    assert model.encoder_reduction == 16 and model.reduction == 8          # layer4 at stride 1 (reduction <= 16)
    assert model.channels == 2048 and model.clip_embed_dim == 1024
    assert all(p.requires_grad for p in model.image_encoder.parameters())  # trainable for ResNet backbones
    assert not any(p.requires_grad for p in model.text_encoder.parameters())


def test_text_features_match_reference(model):
    d = golden("f7_resnet50.npz")
    assert rel_l2(model.text_features.numpy(), d["text_features"]) < 1e-5


def test_encoder_layer4_matches_reference(model):
    from ebc_amd import synthetic as syn
    d = golden("f7_resnet50.npz")
    img, _, _ = syn.synthetic_crops(2, int(d["size"]), seed=int(d["seed"]), counts=list(d["counts"]))
    enc = model.image_encoder
    state = {k: v.clone() for k, v in enc.state_dict().items()}
    enc.train()
    with torch.no_grad():
        out = enc(torch.from_numpy(img).contiguous(memory_format=torch.channels_last))
    enc.load_state_dict(state)                     # undo the BN running-stat update
    assert out.shape == (2, 2048, 28, 28)
    assert rel_l2(out.numpy()[:, ::7, ::3, ::3], d["enc_out_sub"]) < 1e-4

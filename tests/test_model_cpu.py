"""Host-side checks of the drop-in get_model surface (no GPU)."""
import pytest

from conftest import ANCHORS_NWPU, BINS


def test_vit_sequence_limit_is_rejected_at_get_model():
    """clip_vit_b_16 at 448 (the reference trainer's default --input_size: 1 + 32 + 784 = 817 tokens) builds -- the
    attention kernels stream sequences past 256 tokens through LDS in chunks -- and a sequence past the kernels' bound
    (2048x2048: 16417 tokens) is refused when the model is built, not at its first forward."""
    from ebc_amd.model import get_model
    m = get_model("clip_vit_b_16", 448, 8, BINS, ANCHORS_NWPU, prompt_type="word", num_vpt=32, deep_vpt=True,
                  vpt_drop=0.0, vit_layers=1, text_layers=1)
    assert m.image_encoder.positional_embedding.shape[0] == 28 * 28 + 1
    with pytest.raises(NotImplementedError, match="16417 tokens"):
        get_model("clip_vit_b_16", 2048, 8, BINS, ANCHORS_NWPU, prompt_type="word", num_vpt=32, deep_vpt=True,
                  vpt_drop=0.0, vit_layers=1, text_layers=1)
    m = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", num_vpt=32, deep_vpt=True,
                  vpt_drop=0.0, vit_layers=1, text_layers=1)
    assert m.num_vpt == 32


def test_packed_point_views_are_detected():
    """DACELoss's zero-copy path (losses._packed_views): crops' point lists that are consecutive rows of one f32
    [sum n, 2] buffer (incl. empty crops) are used in place; separate tensors, gaps, other dtypes or a different
    device take the concatenation."""
    import torch
    from ebc_amd.losses import _packed_views
    buf = torch.arange(20, dtype=torch.float32).reshape(10, 2)
    views = [buf[0:3], buf[3:3], buf[3:10]]
    assert _packed_views(views, "cpu")
    assert not _packed_views([buf[0:3], buf[4:10]], "cpu")                 # a gap
    assert not _packed_views([buf[3:10], buf[0:3]], "cpu")                 # out of order
    assert not _packed_views([buf[0:3].clone(), buf[3:10]], "cpu")         # another storage
    assert not _packed_views([buf.double()[0:3]], "cpu")
    assert not _packed_views([buf[:, :1]], "cpu")
    assert _packed_views([buf[0:0], buf[0:4], buf[4:10]], "cpu")      # an empty first crop

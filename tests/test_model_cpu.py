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

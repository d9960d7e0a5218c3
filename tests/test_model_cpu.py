"""Host-side checks of the drop-in get_model surface (no GPU)."""
import pytest

from conftest import ANCHORS_NWPU, BINS


def test_vit_sequence_limit_is_rejected_at_get_model():
    """clip_vit_b_16 at 448 (the reference trainer's default --input_size) is 1 + 32 + 784 = 817 tokens: more than the
    attention kernels' LDS-resident 256, refused when the model is built (not at its first forward)."""
    from ebc_amd.model import get_model
    with pytest.raises(NotImplementedError, match="817 tokens"):
        get_model("clip_vit_b_16", 448, 8, BINS, ANCHORS_NWPU, prompt_type="word", num_vpt=32, deep_vpt=True,
                  vpt_drop=0.0)
    m = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", num_vpt=32, deep_vpt=True,
                  vpt_drop=0.0, vit_layers=1, text_layers=1)
    assert m.num_vpt == 32

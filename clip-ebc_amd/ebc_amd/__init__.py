"""ebc_amd — MI355X-native (gfx950) CLIP-EBC training + inference hot path.

Drop-in for the reference's hot-path surface:
  * `get_model(...)`, `CLIP_EBC`          (models/__init__.py:10-44, models/clip/model.py:30-270)
  * `DACELoss`, `DMLoss`, `OTLoss`, `sinkhorn`  (losses/dace_loss.py, dm_loss.py, bregman_pytorch.py)
  * `sliding_window_predict`, `evaluate`  (utils/eval_utils.py, eval.py)
Hot ops run in libebc_hip.so (clip-ebc_amd/csrc, C-ABI in include/ebc_hip.h).
"""
from . import _lib  # noqa: F401
from .losses import DACELoss, DMLoss, OTLoss, sinkhorn  # noqa: F401

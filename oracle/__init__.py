"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference CLIP-EBC hot path, used as the checker for the HIP product
path (clip-ebc_amd/).  Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s
`cpu_baseline` leg may import it; the product never does.

  * `sinkhorn_oracle.c` — plain C Sinkhorn-Knopp + DMCount OT step
    (losses/bregman_pytorch.py:11-144, losses/dm_loss.py:38-79).
  * `ref.py` — torch-fp32 restatement of the model forward (models/clip/model.py:142-217,
    models/clip/_clip/blocks.py:8-42, models/utils.py:254-303) and of the DACE/DMCount loss
    (losses/dace_loss.py:42-70, losses/dm_loss.py:99-124); backward by torch autograd.

Pinned by tests/golden/*.npz, produced by running the reference itself in the build container
(tests/golden/make_golden.py); see tests/test_oracle_golden.py.
"""

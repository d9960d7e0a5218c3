"""GPU: sliding-window tiling + overlap averaging (ebc_tile_gather / ebc_tile_assemble) against the
reference's own outputs (F5 fixture: utils/eval_utils.py:26-96 run with a stub model), and the
full-model sliding-window path."""
import numpy as np
import pytest
import torch

from conftest import ANCHORS_NWPU, BINS, golden

pytestmark = pytest.mark.gpu


class Stub(torch.nn.Module):
    reduction = 8

    def forward(self, x):
        return torch.nn.functional.avg_pool2d(x.mean(1, keepdim=True).abs(), 8)


@pytest.mark.parametrize("case", range(4))
def test_sliding_window_matches_reference_fixture(case):
    from ebc_amd.eval_utils import sliding_window_predict
    d = golden("f5_sliding.npz")
    H, W, win, stride = (int(v) for v in d[f"cfg_{case}"])
    img = np.random.Generator(np.random.PCG64(11 + case)).standard_normal((1, 3, H, W)).astype(np.float32)
    out = sliding_window_predict(Stub(), torch.from_numpy(img).cuda(), win, stride, max_tiles_per_batch=5)
    assert out.shape == d[f"pred_{case}"].shape and out.device.type == "cpu"
    np.testing.assert_allclose(out.numpy(), d[f"pred_{case}"], rtol=2e-6, atol=1e-7)


def test_sliding_window_full_model_counts():
    """2-layer model on a 500x700 image: the tiled eval equals averaging per-tile model outputs."""
    from ebc_amd.eval_utils import sliding_window_predict, tile_grid
    from ebc_amd.model import get_model
    txt = torch.from_numpy(golden("f6_text.npz")["text_features_word"])
    m = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", vit_layers=2, text_features=txt, weights_seed=0).cuda().eval()
    img = torch.randn(1, 3, 500, 700, device="cuda")
    out = sliding_window_predict(m, img, 224, 224)
    rows, cols = tile_grid(500, 700, (224, 224), (224, 224))
    tiles, origins = [], []
    for i in range(rows):
        for j in range(cols):
            y = min(i * 224, 500 - 224); x = min(j * 224, 700 - 224)
            tiles.append(img[:, :, y:y + 224, x:x + 224]); origins.append((y, x))
    with torch.no_grad():
        preds = m(torch.cat(tiles)).cpu()
    acc = torch.zeros(1, 500 // 8, 700 // 8); cnt = torch.zeros_like(acc)
    for t, (y, x) in enumerate(origins):
        acc[:, y // 8:(y + 224) // 8, x // 8:(x + 224) // 8] += preds[t]
        cnt[:, y // 8:(y + 224) // 8, x // 8:(x + 224) // 8] += 1
    np.testing.assert_allclose(out[0].numpy(), (acc / cnt).numpy(), rtol=1e-5, atol=1e-6)


def _assemble(preds, H, W, win=224, r=8):
    from ebc_amd.eval_utils import tile_grid
    rows, cols = tile_grid(H, W, (win, win), (win, win))
    acc = torch.zeros(preds.shape[1], H // r, W // r, dtype=torch.float64)
    cnt = torch.zeros_like(acc)
    t = 0
    for i in range(rows):
        for j in range(cols):
            y, x = min(i * win, H - win), min(j * win, W - win)
            acc[:, y // r:(y + win) // r, x // r:(x + win) // r] += preds[t].double()
            cnt[:, y // r:(y + win) // r, x // r:(x + win) // r] += 1
            t += 1
    return (acc / cnt).float()


def test_sliding_window_qnrf_140_tiles():
    """BASELINE config 5's image: 2048x3072, window = stride = 224 -> 140 tiles in ONE forward (the M = 32060
    eval-batch GEMM instances), 12 layers.  fp32 (the reference's eval precision): equals the per-tile
    outputs (16 tiles per forward) assembled on the host; fp16 autocast: within 2e-2 of fp32."""
    from ebc_amd.eval_utils import sliding_window_predict, tile_grid
    from ebc_amd.model import get_model
    txt = torch.from_numpy(golden("f6_text.npz")["text_features_word"])
    m = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", text_features=txt,
                  weights_seed=0).cuda().eval()
    H, W = 2048, 3072
    g = np.random.Generator(np.random.PCG64(7))
    mean = np.array([0.485, 0.456, 0.406], np.float32).reshape(1, 3, 1, 1)
    std = np.array([0.229, 0.224, 0.225], np.float32).reshape(1, 3, 1, 1)
    img = torch.from_numpy(((g.random((1, 3, H, W), dtype=np.float32) - mean) / std).astype(np.float32)).cuda()
    rows, cols = tile_grid(H, W, (224, 224), (224, 224))
    assert rows * cols == 140
    out32 = sliding_window_predict(m, img, 224, 224)
    tiles = [img[:, :, min(i * 224, H - 224):min(i * 224, H - 224) + 224, min(j * 224, W - 224):min(j * 224, W - 224) + 224]
             for i in range(rows) for j in range(cols)]
    with torch.no_grad():
        preds = torch.cat([m(torch.cat(tiles[k:k + 16])).cpu() for k in range(0, 140, 16)])
    want = _assemble(preds, H, W)
    assert out32.shape == (1, 1, H // 8, W // 8)
    np.testing.assert_allclose(out32[0].numpy(), want.numpy(), rtol=2e-4, atol=1e-5)
    with torch.autocast("cuda", dtype=torch.float16):
        out16 = sliding_window_predict(m, img, 224, 224)
    rel = float((out16 - out32).norm() / out32.norm())
    assert rel < 2e-2, rel


def test_sliding_window_140_tiles_vs_oracle():
    """The config-5 eval (140 tiles of a 2048x3072 image, one forward, fp32) against an independent computation: the
    oracle restatement (oracle/ref.py: ViT-B/16 + deep VPT, eval-mode BasicBlock decoder, head) run per tile in
    fp32 torch on the same device with the model's own state_dict, assembled by the reference's overlap average
    (F5 pins that assembly).  Bar: the fp32 step's (rel-L2 1e-3 of the density map, max-abs 1e-3 of its scale)."""
    from ebc_amd.eval_utils import sliding_window_predict, tile_grid
    from ebc_amd.model import get_model
    from oracle import ref
    txt = torch.from_numpy(golden("f6_text.npz")["text_features_word"])
    m = get_model("clip_vit_b_16", 224, 8, BINS, ANCHORS_NWPU, prompt_type="word", text_features=txt,
                  weights_seed=0).cuda().eval()
    H, W = 2048, 3072
    g = np.random.Generator(np.random.PCG64(11))
    mean = np.array([0.485, 0.456, 0.406], np.float32).reshape(1, 3, 1, 1)
    std = np.array([0.229, 0.224, 0.225], np.float32).reshape(1, 3, 1, 1)
    img = torch.from_numpy(((g.random((1, 3, H, W), dtype=np.float32) - mean) / std).astype(np.float32)).cuda()
    rows, cols = tile_grid(H, W, (224, 224), (224, 224))
    out = sliding_window_predict(m, img, 224, 224)[0].cpu()
    p = {k: v.detach().clone().cuda().float() if v.is_floating_point() else v.detach().clone().cuda()
         for k, v in m.state_dict().items()}
    tiles = [img[:, :, min(i * 224, H - 224):min(i * 224, H - 224) + 224, min(j * 224, W - 224):min(j * 224, W - 224) + 224]
             for i in range(rows) for j in range(cols)]
    with torch.no_grad():
        preds = torch.cat([ref.forward(p, torch.cat(tiles[k:k + 20]), txt.cuda(), ANCHORS_NWPU, 12, train=False)[1].cpu()
                           for k in range(0, len(tiles), 20)])
    want = _assemble(preds, H, W)
    rel = float((out - want).norm() / want.norm())
    assert rel < 1e-3, rel
    assert float((out - want).abs().max()) < 1e-3 * float(want.abs().max())

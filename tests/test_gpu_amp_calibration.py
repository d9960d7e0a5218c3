"""16-bit parity of the ViT train step calibrated against PyTorch's own mixed-precision error.

The reference trains under `torch.cuda.amp.autocast` (train.py:36-40), so its own fp16 / bf16 step differs from an
fp32 step by PyTorch's AMP rounding.  Here the same synthetic weights and crops run three ways:
  truth  the oracle restatement (oracle/ref.py: ViT-B/16 + deep VPT(32), BasicBlock decoder, projection + head,
         DACE/DMCount) in fp32 on the CPU;
  amp    the same oracle on the GPU under torch.autocast(fp16 / bf16): PyTorch's AMP error on this very step;
  hip    the drop-in model + loss under the same autocast (the HIP kernels).
Every quantity must satisfy err(hip) <= 1.5 x err(amp) (relative L2 against truth), per quantity, NOT stacked:
the logits, the expected count, EACH of the 12 layers' prompt gradients (layer 0's comes from the trimmed
backward, vit.hip), the decoder's two conv weight gradients and the projection weight gradient.  At 224 (BASELINE
configs[2]/[3]) and at 448, the reference trainer's default input size (trainer.py:26): 817 tokens through the
chunked long-sequence attention, a 56x56 density grid.
"""
import numpy as np
import pytest
import torch

from conftest import ANCHORS_NWPU, BINS, golden, rel_l2
from oracle import ref
from ebc_amd import synthetic as syn

pytestmark = pytest.mark.gpu
LAYERS = 12
PARAMS = ["image_decoder.0.conv1.weight", "image_decoder.0.conv2.weight", "projection.weight"]


def _oracle(p_cpu, img, txt, dens, pts, device, amp, size=224):
    p = {k: v.detach().to(device).requires_grad_(v.requires_grad) for k, v in p_cpu.items()}
    x = torch.from_numpy(img).to(device)
    with torch.autocast("cuda", dtype=amp, enabled=amp is not None):
        lg, ex, _ = ref.forward(p, x, txt.to(device), ANCHORS_NWPU, LAYERS)
        loss, _ = ref.dace_loss(lg, ex, torch.from_numpy(dens).to(device), pts, BINS, input_size=size)
    loss.backward()
    out = {"logits": lg.detach().float().cpu(), "exp": ex.detach().float().cpu()}
    for l in range(LAYERS):
        out[f"vpt_{l}"] = p[f"vpt_{l}"].grad.detach().float().cpu()
    for k in PARAMS:
        out[k] = p[k].grad.detach().float().cpu()
    return out


def _hip(img, txt, dens, pts, amp, size=224, stats="benign"):
    from ebc_amd.losses import DACELoss
    from ebc_amd.model import get_model
    m = get_model("clip_vit_b_16", size, 8, BINS, ANCHORS_NWPU, prompt_type="word", text_features=txt,
                  weights_seed=0).cuda().train()
    if stats == "outlier":
        from test_gpu_model import load_outlier_stats
        load_outlier_stats(m)
    with torch.autocast("cuda", dtype=amp):
        lg, ex = m(torch.from_numpy(img).cuda())
        loss, _ = DACELoss(BINS, 8, count_loss="dmcount", input_size=size)(
            lg, ex, torch.from_numpy(dens).cuda(), [torch.from_numpy(q).cuda() for q in pts])
    loss.backward()
    torch.cuda.synchronize()
    sd = dict(m.named_parameters())
    out = {"logits": lg.detach().float().cpu(), "exp": ex.detach().float().cpu()}
    for l in range(LAYERS):
        out[f"vpt_{l}"] = sd[f"vpt_{l}"].grad.detach().float().cpu()
    for k in PARAMS:
        out[k] = sd[k].grad.detach().float().cpu()
    return out


@pytest.mark.parametrize("B,amp,size,stats", [(16, torch.float16, 224, "benign"), (32, torch.float16, 224, "benign"),
                                              (16, torch.bfloat16, 224, "benign"), (4, torch.float16, 448, "benign"),
                                              # massive-activation channels, a row offset, gammas over 0.1..10
                                              # (synthetic.outlier_stats)
                                              (16, torch.float16, 224, "outlier"), (16, torch.bfloat16, 224, "outlier")])
def test_step_error_within_pytorch_amp_error(B, amp, size, stats):
    txt = torch.from_numpy(golden("f6_text.npz")["text_features_word"])
    img, pts, dens = syn.synthetic_crops(B, size, seed=900 + B + (size if size != 224 else 0))
    sd = syn.full_state(0, layers=LAYERS, include_text=False, input_size=size)
    if stats == "outlier":
        sd = syn.outlier_stats(sd)
    p = ref.params_from_state(sd)
    truth = _oracle(p, img, txt, dens, pts, torch.device("cpu"), None, size)
    torch_amp = _oracle(p, img, txt, dens, pts, torch.device("cuda"), amp, size)
    hip = _hip(img, txt, dens, pts, amp, size, stats)
    worst, bad = 0.0, []
    for k in truth:
        e_amp, e_hip = rel_l2(torch_amp[k], truth[k]), rel_l2(hip[k], truth[k])
        ratio = e_hip / max(e_amp, 1e-30)
        worst = max(worst, ratio)
        print(f"{k:32s} hip {e_hip:.3e}  torch-amp {e_amp:.3e}  ratio {ratio:.2f}")
        if e_hip > 1.5 * e_amp:
            bad.append((k, e_hip, e_amp))
    print(f"B={B} {amp} {size}x{size} {stats}: worst hip / torch-amp error ratio {worst:.2f}")
    assert not bad, bad

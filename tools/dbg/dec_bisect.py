"""Debug: the f32 decoder block at 2 and 3 crops (28x28, C = 768) against the f64 reference, per parameter and per
image, on the library at EBC_LIB_PATH (bisecting the r04 decoder-gradient regression across builds)."""
import os
import sys
import torch
sys.path.insert(0, "tests")
sys.path.insert(0, "clip-ebc_amd")
from ebc_amd import _lib
import ctypes
lib = ctypes.CDLL(_lib.LIB_PATH)
for name in list(_lib.SIGNATURES):
    if not hasattr(lib, name):
        del _lib.SIGNATURES[name]                 # an older build: entries added since are not called here
from test_gpu_decoder import _block, _ref
from ebc_amd.model import _DecoderFn
print("lib", _lib.LIB_PATH)
for B in (2, 3):
    C, h, up = 768, 14, 2
    blk = _block(C)
    gcpu = torch.Generator().manual_seed(1)
    feat = torch.randn(B, h, h, C, generator=gcpu)
    Hh = h * up
    gy = torch.randn(B, Hh, Hh, C, generator=gcpu)
    params = [p.detach().double().requires_grad_() for p in
              (blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight, blk.bn2.bias)]
    fr = feat.double().requires_grad_()
    rm = [blk.bn1.running_mean.double().clone(), blk.bn2.running_mean.double().clone()]
    rv = [blk.bn1.running_var.double().clone(), blk.bn2.running_var.double().clone()]
    yr = _ref(fr, *params, up, rm, rv, True)
    (yr * gy.double()).sum().backward()
    blk = blk.cuda().train()
    fd = feat.cuda().requires_grad_()
    y = _DecoderFn.apply(fd, blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
                         blk.bn2.bias, blk, up, torch.float32, True)
    (y.float() * gy.cuda()).sum().backward()
    gd = fd.grad.cpu().double()
    print("B", B, "y %.2e" % float((y.detach().cpu().double() - yr.detach()).norm() / yr.detach().norm()),
          "dfeat/img", ["%.2e" % float((gd[b] - fr.grad[b]).norm() / fr.grad[b].norm()) for b in range(B)],
          " ".join("%s %.2e" % (n, float((p.grad.cpu().double() - r.grad).norm() / r.grad.norm()))
                   for n, p, r in zip(("w1", "g1", "b1", "w2", "g2", "b2"),
                                      (blk.conv1.weight, blk.bn1.weight, blk.bn1.bias, blk.conv2.weight, blk.bn2.weight,
                                       blk.bn2.bias), params)))

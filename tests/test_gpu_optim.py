"""ebc_amd.optim (csrc/optim.hip ebc_adam_step) against torch's own optimizer step.

The reference steps Adam(params, lr, weight_decay) (utils/train_utils.py:80-85) under GradScaler (trainer.py:123,
train.py:54-57).  The HIP step restates torch's fused Adam operation for operation (double hyper-parameter
products), so against torch.optim.Adam(fused=True) + torch.amp.GradScaler the scale sequence (a skipped non-finite
step, growth) and the unscaled gradients are the same bits and parameters / moments agree to f32 rounding (the
compilers may contract a*b + c*d into different fused multiply-adds: an exp_avg_sq element can differ in its last
bit); against the reference's default (foreach) Adam, within f32 rounding (rel 1e-6).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _params(shapes, seed, dev, offset=0):
    """Parameters from one seeded stream; offset > 0 puts each at element `offset` of its storage (not 16-B aligned)."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for s in shapes:
        n = 1
        for d in s:
            n *= d
        base = torch.randn(n + offset, generator=g).to(dev)
        out.append(torch.nn.Parameter(base[offset:].reshape(s)))
    return out


def _grads(shapes, step, seed, scale):
    g = torch.Generator().manual_seed(1000 * seed + step)
    return [torch.randn(s, generator=g) * scale for s in shapes]


def _run(shapes, opt_kind, steps, inf_at, seed=0, offset=0, amp=True, growth_interval=2, lr=1e-3, wd=1e-4):
    from ebc_amd import optim as eo
    dev = torch.device("cuda:0")
    ps = _params(shapes, seed, dev, offset)
    if opt_kind == "ebc":
        opt = eo.Adam(ps, lr=lr, weight_decay=wd)
        sc = eo.GradScaler(growth_interval=growth_interval, enabled=amp)
    else:
        opt = torch.optim.Adam(ps, lr=lr, weight_decay=wd, fused=opt_kind == "fused", foreach=opt_kind == "foreach")
        sc = torch.amp.GradScaler("cuda", growth_interval=growth_interval, enabled=amp)
    scales, grads_after = [], []
    for i in range(steps):
        sc.scale(torch.ones((), device=dev))              # torch's scaler creates its scale tensor here
        s = sc.get_scale() if amp else 1.0
        gs = _grads(shapes, i, seed, s)
        if i == inf_at:
            gs[len(gs) // 2].view(-1)[0] = float("inf")
        opt.zero_grad(set_to_none=True)
        for p, g in zip(ps, gs):
            p.grad = g.to(dev)
        sc.step(opt)
        sc.update()
        scales.append(sc.get_scale() if amp else 1.0)
        grads_after.append([p.grad.detach().clone() for p in ps])
    torch.cuda.synchronize()
    mom = [(opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone()) for p in ps]
    return [p.detach().clone() for p in ps], mom, scales, grads_after


SHAPES = [(32, 768)] * 12 + [()] + [(768, 768, 3, 3), (768,), (768,), (768, 768, 3, 3), (768,), (768,), (512, 768, 1, 1), (512,)]


def test_adam_amp_vs_torch_fused():
    pe, me, se, ge = _run(SHAPES, "ebc", 6, inf_at=2)
    pt, mt, st, gt = _run(SHAPES, "fused", 6, inf_at=2)
    assert se == st, (se, st)                             # backoff at the inf step, growth every 2 applied steps
    same = tot = 0
    for i, (a, b) in enumerate(zip(pe, pt)):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-9, msg=f"param {i}")
        same += int((a == b).sum()); tot += a.numel()
    for i, ((a1, a2), (b1, b2)) in enumerate(zip(me, mt)):
        torch.testing.assert_close(a1, b1, rtol=1e-6, atol=1e-12, msg=f"exp_avg {i}")
        torch.testing.assert_close(a2, b2, rtol=1e-6, atol=1e-15, msg=f"exp_avg_sq {i}")
    assert same >= 0.999 * tot, (same, tot)               # the parameters are (nearly all) the same bits
    for step in (0, 1, 3, 5):                             # unscaled gradients written back (applied steps)
        for a, b in zip(ge[step], gt[step]):
            assert torch.equal(a, b)


def test_adam_matches_reference_foreach_adam():
    """The reference constructs Adam with torch's default implementation (foreach on CUDA)."""
    pe, me, _, _ = _run(SHAPES, "ebc", 5, inf_at=3)
    pt, mt, _, _ = _run(SHAPES, "foreach", 5, inf_at=3)
    for a, b in zip(pe, pt):
        assert torch.allclose(a, b, rtol=1e-6, atol=1e-7), float((a - b).abs().max())


def test_adam_no_scaler_many_groups_unaligned():
    """> 32 tensors (several launches), odd sizes, a tensor whose storage offset breaks 16-B alignment, no AMP."""
    shapes = [(7,), (13, 5), (1,), (4099,), (64, 65)] * 8
    pe, me, _, _ = _run(shapes, "ebc", 3, inf_at=-1, amp=False, offset=1)
    pt, mt, _, _ = _run(shapes, "fused", 3, inf_at=-1, amp=False, offset=1)
    for a, b in zip(pe, pt):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-9)


def test_adam_state_dict_roundtrip():
    from ebc_amd import optim as eo
    pe, _, _, _ = _run(SHAPES[:3], "ebc", 2, inf_at=-1)
    dev = torch.device("cuda:0")
    ps = _params(SHAPES[:3], 0, dev)
    opt = eo.Adam(ps, lr=1e-3, weight_decay=1e-4)
    for p in ps:
        p.grad = torch.ones_like(p)
    opt.step()
    sd = opt.state_dict()
    assert float(sd["state"][0]["step"]) == 1.0
    opt2 = eo.Adam(_params(SHAPES[:3], 0, dev), lr=1e-3, weight_decay=1e-4)
    opt2.load_state_dict(sd)
    assert float(opt2.state_dict()["state"][0]["step"]) == 1.0


def test_adam_channels_last_params_and_strided_grads():
    """clip_resnet50's MIOpen stem leaves channels-last conv weights / gradients: the step runs in memory order on a
    parameter's own dense layout and takes a gradient in another layout through a copy in the parameter's."""
    from ebc_amd import optim as eo
    dev = torch.device("cuda:0")
    res = {}
    for kind in ("ebc", "torch"):
        g = torch.Generator().manual_seed(5)
        p1 = torch.nn.Parameter(torch.randn(8, 3, 5, 5, generator=g).to(dev).to(memory_format=torch.channels_last))
        p2 = torch.nn.Parameter(torch.randn(6, 4, generator=g).to(dev))
        opt = eo.Adam([p1, p2], lr=1e-3, weight_decay=1e-4) if kind == "ebc" else \
            torch.optim.Adam([p1, p2], lr=1e-3, weight_decay=1e-4, foreach=True)   # fused refuses mixed layouts
        for i in range(3):
            gg = torch.Generator().manual_seed(100 + i)
            p1.grad = torch.randn(8, 3, 5, 5, generator=gg).to(dev)                  # contiguous: p1 is channels-last
            p2.grad = torch.randn(4, 6, generator=gg).to(dev).t()                     # a transposed view
            opt.step()
        res[kind] = (p1.detach().clone(), p2.detach().clone())
    for a, b in zip(res["ebc"], res["torch"]):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-9)

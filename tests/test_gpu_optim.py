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


def test_adam_resume_torch_state_into_channels_last_params():
    """a torch.optim.Adam checkpoint's moments are contiguous NCHW; resumed into channels-last parameters
    they are re-laid out in the parameter's memory order (values kept), so the next steps match torch resuming the
    same state."""
    from ebc_amd import optim as eo
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(11)
    w0 = torch.randn(8, 3, 5, 5, generator=g)
    src = torch.nn.Parameter(w0.clone().to(dev))                                # contiguous, as a checkpoint holds it
    topt = torch.optim.Adam([src], lr=1e-3, weight_decay=1e-4)
    for i in range(2):
        src.grad = torch.randn(8, 3, 5, 5, generator=torch.Generator().manual_seed(200 + i)).to(dev)
        topt.step()
    sd = topt.state_dict()
    res = {}
    for kind in ("ebc", "torch"):
        p = torch.nn.Parameter(src.detach().clone().to(memory_format=torch.channels_last))
        opt = eo.Adam([p], lr=1e-3, weight_decay=1e-4) if kind == "ebc" else \
            torch.optim.Adam([p], lr=1e-3, weight_decay=1e-4, foreach=True)
        opt.load_state_dict(sd)
        for i in range(3):
            p.grad = torch.randn(8, 3, 5, 5, generator=torch.Generator().manual_seed(300 + i)).to(dev)
            opt.step()
        res[kind] = p.detach().clone()
    assert not res["ebc"].is_contiguous()
    torch.testing.assert_close(res["ebc"], res["torch"], rtol=1e-6, atol=1e-9)


def test_grad_scaler_resume_before_first_step_keeps_tracker():
    """the reference loads the scaler state right after building it (utils/train_utils.py:122-123),
    before any step; the growth tracker must survive, as torch keeps it (_init_growth_tracker)."""
    from ebc_amd import optim as eo
    dev = torch.device("cuda:0")
    seq = {}
    for kind in ("ebc", "torch"):
        p = torch.nn.Parameter(torch.ones(64, device=dev))
        if kind == "ebc":
            opt, sc = eo.Adam([p], lr=1e-3), eo.GradScaler(growth_interval=4)
        else:
            opt, sc = torch.optim.Adam([p], lr=1e-3, fused=True), torch.amp.GradScaler("cuda", growth_interval=4)
        loaded = {"scale": 1024.0, "growth_factor": 2.0, "backoff_factor": 0.5, "growth_interval": 4,
                  "_growth_tracker": 3}
        sc.load_state_dict(loaded)
        # a checkpoint saved right after resuming (before any step) keeps what was loaded
        assert sc.state_dict() == loaded, (kind, sc.state_dict())
        out = []
        for i in range(3):
            sc.scale(torch.ones((), device=dev))
            p.grad = torch.full((64,), 0.5, device=dev) * sc.get_scale()
            sc.step(opt)
            sc.update()
            out.append(sc.get_scale())
        seq[kind] = out
    assert seq["ebc"] == seq["torch"] == [2048.0, 2048.0, 2048.0], seq


def test_grad_scaler_update_new_scale_after_step():
    """update(new_scale) after a step: the scale is set, the tracker stays where it was before that step, and the
    next step runs (it raised 'step() has already been called')."""
    from ebc_amd import optim as eo
    dev = torch.device("cuda:0")
    seq = {}
    for kind in ("ebc", "torch"):
        p = torch.nn.Parameter(torch.ones(64, device=dev))
        if kind == "ebc":
            opt, sc = eo.Adam([p], lr=1e-3), eo.GradScaler(init_scale=256.0, growth_interval=2)
        else:
            opt, sc = torch.optim.Adam([p], lr=1e-3, fused=True), torch.amp.GradScaler("cuda", init_scale=256.0,
                                                                                          growth_interval=2)
        out = []
        for i in range(4):
            sc.scale(torch.ones((), device=dev))
            p.grad = torch.full((64,), 0.5, device=dev) * sc.get_scale()
            sc.step(opt)
            if i == 1:
                sc.update(64.0)
            else:
                sc.update()
            out.append((sc.get_scale(), int(sc.state_dict()["_growth_tracker"])))
        seq[kind] = (out, p.detach().clone())
    assert seq["ebc"][0] == seq["torch"][0], (seq["ebc"][0], seq["torch"][0])
    torch.testing.assert_close(seq["ebc"][1], seq["torch"][1], rtol=1e-6, atol=1e-9)


def test_adam_two_groups_inf_in_second_group_skips_both():
    """with several param groups under one scaler, a non-finite gradient in ANY group skips every group's
    update (torch skips the whole optimizer step); the step counts advance together afterwards."""
    from ebc_amd import optim as eo
    dev = torch.device("cuda:0")
    res = {}
    for kind in ("ebc", "torch"):
        a = torch.nn.Parameter(torch.linspace(-1, 1, 100, device=dev))
        b = torch.nn.Parameter(torch.linspace(2, 3, 50, device=dev))
        groups = [{"params": [a], "lr": 1e-3}, {"params": [b], "lr": 2e-3, "weight_decay": 1e-2}]
        if kind == "ebc":
            opt, sc = eo.Adam(groups), eo.GradScaler(init_scale=8.0, growth_interval=100)
        else:
            opt, sc = torch.optim.Adam(groups, fused=True), torch.amp.GradScaler("cuda", init_scale=8.0, growth_interval=100)
        snaps = []
        for i in range(3):
            sc.scale(torch.ones((), device=dev))
            s = sc.get_scale()
            a.grad = torch.full((100,), 0.25, device=dev) * s
            b.grad = torch.full((50,), -0.5, device=dev) * s
            if i == 1:
                b.grad[7] = float("inf")
            sc.step(opt)
            sc.update()
            snaps.append((a.detach().clone(), b.detach().clone(), sc.get_scale()))
        res[kind] = snaps
    for (ea, eb, es), (ta, tb, ts) in zip(res["ebc"], res["torch"]):
        assert es == ts
        torch.testing.assert_close(ea, ta, rtol=1e-6, atol=1e-9)
        torch.testing.assert_close(eb, tb, rtol=1e-6, atol=1e-9)
    assert torch.equal(res["ebc"][0][0], res["ebc"][1][0])           # group 0 untouched at the skipped step

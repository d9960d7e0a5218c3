"""Adam + GradScaler for the training step, on HIP (csrc/optim.hip, `ebc_adam_step`).

Drop-in for the reference's optimizer step: `Adam(params, lr, weight_decay)` (utils/train_utils.py:80-85) under
`GradScaler()` (trainer.py:123), driven as train.py:53-57::

    optimizer.zero_grad(); grad_scaler.scale(loss).backward(); grad_scaler.step(optimizer); grad_scaler.update()

`Adam` is a torch.optim.Optimizer (param_groups, lr schedulers such as the reference's LambdaLR, state_dict);
`GradScaler` mirrors torch.amp.GradScaler's dynamic loss scaling (init 2**16, growth 2 every 2000 applied steps,
backoff 0.5, a step with a non-finite gradient skipped).  One step is two launches over all trainable tensors
(an inf check, then the update with the unscale; the next scale and step count are written by the same launch)
where torch's GradScaler + fused Adam issue about ten (check, fills, copies, the update, the scale update).
The arithmetic is torch's fused Adam's, operation for operation (tests/test_gpu_optim.py: same scale sequence and
unscaled gradients, parameters and moments to f32 rounding).

Scope: f32 parameters on one HIP device, L2 weight decay (Adam, not AdamW), no amsgrad / maximize; one
optimizer per GradScaler per iteration (the reference has one); several param groups share the scaler's skip decision
(ebc_amp_check over every group, then ebc_adam_update per group).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import torch

from . import _lib


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense: the elements fill numel consecutive slots from data_ptr() in some dim order."""
    if t.is_contiguous():
        return True
    dims = sorted((st, sz) for st, sz in zip(t.stride(), t.shape) if sz != 1)
    expect = 1
    for st, sz in dims:
        if st != expect:
            return False
        expect *= sz
    return True


class Adam(torch.optim.Optimizer):
    """torch.optim.Adam(params, lr, betas, eps, weight_decay) with its step on HIP."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0):
        if lr < 0.0 or eps < 0.0 or weight_decay < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self._steps: Dict[int, torch.Tensor] = {}      # per param group: device float[2] step count (ping-pong)
        self._parity: Dict[int, int] = {}

    def _group_tensors(self, gi: int, group) -> List[_lib.EbcAdamTensor]:
        """The launch's flat view: the update is elementwise, so each tensor is taken in memory order -- param,
        gradient and moments must share one dense layout (a channels-last conv weight from MIOpen included): a
        gradient in another layout is replaced by a copy in the parameter's (p.grad keeps its values)."""
        out = []
        for p in group["params"]:
            if p.grad is None:
                continue
            if p.dtype != torch.float32 or p.grad.dtype != torch.float32 or not p.is_cuda:
                raise RuntimeError("ebc_amd.optim.Adam: f32 HIP parameters and gradients only")
            if p.grad.is_sparse or not _dense(p):
                raise RuntimeError("ebc_amd.optim.Adam: dense (non-overlapping) parameters and gradients only")
            if p.grad.stride() != p.stride() or not _dense(p.grad):
                p.grad = torch.empty_like(p).copy_(p.grad)                  # the parameter's layout
            st = self.state[p]
            if not st:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            for k in ("exp_avg", "exp_avg_sq"):
                # moments loaded from a torch.optim.Adam state_dict keep the layout they were saved in (e.g.
                # contiguous NCHW beside a channels-last conv weight): re-laid out in the parameter's memory order,
                # values kept, so the elementwise update pairs each parameter element with its own moments
                m = st[k]
                if m.stride() != p.stride() or not _dense(m) or m.dtype != torch.float32 or m.device != p.device:
                    st[k] = torch.empty_like(p).copy_(m)
            out.append(_lib.EbcAdamTensor(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                          st["exp_avg_sq"].data_ptr(), p.numel()))
        return out

    def _step_buf(self, gi: int, device) -> torch.Tensor:
        if gi not in self._steps:
            self._steps[gi] = torch.zeros(2, dtype=torch.float32, device=device)
            self._parity[gi] = 0
        return self._steps[gi]

    @torch.no_grad()
    def _launch(self, scaler: Optional["GradScaler"]) -> None:
        lib = _lib.lib()
        groups = []
        for gi, group in enumerate(self.param_groups):
            ts = self._group_tensors(gi, group)
            if not ts:
                continue
            dev = group["params"][0].device
            for p in group["params"]:
                if p.device != dev:
                    raise RuntimeError("ebc_amd.optim.Adam: one device per param group")
            groups.append((gi, group, ts, dev))
        if not groups:
            return
        if scaler is not None:
            devs = {d for _, _, _, d in groups}
            if len(devs) != 1:
                raise RuntimeError("ebc_amd.optim.Adam: a GradScaler'd step runs on one device")
            dev = groups[0][3]
            sbuf, spar = scaler._state(dev), scaler._parity
            sc = _lib.ptr(sbuf, dev)
            gf, bf, gint = scaler._growth_factor, scaler._backoff_factor, scaler._growth_interval
        else:
            sc, spar, gf, bf, gint = None, 0, 2.0, 0.5, 1
        # one group (the reference's case): check + update in one call; several groups sharing a scaler: the inf
        # check over every group's gradients first, so a non-finite gradient in any group skips them all (torch)
        split = scaler is not None and len(groups) > 1
        if split:
            every = [t for _, _, ts, _ in groups for t in ts]
            with _lib.on(dev):
                _lib.check(lib.ebc_amp_check((_lib.EbcAdamTensor * len(every))(*every), len(every), sc, spar,
                                             _lib.stream(dev)), "ebc_amp_check")
        fn = lib.ebc_adam_update if split else lib.ebc_adam_step
        for gi, group, ts, gdev in groups:
            steps = self._step_buf(gi, gdev)
            arr = (_lib.EbcAdamTensor * len(ts))(*ts)
            b1, b2 = group["betas"]
            with _lib.on(gdev):
                _lib.check(fn(arr, len(ts), _lib.ptr(steps, gdev), self._parity[gi], sc, spar,
                              float(group["lr"]), float(b1), float(b2), float(group["eps"]),
                              float(group["weight_decay"]), float(gf), float(bf), int(gint), 1,
                              _lib.stream(gdev)), "ebc_adam_step")
            self._parity[gi] ^= 1

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._launch(None)
        return loss

    def state_dict(self):
        """torch.optim.Adam's layout: per-param exp_avg, exp_avg_sq and `step` (a 0-d f32 tensor)."""
        sd = super().state_dict()
        for gi, group in enumerate(self.param_groups):
            if gi not in self._steps:
                continue
            stepv = self._steps[gi][self._parity[gi]].detach().clone()
            for p in group["params"]:
                idx = self._index_of(p)
                if idx in sd["state"]:
                    sd["state"][idx]["step"] = stepv.clone()
        return sd

    def _index_of(self, p) -> int:
        i = 0
        for group in self.param_groups:
            for q in group["params"]:
                if q is p:
                    return i
                i += 1
        raise KeyError(p)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                st = self.state.get(p, {})
                if "step" in st:
                    buf = self._step_buf(gi, p.device)
                    buf.fill_(float(st.pop("step")))
                    self._parity[gi] = 0


class GradScaler:
    """torch.amp.GradScaler("cuda") for an ebc_amd.optim.Adam: scale(loss), step(optimizer), update().

    The scale, growth tracker and found-inf flag live on the device (float[2][3], ping-pong with the optimizer's
    launch, include/ebc_hip.h ebc_adam_step); nothing is read back to the host."""

    def __init__(self, device: str = "cuda", init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, enabled: bool = True):
        if growth_factor <= 1.0 or not (0.0 < backoff_factor < 1.0) or growth_interval <= 0:
            raise ValueError("invalid GradScaler hyper-parameter")
        self._init_scale = float(init_scale)
        self._growth_factor = float(growth_factor)
        self._backoff_factor = float(backoff_factor)
        self._growth_interval = int(growth_interval)
        self._enabled = bool(enabled)
        self._init_tracker = 0
        self._buf: Optional[torch.Tensor] = None
        self._parity = 0
        self._stepped = False

    def is_enabled(self) -> bool:
        return self._enabled

    def _state(self, device) -> torch.Tensor:
        if self._buf is None:
            # both entries seeded with the scale and growth tracker (a loaded state_dict's, torch's
            # _init_growth_tracker, when load_state_dict ran before the first step: utils/train_utils.py:122-123)
            self._buf = torch.tensor([[self._init_scale, float(self._init_tracker), 0.0]] * 2, dtype=torch.float32,
                                     device=device)
        return self._buf

    def scale(self, outputs):
        if not self._enabled:
            return outputs
        s = self._state(outputs.device)[self._parity, 0]
        return outputs * s.to(outputs.dtype) if outputs.dtype != torch.float32 else outputs * s

    def step(self, optimizer, *args, **kwargs):
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        if not isinstance(optimizer, Adam):
            raise TypeError("ebc_amd.optim.GradScaler steps an ebc_amd.optim.Adam")
        if self._stepped:
            raise RuntimeError("step() has already been called since the last update().")
        optimizer._launch(self)
        self._stepped = True
        return None

    def update(self, new_scale=None) -> None:
        if not self._enabled:
            return
        if new_scale is not None:
            # torch.amp.GradScaler.update(new_scale): the scale becomes new_scale, the growth tracker is left as it
            # was before the step; the step's launch already wrote the other entry, which the next step reads
            buf = self._state(self._buf.device if self._buf is not None else "cuda")
            if self._stepped:
                buf[1 - self._parity, 1].copy_(buf[self._parity, 1])
                self._parity ^= 1
                self._stepped = False
            buf[self._parity, 0].fill_(float(new_scale))
            return
        if self._stepped:
            self._parity ^= 1        # the step's launch wrote the next scale / tracker into the other entry
            self._stepped = False

    def get_scale(self) -> float:
        if not self._enabled:
            return 1.0
        return float(self._state("cuda")[self._parity, 0]) if self._buf is not None else self._init_scale

    def state_dict(self):
        if not self._enabled:
            return {}
        # before the first step: the loaded (or initial) tracker, as torch returns _init_growth_tracker
        tr = float(self._buf[self._parity, 1]) if self._buf is not None else float(self._init_tracker)
        return {"scale": self.get_scale(), "growth_factor": self._growth_factor, "backoff_factor": self._backoff_factor,
                "growth_interval": self._growth_interval, "_growth_tracker": int(tr)}

    def load_state_dict(self, sd) -> None:
        if not sd:
            return
        self._init_scale = float(sd["scale"])
        self._growth_factor = float(sd["growth_factor"])
        self._backoff_factor = float(sd["backoff_factor"])
        self._growth_interval = int(sd["growth_interval"])
        self._init_tracker = int(sd["_growth_tracker"])
        if self._buf is not None:
            self._buf[self._parity, 0] = self._init_scale
            self._buf[self._parity, 1] = float(self._init_tracker)

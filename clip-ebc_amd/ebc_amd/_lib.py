"""ctypes binding of libebc_hip.so (the C-ABI declared in include/ebc_hip.h).

The product path has no fallback: if the library or a HIP device is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("EBC_LIB_PATH") or os.path.join(PKG_ROOT, "lib", "libebc_hip.so")   # override: tuning builds

EBC_F32, EBC_F16, EBC_BF16 = 0, 1, 2
EBC_COUNT_DMCOUNT, EBC_COUNT_MAE, EBC_COUNT_MSE, EBC_COUNT_OT_ONLY = 0, 1, 2, 3
_ERR = {-1: "EBC_E_ARG", -2: "EBC_E_LAUNCH", -3: "EBC_E_UNSUPPORTED"}

_lib: Optional[ctypes.CDLL] = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_Z = ctypes.c_size_t
_D = ctypes.c_double
_L = ctypes.c_long


class EbcCropDesc(ctypes.Structure):
    """include/ebc_hip.h EbcCropDesc (one augmented training crop)."""
    _fields_ = [("src_off", ctypes.c_int64), ("out_off", ctypes.c_int64), ("tmp_off", ctypes.c_int64),
                ("noise_off", ctypes.c_int64),
                ("src_h", ctypes.c_int32), ("src_w", ctypes.c_int32), ("top", ctypes.c_int32), ("left", ctypes.c_int32),
                ("crop_h", ctypes.c_int32), ("crop_w", ctypes.c_int32), ("out_h", ctypes.c_int32), ("out_w", ctypes.c_int32),
                ("flip", ctypes.c_int32), ("jitter_ops", ctypes.c_int32),
                ("brightness", ctypes.c_float), ("contrast", ctypes.c_float), ("saturation", ctypes.c_float),
                ("blur", ctypes.c_int32), ("noise", ctypes.c_int32),
                ("saltiness", ctypes.c_float), ("spiciness", ctypes.c_float),
                ("seed", ctypes.c_uint32), ("normalize", ctypes.c_int32), ("hue", ctypes.c_float)]


class EbcProbeRecord(ctypes.Structure):
    """include/ebc_hip.h EbcProbeRecord (one instrumented launch)."""
    _fields_ = [(n, ctypes.c_int) for n in ("kind", "epi", "bm", "bn", "mode", "m", "n", "k")] + [("ms", ctypes.c_float)]


PROBE_KINDS = {1: "gemm", 2: "dace_loss", 3: "attn_fwd", 4: "attn_bwd_dq", 5: "attn_bwd_dkv", 6: "ln_fwd", 7: "ln_bwd"}


class EbcAugConst(ctypes.Structure):
    """include/ebc_hip.h EbcAugConst (passed by value)."""
    _fields_ = [("mean", ctypes.c_float * 3), ("std", ctypes.c_float * 3), ("blur_k", ctypes.c_int32),
                ("sigma_x", ctypes.c_float), ("sigma_y", ctypes.c_float)]


class EbcAdamTensor(ctypes.Structure):
    """include/ebc_hip.h EbcAdamTensor (one f32 tensor of the optimizer step)."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_long)]


# name -> (restype, argtypes); must mirror include/ebc_hip.h
SIGNATURES = {
    "ebc_version": (_I, []),
    "ebc_dace_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "ebc_scale2": (_I, [_P, _P, _P, _L, _P, _P, _L, _P]),
    "ebc_dace_loss_h": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _F, _F, _I, _F, _I,
                             _P, _P, _P, _P, _P, _P, _P, _Z, _P]),
    "ebc_dace_loss": (_I, [_P, _P, _P, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _F, _F, _F, _F, _I, _F, _I,
                           _P, _P, _P, _P, _P, _P, _P, _Z, _P]),
    "ebc_sinkhorn_workspace_bytes": (_Z, [_I, _I]),
    "ebc_sinkhorn": (_I, [_P, _P, _P, _I, _I, _F, _I, _F, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _Z, _P]),
    "ebc_gemm": (_I, [_I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "ebc_gemm_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "ebc_gemm_tile_config": (_I, [_I, _I, _I, _I, _P]),
    "ebc_conv_tile_config": (_I, [_I, _I, _I, _I, _I, _P]),
    "ebc_gemm_ws": (_I, [_I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P, _Z, _P]),
    "ebc_gemm_wgrad_workspace_bytes": (_Z, [_I, _I, _I, _I]),
    "ebc_gemm_wgrad": (_I, [_I, _P, _P, _P, _I, _I, _I, _P, _Z, _P]),
    "ebc_transpose": (_I, [_I, _P, _P, _I, _I, _L, _P]),
    "ebc_vit_workspace_bytes": (_Z, [_I, _I, _I, _I, _I, _I, _I]),
    "ebc_vit_forward": (_I, [_P, _P, _I, _I, _I, _P, ctypes.c_long, _I, _I, _P, _Z, _P, _P]),
    "ebc_vit_backward": (_I, [_P, _I, _I, _I, _I, _P, _Z, _P, _P, ctypes.c_long, _I, _P]),
    "ebc_set_weight_touch": (_I, [_I]),
    "ebc_layernorm_fwd": (_I, [_I, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _P]),
    "ebc_layernorm_bwd": (_I, [_I, _I, _P, _P, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _I, _P]),
    "ebc_attention_fwd": (_I, [_I, _P, _P, _P, _I, _I, _I, _P]),
    "ebc_attention_bwd": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "ebc_head_fwd": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ebc_head_bwd": (_I, [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _Z, _P]),
    "ebc_head_bwd_workspace_bytes": (_Z, [_I, _I]),
    "ebc_cast_f32": (_I, [_I, _P, _P, _Z, _P]),
    "ebc_tile_gather": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "ebc_tile_assemble": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "ebc_dec_geometry": (_I, [_I, _I, _I, _I, _I, _P]),
    "ebc_dec_workspace_bytes": (_Z, [_I, _I, _I, _I, _I, _I]),
    "ebc_dec_upsample_pad": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "ebc_conv3x3_fwd": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _P]),
    "ebc_conv3x3_wgrad": (_I, [_I, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _P]),
    "ebc_bn_finalize": (_I, [_P, _D, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "ebc_conv3x3_fwd_bn": (_I, [_I, _P, _P, _P, _P, _Z, _I, _I, _I, _I, _I, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P,
                                _P, _P, _P]),
    "ebc_bn_relu_pad": (_I, [_I, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ebc_bn_add_relu": (_I, [_I, _P, _P, _P, _P, _I, _P, _I, _I, _I, _I, _P]),
    "ebc_bn_bwd_reduce": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _Z, _L, _I, _P]),
    "ebc_bn_bwd_finalize": (_I, [_P, _D, _P, _P, _P, _P, _P, _I, _P]),
    "ebc_bn_bwd_apply": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ebc_dec_transpose3": (_I, [_I, _P, _P, _I, _I, _I, _I, _P]),
    "ebc_dec_prep_weights": (_I, [_I, _P, _P, _P, _I, _I, _P]),
    "ebc_dec_upsample_bwd": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "ebc_dec_upsample": (_I, [_I, _P, _P, _I, _I, _I, _I, _I, _P]),
    "ebc_bn_stats": (_I, [_I, _P, _P, _P, _Z, _L, _I, _P]),
    "ebc_bn_stats_finalize": (_I, [_I, _P, _P, _Z, _L, _I, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "ebc_bn_bwd_reduce_finalize": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _Z, _L, _I, _P]),
    "ebc_bn_relu": (_I, [_I, _P, _P, _P, _P, _L, _I, _P]),
    "ebc_bn_bwd_apply_flat": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P]),
    "ebc_bn_relu_avgpool": (_I, [_I, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "ebc_avgpool2": (_I, [_I, _I, _P, _P, _I, _I, _I, _I, _P]),
    "ebc_avgpool2_bwd": (_I, [_I, _I, _P, _P, _I, _I, _I, _I, _P]),
    "ebc_bn_add_relu_flat": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P]),
    "ebc_prep_weights_1x1": (_I, [_I, _P, _P, _P, _I, _I, _P]),
    "ebc_augment_crops": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, EbcAugConst, _P]),
    "ebc_point_map": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "ebc_adam_step": (_I, [_P, _I, _P, _I, _P, _I, _D, _D, _D, _D, _D, _D, _D, _I, _I, _P]),
    "ebc_amp_check": (_I, [_P, _I, _P, _I, _P]),
    "ebc_adam_update": (_I, [_P, _I, _P, _I, _P, _I, _D, _D, _D, _D, _D, _D, _D, _I, _I, _P]),
    "ebc_probe_begin": (_I, [_I]),
    "ebc_probe_end": (_I, [_P, _I]),
    "ebc_marker": (_I, [_I, _P]),
}


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the library (host-side symbols only; no device work)."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise RuntimeError(f"libebc_hip.so not built at {path}: run `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def lib() -> ctypes.CDLL:
    """The library, for a compute call: requires a HIP device."""
    if not torch.cuda.is_available():
        raise RuntimeError("ebc_amd: no HIP device visible; the MI355X path has no CPU fallback")
    return load()


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {_ERR.get(rc, rc)}")


def ptr(t: Optional[torch.Tensor], device: Optional[torch.device] = None):
    """Raw device pointer of a contiguous HIP tensor; with `device`, the tensor must live there (every
    operand of a launch is on the launch stream's device)."""
    if t is None:
        return None
    assert t.is_cuda and t.is_contiguous(), "ebc_amd kernels take contiguous device tensors"
    if device is not None and t.device != _as_device(device):
        raise RuntimeError(f"ebc_amd: operand on {t.device}, launch stream on {device}")
    return ctypes.c_void_p(t.data_ptr())


def _as_device(where) -> Optional[torch.device]:
    if where is None:
        return None
    dev = where.device if isinstance(where, torch.Tensor) else torch.device(where)
    if dev.type == "cuda" and dev.index is None:                     # "cuda" = the current device
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def stream(where=None) -> ctypes.c_void_p:
    """The current torch stream of the device `where` (a tensor or a device) lives on -- NOT the current
    device's: the reference trainer builds its model on f"cuda:{local_rank}" without set_device
    (trainer.py:93, utils/ddp_utils.py:16-22), so the two can differ on ranks > 0."""
    dev = _as_device(where)
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def on(where):
    """Context manager making `where`'s device current for a block of library calls: the library's own
    device queries (hipGetDevice, hipFuncSetAttribute) and its memsets then target the operands' GPU."""
    return torch.cuda.device(_as_device(where))


def dtype_code(dt: torch.dtype) -> int:
    return {torch.float32: EBC_F32, torch.float16: EBC_F16, torch.bfloat16: EBC_BF16}[dt]

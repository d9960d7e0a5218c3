"""CPU checks of the C-ABI boundary: libebc_hip.so loads, exports every symbol include/ebc_hip.h
declares, the ctypes signature table covers them, and host-only entry points answer (no device work)."""
import os
import re
import subprocess

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "ebc_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ebc_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from ebc_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(REPO, "clip-ebc_amd")])
    return _lib.load()


def test_header_declares_the_hot_path():
    fns = declared_functions()
    for f in ("ebc_dace_loss", "ebc_gemm", "ebc_vit_forward", "ebc_vit_backward", "ebc_attention_fwd",
              "ebc_attention_bwd", "ebc_head_fwd", "ebc_head_bwd", "ebc_layernorm_fwd", "ebc_layernorm_bwd"):
        assert f in fns


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", os.path.join(REPO, "clip-ebc_amd", "lib", "libebc_hip.so")]).decode()
    exported = set(re.findall(r"\bT (ebc_[a-z0-9_]+)", out))
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    for f in declared_functions():
        getattr(lib, f)


def test_ctypes_table_matches_header(lib):
    from ebc_amd import _lib
    assert set(_lib.SIGNATURES) == set(declared_functions())


def test_host_only_entry_points(lib):
    assert lib.ebc_version() >= 1
    # workspace sizing is pure host arithmetic
    assert lib.ebc_dace_workspace_bytes(16, 600, 224, 8) >= 4 * 58 * 600
    b_train = lib.ebc_vit_workspace_bytes(16, 224, 224, 12, 32, 1, 1)
    b_eval = lib.ebc_vit_workspace_bytes(16, 224, 224, 12, 32, 1, 0)
    assert b_train > 12 * 16 * 229 * 768 * 4 and b_eval < b_train / 4


def test_argument_validation_without_device(lib):
    # rejected before any device work
    assert lib.ebc_gemm(1, 0, 0, None, None, None, None, None, None, 16, 64, 64, None) == -1
    assert lib.ebc_dace_loss(None, None, None, 0, None, None, None, None, None, 0, 5, 224, 8, 0, 0, 1.0, 0.1,
                             0.01, 10.0, 100, 1e-9, 10, *([None] * 7), 0, None) == -1


def test_product_has_no_cpu_fallback():
    """The product path refuses to run without a HIP device rather than falling back."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ebc_amd import _lib
    with pytest.raises(RuntimeError):
        _lib.lib()

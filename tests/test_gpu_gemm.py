"""GPU numerics of the MFMA GEMM (all epilogues, f32/f16/bf16) against a torch fp64 reference."""
import pytest
import torch

from ebc_amd import _lib

pytestmark = pytest.mark.gpu

DT = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}
TOL = {"f32": 2e-6, "f16": 2e-3, "bf16": 1.6e-2}


def _gemm(dt, epi, out_f32, A, B, bias=None, resid=None, aux=None, C=None):
    M, K = A.shape
    N = B.shape[0]
    if C is None:
        od = torch.float32 if (out_f32 or dt == torch.float32 or epi == 2) else dt
        C = torch.empty(M, N, device=A.device, dtype=od)
    rc = _lib.lib().ebc_gemm(_lib.dtype_code(dt), epi, int(out_f32), _lib.ptr(A), _lib.ptr(B), _lib.ptr(C),
                             _lib.ptr(bias), _lib.ptr(resid), _lib.ptr(aux), M, N, K, _lib.stream())
    _lib.check(rc, "ebc_gemm")
    return C


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("M,N,K", [(3664, 2304, 768), (458, 768, 3072), (37, 128, 64), (1000, 512, 768), (3664, 768, 768)])
def test_gemm_store_bias(dname, M, N, K):
    if dname == "f32" and K % 32:
        pytest.skip()
    dt = DT[dname]
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g)
    ref = A.double() @ B.double().t() + bias.double()
    C = _gemm(dt, 0, 1, A, B, bias=bias)
    assert _rel(C, ref) < TOL[dname]
    if dt != torch.float32:
        C16 = _gemm(dt, 0, 0, A, B, bias=bias)
        assert C16.dtype == dt and _rel(C16, ref) < 2 * TOL[dname] + 4e-3


@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
def test_gemm_gelu_and_backward(dname):
    dt = DT[dname]
    M, N, K = 777, 3072, 768
    g = torch.Generator(device="cuda").manual_seed(7)
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    aux = torch.empty(M, N, device="cuda", dtype=dt)
    C = _gemm(dt, 1, 0, A, B, bias=bias, aux=aux)
    pre = A.double() @ B.double().t() + bias.double()
    ref = pre * torch.sigmoid(1.702 * pre)
    assert _rel(aux, pre) < TOL[dname] + (4e-3 if dt != torch.float32 else 0)
    assert _rel(C, ref) < TOL[dname] + (4e-3 if dt != torch.float32 else 0)
    # backward: dA = (dG . W2) * gelu'(pre)
    W2t = (torch.randn(N, 768, device="cuda", generator=g) / 768 ** 0.5).to(dt)   # [N_out=3072, K=768]
    dG = torch.randn(M, 768, device="cuda", generator=g).to(dt)
    D = _gemm(dt, 3, 0, dG, W2t, aux=aux)
    a = aux.double()
    s = torch.sigmoid(1.702 * a)
    ref_d = (dG.double() @ W2t.double().t()) * (s + 1.702 * a * s * (1 - s))
    assert _rel(D, ref_d) < TOL[dname] + (4e-3 if dt != torch.float32 else 0)


@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
def test_gemm_residual_inplace(dname):
    dt = DT[dname]
    M, N, K = 3664, 768, 3072
    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g)
    X = torch.randn(M, N, device="cuda", generator=g)
    ref = X.double() + A.double() @ B.double().t() + bias.double()
    _gemm(dt, 2, 1, A, B, bias=bias, resid=X, C=X)
    assert _rel(X, ref) < TOL[dname]


def test_gemm_rejects_bad_shapes():
    A = torch.zeros(16, 48, device="cuda", dtype=torch.float16)
    B = torch.zeros(64, 48, device="cuda", dtype=torch.float16)
    C = torch.zeros(16, 64, device="cuda", dtype=torch.float16)
    rc = _lib.lib().ebc_gemm(1, 0, 0, _lib.ptr(A), _lib.ptr(B), _lib.ptr(C), None, None, None, 16, 64, 48, _lib.stream())
    assert rc == -1


def _gemm_ws(dt, epi, out_f32, A, B, ws, bias=None, resid=None, aux=None, C=None):
    M, K = A.shape
    N = B.shape[0]
    if C is None:
        od = torch.float32 if (out_f32 or epi == 2) else dt
        C = torch.empty(M, N, device=A.device, dtype=od)
    rc = _lib.lib().ebc_gemm_ws(_lib.dtype_code(dt), epi, int(out_f32), _lib.ptr(A), _lib.ptr(B), _lib.ptr(C),
                                _lib.ptr(bias), _lib.ptr(resid), _lib.ptr(aux), M, N, K, _lib.ptr(ws), ws.numel(),
                                _lib.stream())
    _lib.check(rc, "ebc_gemm_ws")
    return C


@pytest.mark.parametrize("dname", ["f16", "bf16"])
def test_gemm_wide_tile_gelu(dname):
    """M=3664, N=3072 picks the 256x192 tile (cfg 3: 8 waves, 2-stage ring of 128-B K rows)."""
    import ctypes
    dt = DT[dname]
    M, N, K = 3664, 3072, 768
    tile = (ctypes.c_int * 3)()
    assert _lib.lib().ebc_gemm_tile_config(_lib.dtype_code(dt), M, N, K, tile) == 3 and tuple(tile) == (256, 192, 1)
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    aux = torch.empty(M, N, device="cuda", dtype=dt)
    C = _gemm(dt, 1, 0, A, B, bias=bias, aux=aux)
    pre = A.double() @ B.double().t() + bias.double()
    assert _rel(aux, pre) < TOL[dname] + 4e-3
    assert _rel(C, pre * torch.sigmoid(1.702 * pre)) < TOL[dname] + 4e-3


@pytest.mark.parametrize("dname", ["f16", "bf16"])
@pytest.mark.parametrize("M,N,K,epi", [(3664, 768, 3072, 2), (3664, 768, 2304, 0), (3136, 768, 3072, 0),
                                       (3664, 3072, 768, 3)])
def test_gemm_split_k(dname, M, N, K, epi):
    """Split-K through ebc_gemm_ws: partial tiles + last-arriver reduction, counters re-armed."""
    dt = DT[dname]
    lib = _lib.lib()
    nbytes = lib.ebc_gemm_workspace_bytes(_lib.dtype_code(dt), M, N, K)
    ws = torch.zeros(max(nbytes, 16), device="cuda", dtype=torch.uint8)
    g = torch.Generator(device="cuda").manual_seed(M + K + epi)
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    bias = torch.randn(N, device="cuda", generator=g) if epi != 3 else None
    ref = A.double() @ B.double().t()
    if bias is not None:
        ref = ref + bias.double()
    if epi == 2:
        X = torch.randn(M, N, device="cuda", generator=g)
        ref = ref + X.double()
        for _ in range(2):                          # the second call reuses the re-armed counters
            Xi = X.clone()
            _gemm_ws(dt, 2, 1, A, B, ws, bias=bias, resid=Xi, C=Xi)
            assert _rel(Xi, ref) < TOL[dname]
    elif epi == 3:
        aux = torch.randn(M, N, device="cuda", generator=g).to(dt)
        a = aux.double()
        s = torch.sigmoid(1.702 * a)
        ref = ref * (s + 1.702 * a * s * (1 - s))
        C = _gemm_ws(dt, 3, 0, A, B, ws, aux=aux)
        assert _rel(C, ref) < TOL[dname] + 4e-3
    else:
        for _ in range(2):
            C = _gemm_ws(dt, 0, 1, A, B, ws, bias=bias)
            assert _rel(C, ref) < TOL[dname]
    torch.cuda.synchronize()
    if nbytes:
        assert int(ws[:16384].view(torch.int32).abs().sum()) == 0, "split-K counters not re-armed"


@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("R,C,ld", [(12544, 512, 12544), (1568, 768, 1600), (8, 64, 8)])
def test_transpose_exact(dname, R, C, ld):
    dt = DT[dname]
    x = torch.randn(R, C, device="cuda").to(dt)
    out = torch.full((C, ld), 7.0, device="cuda", dtype=dt)
    _lib.check(_lib.lib().ebc_transpose(_lib.dtype_code(dt), _lib.ptr(x), _lib.ptr(out), R, C, ld, _lib.stream()),
               "ebc_transpose")
    assert torch.equal(out[:, :R], x.t())
    assert bool((out[:, R:] == 7.0).all())                   # padding columns untouched


@pytest.mark.parametrize("dname", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("M,N,K", [(512, 768, 12544), (512, 768, 1600), (128, 64, 64), (300, 192, 2048)])
def test_gemm_wgrad(dname, M, N, K):
    """Projection dW (split-K, deterministic last-arriver sum) vs fp64, and run-to-run bit equality."""
    dt = DT[dname]
    if K % (32 if dname == "f32" else 64):
        pytest.skip()
    g = torch.Generator(device="cuda").manual_seed(M * 7 + K)
    A = torch.randn(M, K, device="cuda", generator=g).to(dt)
    B = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
    L = _lib.lib()
    nb = L.ebc_gemm_wgrad_workspace_bytes(_lib.dtype_code(dt), M, N, K)
    ws = torch.zeros(max(nb, 16), device="cuda", dtype=torch.uint8)
    outs = []
    for _ in range(2):
        C = torch.empty(M, N, device="cuda")
        _lib.check(L.ebc_gemm_wgrad(_lib.dtype_code(dt), _lib.ptr(A), _lib.ptr(B), _lib.ptr(C), M, N, K, _lib.ptr(ws),
                                    ws.numel(), _lib.stream()), "ebc_gemm_wgrad")
        outs.append(C)
    ref = A.double() @ B.double().t()
    assert _rel(outs[0], ref) < TOL[dname]
    assert torch.equal(outs[0], outs[1])
    assert int(ws[:16 * 1024].count_nonzero()) == 0          # split-K counters re-armed

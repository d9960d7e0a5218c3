"""Micro-benchmark of ebc_gemm on the ViT-B/16 (B=16) shapes vs torch/hipBLASLt, HIP-event timed."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

from ebc_amd import _lib  # noqa: E402

M = int(os.environ.get("GB_M", 16 * 229))
SHAPES = [  # (name, N, K, epilogue)
    ("qkv", 2304, 768, 0), ("out+res", 768, 768, 2), ("fc+gelu", 3072, 768, 1), ("proj+res", 768, 3072, 2),
    ("bwd gelu'", 3072, 768, 3), ("bwd dH2", 768, 3072, 0), ("bwd dO", 768, 768, 0), ("bwd dH", 768, 2304, 0),
]
if os.environ.get("GB_SET") == "proj":   # the 1x1 projection conv 768 -> 512 over B*784 pixels and its dX
    M = int(os.environ.get("GB_M", 16 * 784))
    SHAPES = [("proj", 512, 768, 0, 1), ("proj dX", 768, 512, 0, 0)]     # (.., f32 output)


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    L = _lib.lib()
    dt = torch.float16
    tot_e = tot_t = 0.0
    for name, N, K, epi, *of in SHAPES:
        OUT_F32 = of[0] if of else 0
        A = torch.randn(M, K, device="cuda").to(dt)
        B = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        bias = torch.randn(N, device="cuda")
        aux = torch.randn(M, N, device="cuda").to(dt)
        C = torch.empty(M, N, device="cuda", dtype=torch.float32 if epi == 2 or OUT_F32 else dt)
        R = torch.randn(M, N, device="cuda")

        nb = L.ebc_gemm_workspace_bytes(1, M, N, K)
        ws = torch.zeros(max(nb, 16), device="cuda", dtype=torch.uint8)

        def ours():
            _lib.check(L.ebc_gemm_ws(1, epi, OUT_F32, _lib.ptr(A), _lib.ptr(B), _lib.ptr(C), _lib.ptr(bias), _lib.ptr(R),
                                     _lib.ptr(aux), M, N, K, _lib.ptr(ws), ws.numel(), _lib.stream()), "gemm")

        def theirs():
            torch.nn.functional.linear(A, B)
        if os.environ.get("GB_CHECK") and epi == 0:      # the forced tile's main loop against torch (fp32 sum)
            ours()
            ref = A.float() @ B.float().t() + bias
            err = ((C.float() - ref).norm() / ref.norm()).item()
            print(f"  check {name}: rel-L2 {err:.2e}")
            assert err < 2e-3, err
        t1, t2 = timeit(ours), timeit(theirs)
        f = 2.0 * M * N * K
        tot_e += t1; tot_t += t2
        print(f"{name:10s} M={M} N={N:5d} K={K:5d}  ebc {t1*1e6:7.1f} us {f/t1/1e12:6.1f} TF/s | torch {t2*1e6:7.1f} us {f/t2/1e12:6.1f} TF/s")
    print(f"layer total: ebc {tot_e*1e6:.1f} us  torch(plain, no epilogue) {tot_t*1e6:.1f} us")


if __name__ == "__main__":
    main()

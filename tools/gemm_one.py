"""Run one GEMM shape repeatedly (for rocprofv3 PMC passes)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "clip-ebc_amd"))
import torch
from ebc_amd import _lib
M, N, K, epi = (int(x) for x in sys.argv[1:5])
dt = torch.float16
A = torch.randn(M, K, device="cuda").to(dt); B = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
bias = torch.randn(N, device="cuda"); aux = torch.randn(M, N, device="cuda").to(dt)
C = torch.empty(M, N, device="cuda", dtype=torch.float32 if epi == 2 else dt); R = torch.randn(M, N, device="cuda")
L = _lib.lib()
for _ in range(int(os.environ.get("REPS", "20"))):
    _lib.check(L.ebc_gemm(1, epi, 0, _lib.ptr(A), _lib.ptr(B), _lib.ptr(C), _lib.ptr(bias), _lib.ptr(R), _lib.ptr(aux), M, N, K, _lib.stream()), "g")
torch.cuda.synchronize()

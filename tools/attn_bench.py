"""Attention kernels alone at the bench shape (B=16, L=229, H=12, f16), HIP-event timed."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402

from ebc_amd import _lib  # noqa: E402


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
    L_ = _lib.lib()
    B, L, H = int(os.environ.get("AB", 16)), 229, 12
    dt = _lib.EBC_F16
    qkv = (torch.randn(B * L, 3 * H * 64, device="cuda") * 0.5).half()
    out = torch.empty(B * L, H * 64, device="cuda", dtype=torch.float16)
    lse = torch.empty(B, H, L, device="cuda")
    dout = (torch.randn(B * L, H * 64, device="cuda") * 0.1).half()
    delta = torch.empty(B, H, L, device="cuda")
    dqkv = torch.empty_like(qkv)
    st = _lib.stream()
    tf = timeit(lambda: L_.ebc_attention_fwd(dt, _lib.ptr(qkv), _lib.ptr(out), _lib.ptr(lse), B, L, H, st))
    tb = timeit(lambda: L_.ebc_attention_bwd(dt, _lib.ptr(qkv), _lib.ptr(dout), _lib.ptr(out), _lib.ptr(lse),
                                              _lib.ptr(delta), _lib.ptr(dqkv), B, L, H, st))
    f = 4.0 * B * H * L * L * 64
    print(f"attention B={B} L={L} H={H}: fwd {tf*1e6:6.1f} us ({f/tf/1e12:5.0f} TF/s) | bwd (delta+dq+dkv) {tb*1e6:6.1f} us "
          f"({2.5*f/tb/1e12:5.0f} TF/s)")
    # numerics vs torch (fp32 math on the same fp16 inputs)
    q, k, v = qkv.float().view(B, L, 3, H, 64).unbind(2)
    s = torch.einsum("blhd,bmhd->bhlm", q, k) * 0.125
    o = torch.einsum("bhlm,bmhd->blhd", s.softmax(-1), v).reshape(B * L, H * 64)
    print("fwd max abs err", float((out.float() - o).abs().max()))


if __name__ == "__main__":
    main()

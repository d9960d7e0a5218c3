"""CU-masked side stream lab (r06): can a long weight-gradient GEMM run on a few CUs reserved by a CU mask
(hipExtStreamCreateWithCUMask) while the main stream's one-wave GEMMs (<= 240 tiles) keep their time?

For each mask pattern: the c_fc-shaped main product alone (20 launches, HIP events), the decoder conv's
weight-gradient-shaped GEMM alone on the masked stream, then both at once.  Patterns name which of the 256
logical CU bits are set (hip_runtime_api.h: "the first 32 bits represent the first 32 CUs"; how the runtime maps
them onto the 8 XCDs is what the lab finds out).
    python tools/lab/cu_mask_lab.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "clip-ebc_amd"))
import torch  # noqa: E402
from ebc_amd import _lib  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def masked_stream(bits):
    words = (ctypes.c_uint32 * 8)()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(8), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


PATTERNS = {
    "none": None,
    "lo16": list(range(16)),                                  # bits 0..15
    "2per32": [i for i in range(256) if i % 32 in (0, 1)],     # 2 of every 32 consecutive bits
    "every16": [i for i in range(256) if i % 16 == 0],         # 1 of every 16
    "lo32": list(range(32)),
}


def main():
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    h = torch.float16
    M, N, K = 3664, 3072, 768
    A = torch.randn(M, K, device=dev, dtype=h)
    B = torch.randn(N, K, device=dev, dtype=h)
    C = torch.empty(M, N, device=dev, dtype=h)
    WM, WN, WK = 768, 6912, 12544
    WA = torch.randn(WM, WK, device=dev, dtype=h)
    WB = torch.randn(WN, WK, device=dev, dtype=h)
    WC = torch.empty(WM, WN, device=dev, dtype=torch.float32)
    wsb = L.ebc_gemm_wgrad_workspace_bytes(_lib.EBC_F16, WM, WN, WK)
    ws = torch.zeros(max(wsb, 1 << 20), device=dev, dtype=torch.uint8)
    main_st = torch.cuda.current_stream()

    def main_gemm():
        _lib.check(L.ebc_gemm(_lib.EBC_F16, 0, 0, _lib.ptr(A), _lib.ptr(B), _lib.ptr(C), None, None, None, M, N, K,
                              ctypes.c_void_p(main_st.cuda_stream)), "gemm")

    def side_gemm(st):
        _lib.check(L.ebc_gemm_wgrad(_lib.EBC_F16, _lib.ptr(WA), _lib.ptr(WB), _lib.ptr(WC), WM, WN, WK, _lib.ptr(ws),
                                    ws.numel(), ctypes.c_void_p(st.cuda_stream)), "wgrad")

    def time_main(n=20):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main_st)
        for _ in range(n):
            main_gemm()
        e1.record(main_st)
        return e0, e1, n

    for _ in range(3):
        main_gemm()
    torch.cuda.synchronize()
    e0, e1, n = time_main()
    torch.cuda.synchronize()
    base = e0.elapsed_time(e1) * 1e3 / n
    print(f"main GEMM alone: {base:.2f} us", flush=True)
    for name, bits in PATTERNS.items():
        st = torch.cuda.Stream() if bits is None else masked_stream(bits)
        with torch.cuda.stream(st):
            side_gemm(st)
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(st)
        side_gemm(st)
        s1.record(st)
        torch.cuda.synchronize()
        alone = s0.elapsed_time(s1) * 1e3
        # concurrent: the side GEMM, then the main launches on the main stream right behind it
        s0.record(st)
        side_gemm(st)
        s1.record(st)
        e0, e1, n = time_main(40)
        torch.cuda.synchronize()
        conc_side = s0.elapsed_time(s1) * 1e3
        conc_main = e0.elapsed_time(e1) * 1e3 / n
        print(f"{name:8s} side alone {alone:8.1f} us | concurrent: main {conc_main:6.2f} us/launch (x{conc_main / base:.3f}), "
              f"side {conc_side:8.1f} us", flush=True)


if __name__ == "__main__":
    main()

"""Probe the GPU box: device, torch GEMM / SDPA / conv rates at the CLIP-EBC shapes."""
import time, torch, os, json
torch.backends.cudnn.benchmark = True
d = torch.device("cuda:0")
p = torch.cuda.get_device_properties(0)
print("device", p.name, p.multi_processor_count, p.total_memory / 2**30, "GiB", "cpus", len(os.sched_getaffinity(0)))
def t(fn, n=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - s) / n
M = 16 * 229
for (N, K) in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]:
    for dt in [torch.float16, torch.float32]:
        a = torch.randn(M, K, device=d, dtype=dt); w = torch.randn(N, K, device=d, dtype=dt)
        s = t(lambda: torch.nn.functional.linear(a, w))
        print(f"linear M={M} N={N} K={K} {dt}: {s*1e6:.1f} us {2*M*N*K/s/1e12:.1f} TF/s")
q = torch.randn(16, 12, 229, 64, device=d, dtype=torch.float16)
s = t(lambda: torch.nn.functional.scaled_dot_product_attention(q, q, q))
print(f"sdpa fwd: {s*1e6:.1f} us")
x = torch.randn(16, 768, 28, 28, device=d, dtype=torch.float16)
c = torch.nn.Conv2d(768, 768, 3, padding=1, bias=False).to(d).half()
s = t(lambda: c(x)); print(f"conv3x3 NCHW fp16: {s*1e6:.1f} us {2*16*784*768*768*9/s/1e12:.1f} TF/s")
xc = x.to(memory_format=torch.channels_last); cc = c.to(memory_format=torch.channels_last)
s = t(lambda: cc(xc)); print(f"conv3x3 NHWC fp16: {s*1e6:.1f} us {2*16*784*768*768*9/s/1e12:.1f} TF/s")
cb = torch.nn.Conv2d(768, 768, 3, padding=1, bias=False).to(d).bfloat16()
xb = x.bfloat16()
s = t(lambda: cb(xb)); print(f"conv3x3 NCHW bf16: {s*1e6:.1f} us {2*16*784*768*768*9/s/1e12:.1f} TF/s")

"""Vendor-library ceiling for the s16x3 input projection as one plain f16 GEMM with K' = 3K
(A' = [a_hi | a_hi | a_lo'], W' = [2^11 w_hi | w_lo' | w_hi]); timing only, no parity."""
import torch

def t(fn, n=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(n):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1000.0

M, N = 256 * 266, 2048
for K in (512, 768):
    a = torch.randn(M, 3 * K, device="cuda", dtype=torch.float16)
    w = torch.randn(3 * K, N, device="cuda", dtype=torch.float16)
    f = 2.0 * M * N * 3 * K
    us = t(lambda: torch.mm(a, w))
    print(f"K={K} f16 out: {us:.1f} us  {f / us / 1e6:.0f} TF/s (f16)")
    try:
        us = t(lambda: torch.mm(a, w, out_dtype=torch.float32))
        print(f"K={K} f32 out: {us:.1f} us  {f / us / 1e6:.0f} TF/s (f16)")
    except Exception as ex:
        print("out_dtype unsupported:", ex)
    wt = w.t().contiguous()
    us = t(lambda: torch.mm(a, wt.t()))
    print(f"K={K} NT f16 out: {us:.1f} us")

"""fp32 GEMM reference points on MI355X for the decode / encoder shapes (torch.mm -> vendor
BLAS).  Diagnostics only: tells what a plain library GEMM reaches on these skinny shapes."""
import torch

torch.backends.cuda.matmul.allow_tf32 = False


def t(M, N, K, reps=50):
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    for _ in range(5):
        torch.mm(a, b)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / reps
    print(f"M={M:6d} N={N:5d} K={K:5d}: {us:9.2f} us  {2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)


for (M, N, K) in [(256, 5004, 1024), (1024, 5004, 1024), (256, 2048, 1280), (1024, 2048, 1280),
                  (68096, 2048, 720), (68096, 2048, 512), (34048, 2048, 512)]:
    t(M, N, K)

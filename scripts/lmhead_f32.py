"""lm_head at decode batch 256 (128256 x 4096): bf16 GEMM + fp32 reduce vs one GEMM with fp32 output."""
import time
import torch
dev = "cuda:0"
x = torch.randn(256, 4096, device=dev).bfloat16()
ws = [torch.randn(128256, 4096, device=dev).bfloat16() for _ in range(2)]
def t(fn, n=20):
    for _ in range(3): fn(0)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for i in range(n): fn(i)
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e6
a = t(lambda i: torch.matmul(x, ws[i % 2].t()).float())
b = t(lambda i: torch.mm(x, ws[i % 2].t(), out_dtype=torch.float32))
r1 = torch.matmul(x, ws[0].t()).float(); r2 = torch.mm(x, ws[0].t(), out_dtype=torch.float32)
print(f"bf16 GEMM + fp32 cast {a:.1f} us | fp32-output GEMM {b:.1f} us | max diff {(r1 - r2).abs().max().item():.4f}")

"""Round-2 fault follow-up (profiles/r2c_splitk_probe.md): the K-split probe's lm_head case
(N = 128256, K = 4096, M = 256) faulted inside the library GEMM with an OVERLAPPING strided-batched
B view -- W.view(N, S, ks).permute(1, 2, 0): batch stride ks (2048) elements, while one batch's
(ks x N) matrix spans ld x N = 4096 x 128256 elements, so consecutive batches interleave inside the
same 1.05 GB.  This check runs the same GEMM with NON-overlapping batches (each K slice copied to
its own contiguous [N, ks] block: batch stride N * ks) and the plain single GEMM, and compares both
with fp32; it does not re-run the faulting view.  The shipped engine never issues a strided-batched
library GEMM (decode: gemm_q.hip tile kernel; prefill: one torch.matmul on a contiguous dequantised
scratch matrix)."""
import torch

dev = torch.device("cuda:0")
M, N, K, S = 256, 128256, 4096, 2
ks = K // S
W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
x = torch.randn(M, K, device=dev).to(torch.bfloat16)
ref = x.float() @ W.float().t()
single = (x @ W.t()).float()
Wc = W.view(N, S, ks).permute(1, 0, 2).contiguous()          # [S, N, ks], batch stride N * ks: disjoint
xs = x.view(M, S, ks).permute(1, 0, 2).contiguous()          # [S, M, ks]
split = torch.bmm(xs, Wc.transpose(1, 2)).float().sum(0)      # [S, M, N] bf16 slabs summed in fp32
torch.cuda.synchronize()
e1 = float((single - ref).abs().max() / ref.abs().max())
e2 = float((split - ref).abs().max() / ref.abs().max())
print(f"LMHEAD_BMM_OK single rel err {e1:.2e}, disjoint-batch K-split rel err {e2:.2e}")

"""Launch driver for counter runs of the prefill GEMM (gemm_pp.hip) against hipBLASLt on the
Llama-3-8B gate|up shape at M = 8192: Q4_K (in-kernel dequant), bf16 weights (same kernel, W by
DMA) and the library GEMM on the same bf16 weights; 3 warm launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
M, K = 8192, 4096
w = rand_qweight(28672, K, GGMLType.Q4_K, 0)
wf = (torch.randn(28672, K, device=DEV) * 0.02).to(torch.bfloat16)
wb = ops.QWeight.from_float(wf)
x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
out = torch.empty(M, w.N, dtype=torch.bfloat16, device=DEV)
for _ in range(3):
    ops._run_pp(x, [w], 1, out, w.N)
for _ in range(3):
    ops._run_pp(x, [wb], 1, out, w.N)
for _ in range(3):
    torch.matmul(x, wf.t())
torch.cuda.synchronize()
print("done")

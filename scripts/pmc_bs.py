"""Launch driver for counter runs of the shared-dequant-image GEMM (gemm_bs.hip): gate|up shape
(Q4_K, N = 28672, K = 4096, S = 1, bf16 out), variant 0 at M = 8192 and M = 256, and
q32 variant 9 at M = 256 for reference, 10 launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
K, N = 4096, 28672
w = rand_qweight(N, K, GGMLType.Q4_K, 1)
for M in (8192, 256):
    x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    for var in ([0, 2] if M > 256 else [0, 1]):
        for _ in range(10):
            ops._run_bs(x, [w], 1, out, N, var)
    if M == 256:
        for _ in range(10):
            ops._run_q32(x, [w], 1, out, N, 9)
torch.cuda.synchronize()
print("done")

"""Launch driver for counter runs of the round-3 decode hot kernels at batch 256 (Llama-3-8B
shapes): the fused gate|up GLU tile GEMM (tile 7, Q4_K, F = 14336, K = 4096) and the Q4_K down
projection tile GEMM (tile 7, S = 8, K = 14336), 20 warm launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
M, K, F = 256, 4096, 14336
gate, up = rand_qweight(F, K, GGMLType.Q4_K, 1), rand_qweight(F, K, GGMLType.Q4_K, 2)
x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
h = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
for _ in range(20):
    ops._run_glu(x, (gate, 0, up, 0), F, ops.ACT_SWIGLU, 7, h)
down = rand_qweight(K, F, GGMLType.Q4_K, 3)
xd = (torch.randn(M, F, device=DEV) * 0.5).to(torch.bfloat16)
out = torch.empty(8, M, K, dtype=torch.float32, device=DEV)
for _ in range(20):
    ops._run_tile(xd, [down], 8, out, K, 7)
torch.cuda.synchronize()
print("done")

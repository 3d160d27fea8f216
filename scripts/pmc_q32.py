"""Launch driver for counter runs of the 32x32x16 quantised GEMM (gemm_q32.hip) at decode batch
256 (Llama-3-8B gate|up shape, Q4_K, N = 28672, K = 4096): variant 6 (256 x 256, 4 waves, S = 1),
variant 9 (128 x 256, 8 waves, S = 1) and the round-3 tile kernel (tile 7) for reference, 20 warm
launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402
from scripts.q32_bench import q32  # noqa: E402

DEV = torch.device("cuda:0")
M, K, N = 256, 4096, 28672
w = rand_qweight(N, K, GGMLType.Q4_K, 1)
x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
out = torch.empty(1, M, N, dtype=torch.float32, device=DEV)
for var in (6, 9, 0):
    for _ in range(20):
        q32(x, w, 1, var, out=out)
for _ in range(20):
    ops._run_tile(x, [w], 1, out, N, 7)
torch.cuda.synchronize()
print("done")

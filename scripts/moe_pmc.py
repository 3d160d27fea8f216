"""Launch driver for counter runs of the grouped MoE GEMMs on Mixtral-8x7B gate|up (8 experts,
28672 x 4096 Q4_K) at T = 256 tokens, top-2: moe32 variant 4 (gemm_q32.hip moe32_kernel) and the
16-column kernel (moe.hip moe_gemm_kernel); 3 warm launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
E, T, topk, D, F = 8, 256, 2, 4096, 14336
mg = ops.MoEWeights([rand_qweight(2 * F, D, GGMLType.Q4_K, 1 + e) for e in range(E)])
g = torch.Generator(device=DEV).manual_seed(T)
x = (torch.randn(T, D, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
ids = torch.stack([torch.randperm(E, device=DEV, generator=g)[:topk] for _ in range(T)]).to(torch.int32)
order, off = ops.moe_route(ids, E)
for _ in range(3):
    ops.moe_glu32(x, mg, order, off, topk, T, var=4)
for _ in range(3):
    ops.moe_linear(x, mg, order, off, topk, T)
torch.cuda.synchronize()
print("done")

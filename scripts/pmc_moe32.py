"""Launch driver for counter runs of the grouped MoE decode GEMM (gemm_q32.hip moe32_kernel) at
Mixtral-8x7B decode shapes: T = 256 tokens, top-2 of 8 experts (balanced random routing, ~64 rows
per expert), gate|up of every expert (Q4_K, N = 2 x 14336, K = 4096) with the SwiGLU epilogue;
the round-6 default (variant 19: live row blocks, 128-row chunks, 64 columns per wave) and the
round-5 default (variant 4) for reference, 10 warm launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
T, E, topk, K, F = 256, 8, 2, 4096, 14336
mg = ops.MoEWeights([rand_qweight(2 * F, K, GGMLType.Q4_K, e) for e in range(E)])
x = (torch.randn(T, K, device=DEV) * 0.5).to(torch.bfloat16)
g = torch.Generator(device="cpu").manual_seed(0)
ids = torch.stack([torch.randperm(E, generator=g)[:topk] for _ in range(T)]).to(torch.int32).to(DEV)
order, off = ops.moe_route(ids, E)
for var in (19, 4):
    for _ in range(10):
        ops.moe_glu32(x, mg, order, off, topk, T, var=var)
torch.cuda.synchronize()
print("done")

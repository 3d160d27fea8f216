"""Launch driver for counter runs of the wide-batch grouped MoE GEMM (moe.hip moe_gemm_kernel) at
Mixtral-8x7B decode shapes: T = 256 tokens, top-2 of 8 experts (balanced random routing, ~64 rows
per expert), gate|up N = 28672, K = 4096, Q4_K; 64-row tiles in 8-wave workgroups (the default)
and, for reference, the round-3 128-row / 4-wave shape; 10 warm launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
T, E, topk, K, N = 256, 8, 2, 4096, 28672
mw = ops.MoEWeights([rand_qweight(N, K, GGMLType.Q4_K, e) for e in range(E)])
x = (torch.randn(T, K, device=DEV) * 0.5).to(torch.bfloat16)
ids = torch.stack([torch.randperm(E)[:topk] for _ in range(T)]).to(torch.int32).to(DEV)
order, off = ops.moe_route(ids, E)
for mt, nw in ((4, 8), (8, 4)):
    ops._check(ops.lib().la_moe_tune(mt, nw), "la_moe_tune")
    for _ in range(10):
        ops.moe_linear(x, mw, order, off, topk, T)
torch.cuda.synchronize()
print("done")

"""Runs only the skinny GEMM at decode shapes (for rocprofv3 --pmc counter collection)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from localai_amd import ops
from localai_amd.gguf import GGMLType, random_q4_k_blocks, random_q6_k_blocks
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
for name, N, K, t in (("gate_up", 28672, 4096, GGMLType.Q4_K), ("lm_head", 128256, 4096, GGMLType.Q6_K)):
    raw = (random_q4_k_blocks if t == GGMLType.Q4_K else random_q6_k_blocks)(rng, N * K // 256, 0.02)
    w = ops.QWeight.from_raw(raw, t, (N, K), dev)
    x = torch.randn(1, K, device=dev).to(torch.bfloat16)
    for _ in range(20):
        ops.linear(x, w, force="skinny")
    torch.cuda.synchronize()
print("done")

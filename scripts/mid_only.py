"""Runs only the mid-M quantised GEMM at M=256 decode shapes (for rocprofv3 --pmc runs)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from localai_amd import ops
from localai_amd.gguf import GGMLType, random_q4_k_blocks
dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
M = int(os.environ.get("MID_M", 256))
for name, N, K in (("gate_up", 28672, 4096), ("o", 4096, 4096)):
    w = ops.QWeight.from_raw(random_q4_k_blocks(rng, N * K // 256, 0.02), GGMLType.Q4_K, (N, K), dev)
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    for _ in range(10):
        ops.linear(x, w, force="mid")
    torch.cuda.synchronize()
print("done")

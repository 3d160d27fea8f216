"""Probe library GEMM choices for the mid-M (64..512) decode/prefill projections of Llama-3-8B:
torch.matmul on [N,K] weights (x @ w.t()), on pre-transposed [K,N] weights, and our skinny
quantised kernel.  Prints TFLOP/s and effective weight bandwidth."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType, random_q4_k_blocks  # noqa: E402

dev = torch.device("cuda:0")
SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336),
          ("lm_head", 128256, 4096)]
MS = [64, 128, 256, 512, 1024]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


out = []
for name, N, K in SHAPES:
    w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
    wt = w.t().contiguous()
    raw = random_q4_k_blocks(np.random.default_rng(0), N * K // 256, 0.02)
    qw = ops.QWeight.from_raw(raw, GGMLType.Q4_K, (N, K), dev)
    for M in MS:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        r = {"shape": name, "N": N, "K": K, "M": M}
        t = bench(lambda: torch.matmul(x, w.t()))
        r["nt_us"] = t * 1e6
        t2 = bench(lambda: torch.matmul(x, wt))
        r["nn_us"] = t2 * 1e6
        if M <= 64:
            t3 = bench(lambda: ops.linear(x, qw, force="skinny"))
            r["skinny_us"] = t3 * 1e6
        fl = 2.0 * M * N * K
        r["nt_tflops"] = fl / t / 1e12
        r["nn_tflops"] = fl / t2 / 1e12
        r["q4_floor_us"] = N * K * 0.5625 / 5e12 * 1e6
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        out.append(r)

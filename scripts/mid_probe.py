"""Probe the mid-M GEMM: activation row pitch (L2 channel camping), split-K, per-format."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from localai_amd import ops
from localai_amd.gguf import GGMLType, random_q4_k_blocks

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)


def timeit(fn, iters=20):
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
    return (time.perf_counter() - t0) / iters * 1e6


for name, N, K in (("qkv", 6144, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)):
    w = ops.QWeight.from_raw(random_q4_k_blocks(rng, N * K // 256, 0.02), GGMLType.Q4_K, (N, K), dev)
    for M in (128, 256):
        for pad in (0, 64, 128, 256):
            ldx = K + pad
            xb = torch.randn(M, ldx, device=dev).to(torch.bfloat16)
            for S in (1, 4):
                out = torch.empty(S, M, N, dtype=torch.float32, device=dev)
                us = timeit(lambda: ops.lib().la_qgemm_mid(w.fmt, *w.ptrs(), N, K, xb.data_ptr(), ldx, M, S,
                                                           out.data_ptr(), N, M * N, ops._stream()))
                print(f"{name:8s} M={M} ldx=K+{pad:3d} S={S} {us:8.2f} us {2*M*N*K/us/1e6:7.1f} TF/s", flush=True)

"""dp4 decode GEMV variants on the Llama-3-8B Q4_K_M decode shapes, cold weights, inside a
captured hipGraph (like the engine): variant bit 0 = non-temporal weight loads, bit 1 = weights
requested before the activation prologue.  Also times the fused q|k (Q4_K) + v (Q6_K) launch
against two separate launches."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType, random_q4_k_blocks, random_q6_k_blocks, random_q8_0_blocks

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters * 1e6)
    return best


BYTES_256 = {"q4k": 144, "q6k": 210, "q8": 272}


def mk(fmt, N, K):
    if fmt == "q8":
        return ops.QWeight.from_raw(random_q8_0_blocks(rng, N * K // 32, 0.02), GGMLType.Q8_0, (N, K), dev)
    if fmt == "q4k":
        return ops.QWeight.from_raw(random_q4_k_blocks(rng, N * K // 256, 0.02), GGMLType.Q4_K, (N, K), dev)
    return ops.QWeight.from_raw(random_q6_k_blocks(rng, N * K // 256, 0.02), GGMLType.Q6_K, (N, K), dev)


def copies(specs):
    """enough copies of the weight group that one rotation overflows L2 + the 256 MiB MALL"""
    one = sum(N * K // 256 * BYTES_256[f] for f, N, K in specs)
    n = max(2, min(48, -(-640 * 2**20 // one)))
    return [[mk(f, N, K) for f, N, K in specs] for _ in range(n)], one


SHAPES = [("qk", [("q4k", 5120, 4096)]), ("v", [("q6k", 1024, 4096)]), ("qkv", [("q4k", 5120, 4096), ("q6k", 1024, 4096)]),
          ("o", [("q4k", 4096, 4096)]), ("gate_up", [("q4k", 28672, 4096)]), ("down", [("q4k", 4096, 14336)]),
          ("down6", [("q6k", 4096, 14336)]), ("lm_head", [("q6k", 128256, 4096)])]
if os.environ.get("GEMV_SHAPES") == "q8":  # Llama-3-8B Q8_0
    SHAPES = [("qkv8", [("q8", 6144, 4096)]), ("o8", [("q8", 4096, 4096)]), ("gate_up8", [("q8", 28672, 4096)]),
              ("down8", [("q8", 4096, 14336)])]
variants = [int(v) for v in os.environ.get("GEMV_VARIANTS", "0,1,2,3").split(",")]
sweep_s = os.environ.get("GEMV_SWEEP_S") == "1"   # time every split-K factor (variant 1) instead
M = int(os.environ.get("GEMV_M", "1"))
for name, specs in SHAPES:
    groups, wbytes = copies(specs)
    K = specs[0][2]
    Ntot = sum(N for _, N, _ in specs)
    x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    S0 = ops._gemv_splits(groups[0], K, M)
    nsb = K // 256
    runs = [(int(os.environ.get("GEMV_SWEEP_VAR", "5")), S) for S in range(1, min(nsb, 32) + 1) if nsb % S == 0] if sweep_s else [(v, S0) for v in variants]
    for v, S in runs:
        out = torch.empty(S, M, Ntot, dtype=torch.float32, device=dev)
        assert ops.lib().la_gemv_variant(v) == 0
        cnt = [0]

        def fn():
            i = cnt[0]
            cnt[0] += 1
            ops.gemv_dp4(x, groups[i % len(groups)], S, out)
        us = timeit(fn, max(20, 2 * len(groups)))
        print(f"{name:8s} M={M} S={S:2d}{'*' if S == S0 else ' '} var={v} {us:8.2f} us  {wbytes / us / 1e6:5.2f} TB/s",
              flush=True)
ops.lib().la_gemv_variant(5)

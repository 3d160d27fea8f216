"""Per-shape map of the quantised GEMM paths on the Llama-3-8B decode shapes.

For each (shape, M) time every applicable path inside a captured hipGraph (20 back-to-back
launches, so launch overhead is the graph's, like the engine's decode graphs) and print
us / effective weight TB/s / TF/s.  Output: one line per (shape, M, path).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType, random_q4_k_blocks, random_q6_k_blocks

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
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters * 1e6)
    return best


def mk(fmt, N, K):
    if fmt == "q4k":
        return ops.QWeight.from_raw(random_q4_k_blocks(rng, N * K // 256, 0.02), GGMLType.Q4_K, (N, K), dev)
    return ops.QWeight.from_raw(random_q6_k_blocks(rng, N * K // 256, 0.02), GGMLType.Q6_K, (N, K), dev)


SHAPES = [("qk", "q4k", 5120, 4096), ("v", "q6k", 1024, 4096), ("o", "q4k", 4096, 4096),
          ("gate_up", "q4k", 28672, 4096), ("down", "q4k", 4096, 14336), ("down6", "q6k", 4096, 14336),
          ("lm_head", "q6k", 128256, 4096)]
Ms = [int(m) for m in os.environ.get("GEMM_MS", "1,4,16,64,128,256").split(",")]
only = os.environ.get("GEMM_SHAPES")
for name, fmt, N, K in SHAPES:
    if only and name not in only.split(","):
        continue
    # enough distinct copies that the rotation overflows the 256 MiB Infinity Cache: weights
    # arrive cold from HBM like in the engine (one pass over the model per decode step)
    w0 = mk(fmt, N, K)
    wbytes = N * K // 256 * (144 if fmt == "q4k" else 210)   # GGUF bytes (extra load-time planes not counted)
    ncopy = max(2, -(-640 * 2**20 // wbytes))
    ws = [w0] + [mk(fmt, N, K) for _ in range(ncopy - 1)] if ncopy <= 64 else [w0]
    wbf = [w.materialize_bf16() for w in ws[:max(2, -(-640 * 2**20 // (N * K * 2)))]]
    for M in Ms:
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        outs = {S: torch.empty(S, M, N, dtype=torch.float32, device=dev) for S in (1, 2, 4, 8)}
        paths = []
        if M <= ops.SKINNY_MAX_M:
            paths.append("skinny")
        if M <= ops.GEMV_MAX_M:
            paths.append("dp4")
        if M > 16:
            paths += ["blas"] + [f"mid:{t}:{S}" for t in ((42, 41, 22, 21) if M > 128 else (22, 21))
                                 for S in (1, 2, 4, 8) if ops._mid_split_ok(K, S)]
            if M > 128 and fmt == "q4k":
                paths += [f"ws:{S}" for S in (1, 2, 4, 8) if (K // 64) % S == 0]
        for p in paths:
            cnt = [0]

            def fn(p=p):
                i = cnt[0]
                cnt[0] += 1
                if p == "blas":
                    return torch.matmul(x, wbf[i % len(wbf)].t())
                if p.startswith("ws:"):
                    S = int(p.split(":")[1])
                    return ops._run_ws(x, [ws[i % len(ws)]], S, outs[S], N)
                if p.startswith("mid:"):
                    _, t, S = p.split(":")
                    return ops._run_mid(x, [ws[i % len(ws)]], int(S), outs[int(S)], N, int(t))
                return ops.linear(x, ws[i % len(ws)], force=p)
            try:
                us = timeit(fn, iters=max(20, 2 * len(ws)))
            except Exception as e:  # noqa: BLE001
                print(f"{name:8s} M={M:4d} {p:7s} ERR {e}", flush=True)
                continue
            wb = wbytes if p != "blas" else N * K * 2
            print(f"{name:8s} M={M:4d} {p:7s} {us:9.2f} us  {wb / us / 1e6:6.2f} TB/s  "
                  f"{2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)

"""rope_kv timing at the Llama-3-8B decode shape (T rows of q|k|v = 6144 bf16 from hipBLASLt, or
fp32 split-K slabs from the GEMV), with and without the paged-KV append, inside a hipGraph."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from localai_amd import ops

dev = torch.device("cuda:0")
Hq, Hkv, Dh, BS = 32, 8, 128, 32
W = (Hq + 2 * Hkv) * Dh
cs = ops.rope_cos_sin(4096, Dh, 500000.0, dev)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters * 1e6)
    return best


for T, S in [(1, 8), (256, 0)]:
    nblk = T * 8 + 8
    kc = torch.zeros(nblk, Hkv, BS, Dh, dtype=torch.bfloat16, device=dev)
    vc = ops.v_pages(nblk, Hkv, BS, Dh, device=dev)
    src = (torch.randn(T, W, device=dev).to(torch.bfloat16) if S == 0
           else torch.randn(S, T, W, device=dev))
    p = ops.Partial(src)
    pos = torch.randint(0, 2000, (T,), dtype=torch.int32, device=dev)
    slots = (torch.randperm(T, device=dev).to(torch.int32) * 8 * BS + 5)
    none = torch.full((T,), -1, dtype=torch.int32, device=dev)
    q = torch.empty(T, Hq, Dh, dtype=torch.bfloat16, device=dev)
    for name, sl in (("append", slots), ("no-append", none)):
        us = timeit(lambda: ops.rope_kv(p, pos, sl, cs, Hq, Hkv, Dh, Dh, 0, kc, vc, BS, q_out=q))
        print(f"rope_kv T={T:3d} S={S} {name:9s} {us:7.2f} us", flush=True)

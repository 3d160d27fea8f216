"""Decode attention timing at Llama-3-8B head shapes (Hq 32, Hkv 8, Dh 128, 32-key pages), inside
a captured hipGraph with the engine's graph bound (max_len 2048); prints us and KV TB/s."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from localai_amd import ops

dev = torch.device("cuda:0")
Hq, Hkv, Dh, BS = 32, 8, 128, 32
cases = [(1, 128), (1, 256), (1, 512), (2, 300), (1, 2000), (64, 512), (128, 384), (256, 256), (256, 384), (512, 300)]
runs = [(B, L, nw1) for B, L in cases for nw1 in ((False, True) if B * Hkv >= 512 else (False,))]
for B, L, nw1 in runs:
    ops.DEC_NW1_MIN = 1 if nw1 else 1 << 30
    nb = (L + BS - 1) // BS
    nblk = B * nb + 8
    # several "layers" of KV, cycled through, so the timed reads come from HBM (not the 256 MiB MALL)
    nl = max(1, min(8, (1 << 30) // (nblk * Hkv * BS * Dh * 4)))
    kcs = [(torch.randn(nblk, Hkv, BS, Dh, device=dev) * 0.5).to(torch.bfloat16) for _ in range(nl)]
    vcs = [ops.v_from_rows((torch.randn(nblk, Hkv, BS, Dh, device=dev) * 0.5).to(torch.bfloat16))
           for _ in range(nl)]
    bt = torch.randperm(B * nb, device=dev).to(torch.int32).view(B, nb)
    sl = torch.full((B,), L, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq, Dh, device=dev).to(torch.bfloat16)
    ws = ops.decode_workspace(B, Hq, Hkv, Dh, 2048, dev, BS)
    out = torch.empty(B, Hq, Dh, dtype=torch.bfloat16, device=dev)
    it = [0]

    def fn():
        i = it[0] % nl
        it[0] += 1
        ops.attn_decode(q, kcs[i], vcs[i], bt, sl, 0.088, 2048, out=out, workspace=ws)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    iters = 8 * nl if nl < 4 else 2 * nl * 4
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
    kv = B * L * Hkv * Dh * 2 * 2
    print(f"attn_decode B={B:3d} L={L:5d} waves/WG={ops.decode_waves(B, Hkv)} {best:8.2f} us  "
          f"{kv / best / 1e6:5.2f} TB/s", flush=True)

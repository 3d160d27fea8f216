"""Per-op microbenchmark on the GPU: time (us) and effective bandwidth of every hot kernel at
the Llama-3-8B decode shapes.  Usage: python scripts/microbench.py [--out file.json]"""
import json, math, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from localai_amd import ops
from localai_amd.gguf import GGMLType, random_q4_k_blocks, random_q6_k_blocks

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)


def qw(N, K, t=GGMLType.Q4_K):
    raw = random_q4_k_blocks(rng, N * K // 256, 0.02) if t == GGMLType.Q4_K else random_q6_k_blocks(rng, N * K // 256, 0.02)
    return ops.QWeight.from_raw(raw, t, (N, K), dev)


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
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


res = {}
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336), "lm_head": (128256, 4096)}
W = {k: qw(*v, GGMLType.Q6_K if k == "lm_head" else GGMLType.Q4_K) for k, v in shapes.items()}
for M in (1, 8, 16, 32, 64):
    for k, w in W.items():
        x = torch.randn(M, w.K, device=dev).to(torch.bfloat16)
        us = timeit(lambda: ops.linear(x, w, force="skinny"))
        gbs = w.nbytes / us / 1e3
        S = ops.pick_splits(w.N, w.K, M)
        res[f"skinny_{k}_M{M}"] = (round(us, 2), round(gbs, 1), S)
        print(f"skinny {k:8s} M={M:3d} S={S:2d} {us:8.2f} us  {gbs:7.1f} GB/s", flush=True)
for M in (96, 128, 256, 512):
    for k, w in W.items():
        x = torch.randn(M, w.K, device=dev).to(torch.bfloat16)
        S0 = ops.pick_mid_splits(w.N, w.K, M)
        best = None
        for S in sorted({1, 2, 3, 4, 6, 8, S0}):
            if -(-(w.K // 64) // S) * (S - 1) >= w.K // 64:
                continue
            out = torch.empty(S, M, w.N, dtype=torch.float32, device=dev)
            us = timeit(lambda: ops.lib().la_qgemm_mid(w.fmt, *w.ptrs(), w.N, w.K, x.data_ptr(), w.K, M, S,
                                                       out.data_ptr(), w.N, M * w.N, ops._stream()), iters=20)
            tf = 2 * M * w.N * w.K / us / 1e6
            res[f"mid_{k}_M{M}_S{S}"] = (round(us, 2), round(tf, 1))
            print(f"mid {k:8s} M={M:3d} S={S:2d}{'*' if S == S0 else ' '} {us:8.2f} us  {tf:7.1f} TF/s", flush=True)
    for k, w in W.items():
        x = torch.randn(M, w.K, device=dev).to(torch.bfloat16)
        wb = w.materialize_bf16()
        us = timeit(lambda: torch.matmul(x, wb.t()))
        tf = 2 * M * w.N * w.K / us / 1e6
        res[f"hipblaslt_{k}_M{M}"] = (round(us, 2), round(tf, 1))
        print(f"hipblaslt {k:8s} M={M:3d} {us:8.2f} us  {tf:7.1f} TF/s  {wb.numel()*2/us/1e3:7.1f} GB/s", flush=True)
if os.environ.get("MB_ONLY_GEMM"):
    sys.exit(0)
# attention decode
Hq, Hkv, Dh, BS = 32, 8, 128, 32
for B, L in ((1, 384), (1, 4096), (64, 384), (256, 384), (64, 2048)):
    nb = (L + BS - 1) // BS
    kc = torch.randn(B * nb + 1, Hkv, BS, Dh, device=dev).to(torch.bfloat16)
    vc = torch.randn(B * nb + 1, Hkv, Dh, BS, device=dev).to(torch.bfloat16)
    bt = torch.arange(B * nb, device=dev, dtype=torch.int32).view(B, nb)
    sl = torch.full((B,), L, dtype=torch.int32, device=dev)
    q = torch.randn(B, Hq, Dh, device=dev).to(torch.bfloat16)
    for ml in (L, 2048):
        us = timeit(lambda: ops.attn_decode(q, kc, vc, bt, sl, 0.088, max(ml, L)))
        by = B * L * Hkv * Dh * 2 * 2
        res[f"attn_decode_B{B}_L{L}_ml{ml}"] = (round(us, 2), round(by / us / 1e3, 1))
        print(f"attn_decode B={B:3d} L={L:5d} maxlen={max(ml,L):5d} {us:8.2f} us {by/us/1e3:7.1f} GB/s", flush=True)
# small fused kernels
for T in (1, 64, 256):
    D = 4096
    res_ = torch.randn(T, D, device=dev)
    add = torch.randn(2, T, D, device=dev)
    w = torch.ones(D, device=dev)
    us = timeit(lambda: ops.add_norm(res_, ops.Partial(add), w, None, 1e-5))
    res[f"add_norm_T{T}"] = round(us, 2)
    qkv = torch.randn(1, T, 6144, device=dev)
    pos = torch.arange(T, dtype=torch.int32, device=dev)
    slots = torch.arange(T, dtype=torch.int32, device=dev)
    kc = torch.zeros(T // 32 + 2, 8, 32, 128, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(T // 32 + 2, 8, 128, 32, device=dev, dtype=torch.bfloat16)
    cs = ops.rope_cos_sin(4096, 128, 5e5, dev)
    us2 = timeit(lambda: ops.rope_kv(ops.Partial(qkv), pos, slots, cs, 32, 8, 128, 128, 0, kc, vc, 32))
    gu = torch.randn(1, T, 28672, device=dev)
    us3 = timeit(lambda: ops.act(ops.Partial(gu), 14336, 0))
    lg = torch.randn(T, 128256, device=dev)
    p = np.zeros(T, dtype=ops.SAMPLE_ROW_DTYPE)
    us4 = timeit(lambda: ops.sample(lg, p), iters=20)
    p["temp"] = 0.8; p["top_k"] = 40; p["top_p"] = 0.95; p["min_p"] = 0.05
    us5 = timeit(lambda: ops.sample(lg, p), iters=20)
    res[f"rope_T{T}"], res[f"act_T{T}"], res[f"sample_greedy_T{T}"], res[f"sample_topk_T{T}"] = us2, us3, us4, us5
    print(f"T={T:3d} add_norm {us:7.2f} us  rope_kv {us2:7.2f} us  act {us3:7.2f} us  sample greedy {us4:7.2f} us topk {us5:7.2f} us", flush=True)
if "--out" in sys.argv:
    json.dump(res, open(sys.argv[sys.argv.index("--out") + 1], "w"), indent=1)

"""Tile GEMM (gemm_q.hip) vs hipBLASLt on a bf16 copy, Llama-3-8B Q4_K_M projection shapes.

Cold weights (L2 + Infinity Cache flushed by a 384 MiB read before every timed call), warm
activations, as in a decode step.  Prints a markdown table: best (tile, split) per shape with
its time and TFLOP/s, and the library time on the same shape.

  python scripts/gq_bench.py [--m 256] [--shapes qkv,o,gate_up,down,lm_head] [--abl]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402

DEV = torch.device("cuda:0")

SHAPES = {  # name: ([(N, type)], K)
    "qkv": ([(4096, GGMLType.Q4_K), (1024, GGMLType.Q4_K), (1024, GGMLType.Q6_K)], 4096),
    "o": ([(4096, GGMLType.Q4_K)], 4096),
    "gate_up": ([(28672, GGMLType.Q4_K)], 4096),
    "down": ([(4096, GGMLType.Q4_K)], 14336),
    "down6": ([(4096, GGMLType.Q6_K)], 14336),
    "lm_head": ([(128256, GGMLType.Q6_K)], 4096),
}


def rand_qweight(N, K, t, seed):
    """Random quantised planes made on the device (no host quantise): random bytes for the
    codes, sane scales.  Timing only."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    if t == GGMLType.Q4_K:
        raw = torch.randint(0, 256, (N, K // 256, 144), dtype=torch.uint8, device=DEV, generator=g)
        hdr = torch.tensor(np.array([0.01, 0.002], dtype=np.float16).view(np.uint8), device=DEV)
        raw[:, :, 0:4] = hdr
        raw[:, :, 4:16] &= 0x3F
    elif t == GGMLType.Q6_K:
        raw = torch.randint(0, 256, (N, K // 256, 210), dtype=torch.uint8, device=DEV, generator=g)
        raw[:, :, 192:208] &= 0x3F
        raw[:, :, 208:210] = torch.tensor(np.array([0.001], dtype=np.float16).view(np.uint8), device=DEV)
    else:
        raise ValueError(t)
    return ops.QWeight.from_raw(raw.cpu().numpy().reshape(-1), t, (N, K), DEV)


def timeit(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        ops._cold_caches(DEV)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,down6,lm_head")
    ap.add_argument("--blas", action="store_true", help="also time hipBLASLt on a bf16 copy")
    ap.add_argument("--abl", action="store_true", help="ablation builds on gate_up (Q4_K)")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = []
    print("| M | shape | N x K | best tile/S | us | TF/s | blas us | all candidates (tile,S:us) |", flush=True)
    print("|---|---|---|---|---:|---:|---:|---|", flush=True)
    for name in a.shapes.split(","):
        parts, K = SHAPES[name]
        ws = [rand_qweight(n, K, t, i) for i, (n, t) in enumerate(parts)]
        Ntot = sum(w.N for w in ws)
        for M in a.m:
            x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
            flops = 2.0 * M * Ntot * K
            res = {}
            tiles = (6, 1, 7, 8, 12) if M > 128 else (7, 12, 14, 3)
            if M > 256:
                tiles = (6, 16, 10)
            for t in tiles:
                g = ops._tile_grid(M, max(w.N for w in ws), t)
                base = max(1, round(256 / g))
                for S in sorted({1, max(1, base // 2), base, base * 2}):
                    if S > K // 256 or not ops._tile_split_ok(K, S):
                        continue
                    if M > 256 and S > 1:
                        continue
                    if M > 256:
                        out = torch.empty(M, Ntot, dtype=torch.bfloat16, device=DEV)
                    else:
                        out = torch.empty(S, M, Ntot, dtype=torch.float32, device=DEV)
                    res[(t, S)] = timeit(lambda: ops._run_tile(x, ws, S, out, Ntot, t))
            best = min(res, key=res.get)
            blas = ""
            if a.blas:
                for w in ws:
                    w.materialize_bf16()
                blas = "%.1f" % timeit(lambda: ops._run_blas(x, ws, Ntot))
                for w in ws:
                    w.bf16 = None
                torch.cuda.empty_cache()
            us = res[best]
            cands = " ".join("%d,%d:%.1f" % (k[0], k[1], v) for k, v in sorted(res.items()))
            print(f"| {M} | {name} | {Ntot}x{K} | {best[0]}/{best[1]} | {us:.1f} | {flops / us / 1e6:.0f} | {blas} | {cands} |",
                  flush=True)
            rows.append({"M": M, "shape": name, "N": Ntot, "K": K, "best": best, "us": us,
                         "tflops": flops / us / 1e6, "blas_us": blas, "cands": {f"{k[0]},{k[1]}": v for k, v in res.items()}})
    if a.abl:
        parts, K = SHAPES["gate_up"]
        w = rand_qweight(parts[0][0], K, parts[0][1], 0)
        p0, _, g = w.tile_planes()
        for M in a.m:
            x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
            for tile, S in ((16, 2), (10, 2), (11, 1)):
                out = torch.empty(S, M, w.N, dtype=torch.float32, device=DEV)
                line = []
                for abl in (0, 1, 2, 3, 4, 8, 12, 15, 32, 47, 64, 79, 111):
                    def fn(abl=abl):
                        if abl == 0:
                            ops._run_tile(x, [w], S, out, w.N, tile)
                        else:
                            rc = ops.lib().la_qgemm_tile_probe(p0, g, w.N, K, x.data_ptr(), M, S, out.data_ptr(), tile,
                                                               abl, ops._stream())
                            assert rc == 0, rc
                    line.append("abl%d=%.1f" % (abl, timeit(fn)))
                print(f"ablation gate_up M={M} tile={tile} S={S}: " + " ".join(line), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

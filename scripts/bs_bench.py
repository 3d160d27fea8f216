"""Shared-dequant-image GEMM (ops/csrc/gemm_bs.hip) against the current decode kernels
(gemm_q32.hip / gemm_q.hip, autotuned) and the prefill library path (dequant + hipBLASLt, and
hipBLASLt on a resident bf16 copy), on the Llama-3-8B Q4_K_M projection shapes.

Cold weights (L2 + Infinity Cache flushed before every timed call), as in a decode step.

  python scripts/bs_bench.py --m 256            # decode batch
  python scripts/bs_bench.py --m 2048 8192      # prefill chunks
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import SHAPES, rand_qweight, timeit  # noqa: E402

DEV = torch.device("cuda:0")


def splits_for(M, N, K, var):
    g = ops._bs_grid(M, N, var)
    base = max(1, round(256 / g))
    return [S for S in sorted({1, max(1, base // 2), base, base * 2, base * 3})
            if S <= K // 256 * 4 and ops._tile_split_ok(K, S) and S <= 16]


def decode(ms, shapes, q32=True):
    print("| M | shape | N x K | bs best var/S | us | TF/s | q32/tile best | us | bs candidates |", flush=True)
    print("|---|---|---|---|---:|---:|---|---:|---|", flush=True)
    for name in shapes:
        parts, K = SHAPES[name]
        ws = ops.fuse_runs([rand_qweight(n, K, t, i) for i, (n, t) in enumerate(parts)])
        Ntot = sum(w.N for w in ws)
        N = max(w.N for w in ws)
        for M in ms:
            x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
            flops = 2.0 * M * Ntot * K
            res = {}
            for var in ops.BS_TILES:
                for S in splits_for(M, N, K, var):
                    out = (torch.empty(M, Ntot, dtype=torch.bfloat16, device=DEV) if S == 1 else
                           torch.empty(S, M, Ntot, dtype=torch.float32, device=DEV))
                    t = timeit(lambda: ops._run_bs(x, ws, S, out, Ntot, var))
                    # slab traffic the consumer pays (as the autotuner charges it)
                    if S > 1:
                        t += 2 * (S * M * Ntot * 4 - M * Ntot * 2) / 4e6
                    res[(var, S)] = t
            best = min(res, key=res.get)
            ob, ot = "-", float("nan")
            if q32:
                key = ((M + 31) // 32 * 32, K, tuple((w.fmt, w.N) for w in ws))
                ops._GEMM_CHOICE.pop(key, None)
                saved = ops.BS
                ops.BS = False
                ch = ops._autotune_mid(x, ws, key, Ntot)
                ops.BS = saved
                kind, S, t = ch
                out = (torch.empty(M, Ntot, dtype=torch.bfloat16, device=DEV) if S <= 1 else
                       torch.empty(S, M, Ntot, dtype=torch.float32, device=DEV))
                if kind == "q32":
                    ot = timeit(lambda: ops._run_q32(x, ws, S, out, Ntot, t))
                elif kind == "tile":
                    ot = timeit(lambda: ops._run_tile(x, ws, S, out, Ntot, t))
                if S > 1:
                    ot += 2 * (S * M * Ntot * 4 - M * Ntot * 2) / 4e6
                ob = f"{kind}{t}/{S}"
            cands = " ".join("%d,%d:%.1f" % (k[0], k[1], v) for k, v in sorted(res.items()))
            print(f"| {M} | {name} | {Ntot}x{K} | {best[0]}/{best[1]} | {res[best]:.1f} | "
                  f"{flops / res[best] / 1e6:.0f} | {ob} | {ot:.1f} | {cands} |", flush=True)
    # fused GLU gate|up (one [2F, K] Q4_K weight)
    F, K = 14336, 4096
    w = rand_qweight(2 * F, K, GGMLType.Q4_K, 0)
    pair = (w, 0, w, F)
    for M in ms:
        x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
        out = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
        flops = 2.0 * M * 2 * F * K
        line = []
        for var in ops.BS_TILES:
            t = timeit(lambda: ops._run_bs_glu(x, pair, F, 0, var, out))
            line.append("bs%d %.1f (%.0f TF/s)" % (var, t, flops / t / 1e6))
        if q32:
            for v in (9, 8):
                line.append("q32_%d %.1f" % (v, timeit(lambda: ops._run_glu(x, pair, F, 0, 100 + v, out))))
        print(f"glu M={M}: " + ", ".join(line), flush=True)


def prefill(ms, shapes):
    print("| M | shape | N x K | bs var: us | best TF/s | dequant+blas us | blas on bf16 copy us |", flush=True)
    print("|---|---|---|---|---:|---:|---:|", flush=True)
    for name in shapes:
        parts, K = SHAPES[name]
        ws = ops.fuse_runs([rand_qweight(n, K, t, i) for i, (n, t) in enumerate(parts)])
        Ntot = sum(w.N for w in ws)
        for M in ms:
            x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
            flops = 2.0 * M * Ntot * K
            out = torch.empty(M, Ntot, dtype=torch.bfloat16, device=DEV)
            res = {var: timeit(lambda: ops._run_bs(x, ws, 1, out, Ntot, var)) for var in ops.BS_TILES}
            tb = timeit(lambda: ops._run_scratch_blas(x, ws, Ntot))
            cp = torch.cat([w.materialize_bf16() for w in ws], 0)
            tc = timeit(lambda: torch.matmul(x, cp.t()))
            for w in ws:
                w.bf16 = None
            del cp
            best = min(res.values())
            cells = " ".join("%d:%.0f" % (k, v) for k, v in res.items())
            print(f"| {M} | {name} | {Ntot}x{K} | {cells} | {flops / best / 1e6:.0f} | {tb:.0f} | {tc:.0f} |",
                  flush=True)
    F, K = 14336, 4096
    w = rand_qweight(2 * F, K, GGMLType.Q4_K, 0)
    pair = (w, 0, w, F)
    for M in ms:
        x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
        out = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
        flops = 2.0 * M * 2 * F * K
        line = []
        for var in ops.BS_TILES:
            t = timeit(lambda: ops._run_bs_glu(x, pair, F, 0, var, out))
            line.append("bs%d %.0f (%.0f TF/s)" % (var, t, flops / t / 1e6))
        print(f"glu M={M}: " + ", ".join(line), flush=True)


def ablate(ms):
    """la_bsgemm_probe (Q4_K, variant 0, S = 1) on gate_up (N = 28672, K = 4096): bits 1 no MFMA,
    2 no dequant, 4 no X loads, 8 no W loads, 16 no barrier, 32 no X image writes, 64 no B
    fragment reads, 128 no A fragment reads."""
    import ctypes
    L = ops.lib()
    L.la_bsgemm_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    K, N = 4096, 28672
    w = rand_qweight(N, K, GGMLType.Q4_K, 0)
    p0, _, g = w.tile_planes()
    for M in ms:
        xp = (torch.randn(M, K + 64, device=DEV) * 0.5).to(torch.bfloat16)
        xb = xp[:, :K].contiguous().view(M // 32, 32, K // 8, 8).permute(0, 2, 1, 3).contiguous()
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        line = []
        ref = None
        # codes repacked [N/32][K/64][32][32 B] for the 16384 probes
        qb = w.planes[0].view(N // 32, 32, K // 64, 32).permute(0, 2, 1, 3).contiguous()
        for abl, ldx in ((0, K + 64), (512, K + 64), (8192, 0), (8704, 0), (24576, 0), (25088, 0), (24580, 0), (8196, 0),
                         (8200, 0), (8208, 0), (254, K + 64)):
            src = xb if abl & 8192 else xp
            def fn(abl=abl, ldx=ldx, src=src):
                rc = L.la_bsgemm_probe(abl, qb.data_ptr() if abl & 16384 else p0, g, N, K, src.data_ptr(), ldx, M,
                                       out.data_ptr(), ops._stream())
                assert rc == 0, rc
            tt = timeit(fn)
            if abl in (0, 256, 512, 8192, 8448, 8704, 24576, 25088):
                fn()
                torch.cuda.synchronize()
                if ref is None:
                    ref = out.float().clone()
                err = (out.float() - ref).abs().max().item()
                line.append("abl%d %.0f (diff %.2g)" % (abl, tt, err))
            else:
                line.append("abl%d %.0f" % (abl, tt))
        print(f"ablate M={M}: " + ", ".join(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,down6,lm_head")
    ap.add_argument("--no-q32", action="store_true")
    ap.add_argument("--abl", action="store_true")
    a = ap.parse_args()
    if a.abl:
        ablate(a.m)
        return
    shapes = a.shapes.split(",")
    dec = [m for m in a.m if m <= 256]
    pre = [m for m in a.m if m > 256]
    if dec:
        decode(dec, shapes, not a.no_q32)
    if pre:
        prefill(pre, shapes)


if __name__ == "__main__":
    main()

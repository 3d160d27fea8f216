"""Prefill-size (M = 2048..8192) GEMMs on the Llama-3-8B Q4_K_M projection shapes: the current
serving path (dequantise into scratch + hipBLASLt, ops._run_scratch_blas) against the hand-written
quantised kernels (gemm_q32.hip variants, gemm_q.hip tiles) with a bf16 output.  Warm timing (a
prefill chunk re-reads each weight tile from L2 for every row block).

  python scripts/prefill_gemm_bench.py [--m 8192] [--shapes qkv,o,gate_up,down,down6] [--check]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from scripts.gq_bench import SHAPES, rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")


def timeit(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[8192])
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,down6")
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    print("| M | shape | N x K | blas (dequant+GEMM) us | TF/s | best hand-written | us | TF/s | all (kind var:us) |",
          flush=True)
    print("|---|---|---|---:|---:|---|---:|---:|---|", flush=True)
    for name in a.shapes.split(","):
        parts, K = SHAPES[name]
        ws = ops.fuse_runs([rand_qweight(n, K, t, i) for i, (n, t) in enumerate(parts)])
        Ntot = sum(w.N for w in ws)
        for M in a.m:
            x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
            flops = 2.0 * M * Ntot * K
            t_blas = timeit(lambda: ops._run_scratch_blas(x, ws, Ntot))
            ref = ops._run_scratch_blas(x, ws, Ntot).float() if a.check else None
            out = torch.empty(M, Ntot, dtype=torch.bfloat16, device=DEV)
            res = {}
            for v in (2, 6, 0, 4, 1, 5, 8, 9):
                if not ops.q32_ok(ws, v) or len(ws) > 2:
                    continue
                if len(ws) == 2 and (ws[0].fmt, ws[1].fmt) not in ops._TILE2_PAIRS:
                    continue
                try:
                    res[("q32", v)] = timeit(lambda v=v: ops._run_q32(x, ws, 1, out, Ntot, v))
                except RuntimeError:
                    continue
                if ref is not None:
                    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
                    print(f"check {name} M={M} q32 var{v}: rel {err:.2e}", flush=True)
            if all(w.tile_ok for w in ws):
                for t in (6, 0, 1, 7, 16, 10):
                    try:
                        res[("tile", t)] = timeit(lambda t=t: ops._run_tile(x, ws, 1, out, Ntot, t))
                    except RuntimeError:
                        continue
            if res:
                best = min(res, key=res.get)
                cands = " ".join("%s%d:%.0f" % (k[0], k[1], v) for k, v in sorted(res.items()))
                print(f"| {M} | {name} | {Ntot}x{K} | {t_blas:.0f} | {flops / t_blas / 1e6:.0f} | {best[0]} {best[1]} | "
                      f"{res[best]:.0f} | {flops / res[best] / 1e6:.0f} | {cands} |", flush=True)
            else:
                print(f"| {M} | {name} | {Ntot}x{K} | {t_blas:.0f} | {flops / t_blas / 1e6:.0f} | - | - | - | |",
                      flush=True)


if __name__ == "__main__":
    main()

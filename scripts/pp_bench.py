"""Prefill GEMM (gemm_pp.hip) against the dequant + hipBLASLt path it replaces
(ops._run_scratch_blas: Q4_K/Q6_K dequantised into a bf16 scratch, then torch.matmul), on the
Llama-3-8B Q4_K_M projection shapes at prefill chunk sizes.  Both timed warm (median of 7),
the library path INCLUDING its dequant pass.  --check compares every output against the fp32
product of the same bf16-rounded weights.

  python scripts/pp_bench.py [--m 2048 8192] [--shapes qkv,o,gate_up,down,down6] [--check] [--glu]
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


def wbf16(ws):
    Ntot, K = sum(w.N for w in ws), ws[0].K
    wt = torch.empty(Ntot, K, dtype=torch.bfloat16, device=DEV)
    row = 0
    for w in ws:
        ops._check(ops.lib().la_dequant(w.fmt, *w.ptrs(), w.N, w.K, wt[row:row + w.N].data_ptr(), ops._stream()),
                   "la_dequant")
        row += w.N
    return wt


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item(), \
        ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[2048, 8192])
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,down6")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--glu", action="store_true", help="also the fused gate|up + SwiGLU launch")
    ap.add_argument("--splits", type=int, default=0, help="force split-K (0: pp_splits heuristic)")
    a = ap.parse_args()
    print("| M | shape | N x K | blas (dequant+GEMM) us | TF/s | pp S | pp us | TF/s | pp / blas |", flush=True)
    print("|---|---|---|---:|---:|---:|---:|---:|---:|", flush=True)
    for name in a.shapes.split(","):
        parts, K = SHAPES[name]
        ws = ops.fuse_runs([rand_qweight(n, K, t, i) for i, (n, t) in enumerate(parts)])
        Ntot = sum(w.N for w in ws)
        wt = wbf16(ws) if a.check else None
        for M in a.m:
            x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
            flops = 2.0 * M * Ntot * K
            S = a.splits or ops.pp_splits(M, Ntot, K)
            assert ops.pp_ok(ws, K, S), (name, S)
            t_blas = timeit(lambda: ops._run_scratch_blas(x, ws, Ntot))
            if S == 1:
                out = torch.empty(M, Ntot, dtype=torch.bfloat16, device=DEV)
            else:
                out = torch.empty(S, M, Ntot, dtype=torch.float32, device=DEV)
            t_pp = timeit(lambda: ops._run_pp(x, ws, S, out, Ntot))
            print(f"| {M} | {name} | {Ntot}x{K} | {t_blas:.0f} | {flops / t_blas / 1e6:.0f} | {S} | {t_pp:.0f} | "
                  f"{flops / t_pp / 1e6:.0f} | {t_pp / t_blas:.2f} |", flush=True)
            if a.check:
                ref = x.float() @ wt.float().t()
                got = out if S == 1 else out.sum(0)
                r2, rm = rel(got, ref)
                rb2, rbm = rel(ops._run_scratch_blas(x, ws, Ntot), ref)
                print(f"check {name} M={M} S={S}: pp rel-L2 {r2:.2e} max {rm:.2e} | blas rel-L2 {rb2:.2e} max {rbm:.2e}",
                      flush=True)
                assert r2 < 1e-2 and rm < 5e-2, "pp mismatch"
        if a.glu and name == "gate_up":
            F = Ntot // 2
            pair = (ws[0], 0, ws[0], F)
            for M in a.m:
                x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
                h = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
                t_glu = timeit(lambda: ops._run_pp_glu(x, pair, F, 0, h))

                def unfused():
                    y = ops._run_scratch_blas(x, ws, Ntot)
                    return torch.nn.functional.silu(y[:, :F].float()) * y[:, F:].float()
                t_ref = timeit(unfused)
                print(f"glu M={M}: pp fused {t_glu:.0f} us ({2.0 * M * Ntot * K / t_glu / 1e6:.0f} TF/s) vs "
                      f"blas+act {t_ref:.0f} us", flush=True)
                if a.check:
                    y = x.float() @ wt.float().t()
                    ref = torch.nn.functional.silu(y[:, :F]) * y[:, F:]
                    r2, rm = rel(h, ref)
                    print(f"check glu M={M}: rel-L2 {r2:.2e} max {rm:.2e}", flush=True)
                    assert r2 < 1e-2, "glu mismatch"


if __name__ == "__main__":
    main()

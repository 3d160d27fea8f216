"""32x32x16 quantised GEMM (ops/csrc/gemm_q32.hip): numerics against fp32, then timing against
the 16x16x32 tile kernel (gemm_q.hip) on the Llama-3-8B Q4_K_M projection shapes.

Cold weights (L2 + Infinity Cache flushed before every timed call, as in a decode step).

  python scripts/q32_bench.py [--m 256] [--shapes qkv,o,gate_up,down,down6,lm_head] [--check]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType, quantize  # noqa: E402
from scripts.gq_bench import SHAPES, rand_qweight, timeit  # noqa: E402

DEV = torch.device("cuda:0")
VARS = {0: (256, 128), 1: (128, 256), 2: (256, 256), 3: (128, 128), 4: (256, 128), 5: (128, 256), 6: (256, 256),
        7: (128, 128), 8: (128, 256), 9: (128, 256)}


def q32(x, w, S, var, bf16=False, out=None):
    M, K = x.shape
    p0, p1, g = w.tile_planes()
    if out is None:
        out = torch.empty((M, w.N) if bf16 else (S, M, w.N), dtype=torch.bfloat16 if bf16 else torch.float32,
                          device=DEV)
    rc = ops.lib().la_qgemm32(w.fmt, p0, p1, g, w.N, K, x.data_ptr(), K, M, S, out.data_ptr(), w.N,
                              0 if bf16 else M * w.N, int(bf16), var, ops._stream())
    assert rc == 0, rc
    return out


def q32_pair(x, wa, wb, S, var, out):
    M, K = x.shape
    a0, a1, ag = wa.tile_planes()
    b0, b1, bg = wb.tile_planes()
    N = wa.N + wb.N
    rc = ops.lib().la_qgemm32_2(wa.fmt, a0, a1, ag, wa.N, wb.fmt, b0, b1, bg, wb.N, K, x.data_ptr(), K, M, S,
                                out.data_ptr(), N, M * N, 0, var, ops._stream())
    assert rc == 0, rc


def q32_glu(x, w, F, var, out, act=0):
    M, K = x.shape
    p0, p1, g = w.tile_planes()
    rc = ops.lib().la_qgemm32_glu(w.fmt, p0, p1, g, 0, p0, p1, g, F, F, K, x.data_ptr(), K, M, out.data_ptr(), F,
                                  act, var, ops._stream())
    assert rc == 0, rc


def _qw(N, K, t, seed=0, std=0.05):
    rng = np.random.default_rng(seed)
    w = rng.standard_normal((N, K)).astype(np.float32) * std
    return ops.QWeight.from_raw(quantize(w, t), t, (N, K), DEV, keep_ref=True)


def check():
    torch.manual_seed(0)
    bad = 0
    for t in (GGMLType.Q4_K, GGMLType.Q6_K, GGMLType.Q8_0):
        for (N, K, M) in ((200, 1536, 150), (384, 2048, 256), (96, 512, 70)):
            w = _qw(N, K, t, seed=N + K)
            x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
            ref = x.float().cpu() @ w.ref.t()
            for var in VARS:
                if var in (2, 6) and t != GGMLType.Q4_K:
                    continue
                for S in (1, 3):
                    if S > K // 64:
                        continue
                    y = q32(x, w, S, var).sum(0).cpu()
                    err = (y - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                    ok = torch.isfinite(y).all().item() and err < 2e-2
                    bad += not ok
                    print(f"check fmt={int(t)} N={N} K={K} M={M} var={var} S={S}: rel {err:.2e} {'ok' if ok else 'FAIL'}",
                          flush=True)
                yb = q32(x, w, 1, var, bf16=True).float().cpu()
                err = (yb - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                ok = err < 2e-2
                bad += not ok
                print(f"check fmt={int(t)} bf16 var={var}: rel {err:.2e} {'ok' if ok else 'FAIL'}", flush=True)
    # GLU on one [2F, K] weight, pair Q4_K + Q6_K
    F, K, M = 320, 1024, 200
    w = _qw(2 * F, K, GGMLType.Q4_K, seed=7)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    g = x.float().cpu() @ w.ref[:F].t()
    u = x.float().cpu() @ w.ref[F:].t()
    ref = torch.nn.functional.silu(g) * u
    for var in VARS:
        out = torch.full((M, F), float("nan"), dtype=torch.bfloat16, device=DEV)
        q32_glu(x, w, F, var, out)
        y = out.float().cpu()
        err = (y - ref).abs().max().item() / max(1.0, ref.abs().max().item())
        ok = torch.isfinite(y).all().item() and err < 2e-2
        bad += not ok
        print(f"check glu var={var}: rel {err:.2e} {'ok' if ok else 'FAIL'}", flush=True)
    wa = _qw(300, K, GGMLType.Q4_K, seed=8)
    wb = _qw(100, K, GGMLType.Q6_K, seed=9)
    ref = x.float().cpu() @ torch.cat([wa.ref, wb.ref]).t()
    for var in VARS:
        if var in (2, 6):
            continue
        for S in (1, 2):
            out = torch.full((S, M, 400), float("nan"), dtype=torch.float32, device=DEV)
            q32_pair(x, wa, wb, S, var, out)
            y = out.sum(0).cpu()
            err = (y - ref).abs().max().item() / max(1.0, ref.abs().max().item())
            ok = torch.isfinite(y).all().item() and err < 2e-2
            bad += not ok
            print(f"check pair var={var} S={S}: rel {err:.2e} {'ok' if ok else 'FAIL'}", flush=True)
    print(f"CHECK {'PASS' if bad == 0 else 'FAIL %d' % bad}", flush=True)
    return bad == 0


def bench(ms, shapes):
    print("| M | shape | N x K | q32 best var/S | us | TF/s | tile best | us | all q32 (var,S:us) |", flush=True)
    print("|---|---|---|---|---:|---:|---|---:|---|", flush=True)
    for name in shapes:
        parts, K = SHAPES[name]
        ws = ops.fuse_runs([rand_qweight(n, K, t, i) for i, (n, t) in enumerate(parts)])
        Ntot = sum(w.N for w in ws)
        for M in ms:
            x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
            flops = 2.0 * M * Ntot * K
            res = {}
            for var, (bm, bn) in VARS.items():
                tiles = -(-M // bm) * -(-max(w.N for w in ws) // bn)
                base = max(1, round(256 / tiles))
                for S in sorted({1, max(1, base // 2), base, base * 2}):
                    if S > K // 256 or not ops._tile_split_ok(K, S):
                        continue
                    out = torch.empty(S, M, Ntot, dtype=torch.float32, device=DEV)
                    if len(ws) == 2:
                        fn = lambda: q32_pair(x, ws[0], ws[1], S, var, out)  # noqa: E731
                    elif len(ws) == 1:
                        fn = lambda: q32(x, ws[0], S, var, out=out)  # noqa: E731
                    else:
                        continue
                    try:
                        fn()
                    except AssertionError:
                        continue  # variant not built for this format pair
                    res[(var, S)] = timeit(fn)
            old = {}
            tiles_old = (6, 1, 7, 8, 12) if M > 128 else (7, 12, 14, 3)
            for t in tiles_old:
                g = ops._tile_grid(M, max(w.N for w in ws), t)
                base = max(1, round(256 / g))
                for S in sorted({1, max(1, base // 2), base, base * 2}):
                    if S > K // 256 or not ops._tile_split_ok(K, S):
                        continue
                    out = torch.empty(S, M, Ntot, dtype=torch.float32, device=DEV)
                    old[(t, S)] = timeit(lambda: ops._run_tile(x, ws, S, out, Ntot, t))
            ob = min(old, key=old.get)
            if res:
                best = min(res, key=res.get)
                us = res[best]
                cands = " ".join("%d,%d:%.1f" % (k[0], k[1], v) for k, v in sorted(res.items()))
                print(f"| {M} | {name} | {Ntot}x{K} | {best[0]}/{best[1]} | {us:.1f} | {flops / us / 1e6:.0f} | "
                      f"{ob[0]}/{ob[1]} | {old[ob]:.1f} | {cands} |", flush=True)
    # fused GLU gate|up (one [2F, K] Q4_K weight)
    F, K = 14336, 4096
    w = rand_qweight(2 * F, K, GGMLType.Q4_K, 0)
    for M in ms:
        x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
        out = torch.empty(M, F, dtype=torch.bfloat16, device=DEV)
        line = []
        for var in VARS:
            line.append("q32 var%d %.1f" % (var, timeit(lambda: q32_glu(x, w, F, var, out))))
        if 2 in VARS:
            # gate|up as one plain GEMM with split-K 2 on the 256 x 256 tile (no GLU epilogue)
            o2 = torch.empty(2, M, 2 * F, dtype=torch.float32, device=DEV)
            for var in (2, 6):
                line.append("plain var%d S2 %.1f" % (var, timeit(lambda: q32(x, w, 2, var, out=o2))))
        pair = (w, 0, w, F)
        for t in ((6, 7, 8) if M > 128 else (7, 12, 14)):
            line.append("tile%d %.1f" % (t, timeit(lambda: ops._run_glu(x, pair, F, 0, t, out))))
        print(f"glu M={M}: " + ", ".join(line), flush=True)


def ablate(ms):
    """Ablation builds of variants 0, 4, 8 on gate_up (Q4_K, N = 28672, K = 4096, S = 1): bits
    1 no MFMA, 2 no dequant, 4 no DMA, 8 no A LDS reads, 16 no mid-step barrier."""
    K, N = 4096, 28672
    w = rand_qweight(N, K, GGMLType.Q4_K, 0)
    p0, _, g = w.tile_planes()
    for M in ms:
        x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
        out = torch.empty(1, M, N, dtype=torch.float32, device=DEV)
        for var in (0, 4, 8):
            line = ["full %.1f" % timeit(lambda: q32(x, w, 1, var, out=out))]
            for abl in (1, 2, 3, 4, 8, 12, 15, 16, 20, 31):
                def fn(abl=abl):
                    rc = ops.lib().la_qgemm32_probe(var, abl, p0, g, N, K, x.data_ptr(), M, 1, out.data_ptr(),
                                                    ops._stream())
                    assert rc == 0, rc
                line.append("abl%d %.1f" % (abl, timeit(fn)))
            print(f"ablation gate_up M={M} var={var}: " + ", ".join(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256])
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,down6,lm_head")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--no-bench", action="store_true")
    ap.add_argument("--vars", default="")
    ap.add_argument("--abl", action="store_true")
    a = ap.parse_args()
    if a.vars:
        for k in list(VARS):
            if str(k) not in a.vars.split(","):
                del VARS[k]
    if a.check and not check():
        sys.exit(1)
    if a.abl:
        ablate(a.m)
    if not a.no_bench:
        bench(a.m, a.shapes.split(","))


if __name__ == "__main__":
    main()

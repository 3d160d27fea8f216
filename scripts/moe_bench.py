"""Mixtral-8x7B-shaped MoE layer on the GPU: the 16-column grouped GEMM (moe.hip, moe_linear +
act + moe_linear down) vs the 32x32x16 grouped tiles (gemm_q32.hip moe32, moe_glu32 +
moe_down32), per variant, cold caches (each decode step streams every expert once).

  python scripts/moe_bench.py [--T 64 128 256] [--vars 0 1 2 3 4 5 6] [--down-fmt q4k|q6k]
  python scripts/moe_bench.py --prefill [--T 1024 4096]   # prefill chunks: grouped bs tile
      (gemm_bs.hip bsmoe_kernel, every variant) vs the dense per-expert path (one host read of the
      grouping, dequant + hipBLASLt per expert) vs moe32"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight, timeit  # noqa: E402

DEV = torch.device("cuda:0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[64, 128, 256])
    ap.add_argument("--vars", type=int, nargs="+", default=sorted(ops.MOE32_TILES))
    ap.add_argument("--down-fmt", default="q4k")
    ap.add_argument("--E", type=int, default=8)
    ap.add_argument("--abl", action="store_true", help="ablation probes of the gate|up kernel (variant 4)")
    ap.add_argument("--prefill", action="store_true", help="prefill chunks: bs grouped vs dense per expert")
    a = ap.parse_args()
    E, topk, D, F = a.E, 2, 4096, 14336
    td = GGMLType.Q6_K if a.down_fmt == "q6k" else GGMLType.Q4_K
    mg = ops.MoEWeights([rand_qweight(2 * F, D, GGMLType.Q4_K, 1 + e) for e in range(E)])
    md = ops.MoEWeights([rand_qweight(D, F, td, 100 + e) for e in range(E)])
    print(f"E={E} D={D} F={F} down={a.down_fmt} gate|up bytes/expert ~{2 * F * D * 0.5625 / 1e6:.0f} MB", flush=True)
    if a.prefill:
        return prefill(a, mg, md, E, topk, D, F)
    for T in a.T:
        g = torch.Generator(device=DEV).manual_seed(T)
        x = (torch.randn(T, D, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
        ids = torch.stack([torch.randperm(E, device=DEV, generator=g)[:topk] for _ in range(T)]).to(torch.int32)
        wts = torch.rand(T * topk, device=DEV, generator=g)
        order, off = ops.moe_route(ids, E)
        gu_old = lambda: ops.moe_linear(x, mg, order, off, topk, T)  # noqa: E731
        gu = gu_old()
        h_old = ops.act(gu, F, ops.ACT_SWIGLU)
        t_gu = timeit(gu_old)
        t_act = timeit(lambda: ops.act(gu, F, ops.ACT_SWIGLU))
        t_dn = timeit(lambda: ops.moe_linear(h_old, md, order, off, topk, T, down=True, wts=wts))
        ref = ops.moe_linear(h_old, md, order, off, topk, T, down=True, wts=wts).dense().float()
        print(f"T={T} old: gate|up {t_gu:.1f} us + act {t_act:.1f} + down {t_dn:.1f} = {t_gu + t_act + t_dn:.1f} us",
              flush=True)
        if a.abl:
            F_ = mg.N // 2
            h = torch.empty(T * topk, F_, dtype=torch.bfloat16, device=DEV)
            base = timeit(lambda: ops.moe_glu32(x, mg, order, off, topk, T, var=4))
            res = [f"base {base:.1f}"]
            for ab in (1, 2, 3, 4, 8, 11, 16):
                def fn(ab=ab):
                    rc = ops.lib().la_moe32_probe(ab, mg.desc32().data_ptr(), F_, mg.K, mg.E, order.data_ptr(),
                                                  off.data_ptr(), topk, x.data_ptr(), x.shape[1], T, h.data_ptr(),
                                                  F_, ops._stream())
                    assert rc == 0, rc
                res.append(f"abl{ab} {timeit(fn):.1f}")
            print(f"T={T} gate|up var 4 ablations (us): " + "  ".join(res), flush=True)
            continue
        for v in a.vars:
            h = ops.moe_glu32(x, mg, order, off, topk, T, var=v)
            d = ops.moe_down32(h, md, order, off, topk, T, wts, var=v).dense().float()
            rel = ((d - ref).norm() / ref.norm()).item()
            t1 = timeit(lambda: ops.moe_glu32(x, mg, order, off, topk, T, var=v))
            t2 = timeit(lambda: ops.moe_down32(h, md, order, off, topk, T, wts, var=v))
            gbs = E * 2 * F * D * 0.625 / t1 / 1e6
            print(f"T={T} moe32 var {v}: glu {t1:.1f} us ({gbs:.2f} TB/s codes+scales) + down {t2:.1f} "
                  f"(S={ops._moe32_splits(md, T, topk, v)}) = {t1 + t2:.1f} us  rel-L2 vs old {rel:.2e}", flush=True)


def prefill(a, mg, md, E, topk, D, F):
    for T in a.T:
        g = torch.Generator(device=DEV).manual_seed(T)
        x = (torch.randn(T, D, device=DEV, generator=g) * 0.5).to(torch.bfloat16)
        # Mixtral-like skew: expert popularity varies 3:1
        pop = torch.linspace(1.0, 3.0, E, device=DEV)
        ids = torch.stack([torch.multinomial(pop, topk, generator=g) for _ in range(T)]).to(torch.int32)
        wts = torch.rand(T * topk, device=DEV, generator=g)
        flops = 2.0 * T * topk * 3 * F * D

        def dense():
            order, off = ops.moe_route(ids, E)
            off_h = off.cpu().tolist()
            order_l = order.long()
            tok = order_l // topk
            xs = x.index_select(0, tok)
            wsel = wts.index_select(0, order_l)
            out = torch.zeros(T, D, dtype=torch.float32, device=DEV)
            with ops.blas_tuning_paused():
                for e in range(E):
                    r0, r1 = off_h[e], off_h[e + 1]
                    if r1 <= r0:
                        continue
                    gu = ops.linear(xs[r0:r1], mg.experts[e])
                    h = ops.act(gu, F, ops.ACT_SWIGLU)
                    d = ops.reduce(ops.linear(h, md.experts[e]))
                    out.index_add_(0, tok[r0:r1], d * wsel[r0:r1].unsqueeze(1))
            return out

        ref = dense().float()
        td = timeit(dense)
        print(f"T={T} dense per-expert: {td:.1f} us ({flops / td / 1e6:.0f} TF/s)", flush=True)

        def bs(v):
            order, off = ops.moe_route(ids, E)
            h = ops.moe_glu_bs(x, mg, order, off, topk, T, var=v)
            return ops.moe_down_bs(h, md, order, off, topk, T, wts, var=v)

        order, off = ops.moe_route(ids, E)
        for v in sorted(ops.BS_TILES):
            d = bs(v).dense().float()
            rel = ((d - ref).norm() / ref.norm()).item()
            t = timeit(lambda: bs(v))
            h = ops.moe_glu_bs(x, mg, order, off, topk, T, var=v)
            t1 = timeit(lambda: ops.moe_glu_bs(x, mg, order, off, topk, T, var=v))
            t2 = timeit(lambda: ops.moe_down_bs(h, md, order, off, topk, T, wts, var=v))
            print(f"T={T} bs var {v}: {t:.1f} us ({flops / t / 1e6:.0f} TF/s; glu {t1:.1f} + down {t2:.1f})  "
                  f"rel-L2 vs dense {rel:.2e}", flush=True)
        for v in (15, 19):
            t = timeit(lambda: ops.moe_down32(ops.moe_glu32(x, mg, order, off, topk, T, var=v), md, order, off, topk,
                                              T, wts, var=v))
            print(f"T={T} moe32 var {v}: {t:.1f} us ({flops / t / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()

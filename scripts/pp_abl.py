"""Ablation / A-B builds of the prefill GEMM (ops/csrc/gemm_pp.hip), each a standalone .so with
the same C ABI, timed in ONE process interleaved (cdna_hip_programming.md §5.4 rule 24).

  python scripts/pp_abl.py --build                    # on the CPU host: compile the variants
  python scripts/pp_abl.py [--m 8192] [--rounds 5]    # on the GPU: time every built variant

Variants: name -> extra hipcc flags.  ABL bits (LA_PP_ABL): 1 no MFMA, 2 no dequant VALU,
4 no X DMA, 8 no W register loads, 16 no fragment LDS reads."""
import argparse
import ctypes
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
OUT = ROOT / "localai_amd" / "ops" / "build_pp"
SRC = ROOT / "localai_amd" / "ops" / "csrc" / "gemm_pp.hip"

NS = ["-fno-slp-vectorize"]  # the library's flag for gemm_pp.hip (ops/_build.py FILE_FLAGS)
VARIANTS = {
    "base": NS,
    "slp": [],
    "abl1": NS + ["-DLA_PP_ABL=1"],
    "abl2": NS + ["-DLA_PP_ABL=2"],
    "abl4": NS + ["-DLA_PP_ABL=4"],
    "abl8": NS + ["-DLA_PP_ABL=8"],
    "abl16": NS + ["-DLA_PP_ABL=16"],
    "abl10": NS + ["-DLA_PP_ABL=10"],
    "abl30": NS + ["-DLA_PP_ABL=30"],
    "gm1": NS + ["-DLA_PP_GM=1"],
    "gm4": NS + ["-DLA_PP_GM=4"],
    "stamp": NS + ["-DLA_PP_STAMP=1"],
}
for extra in os.environ.get("PP_EXTRA_VARIANTS", "").split(";"):
    if "=" in extra:
        k, v = extra.split("=", 1)
        VARIANTS[k] = v.split()


def build(names):
    OUT.mkdir(parents=True, exist_ok=True)
    procs = []
    for n in names:
        cmd = ["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-std=c++17",
               "-I", str(SRC.parent), *VARIANTS[n], str(SRC), "-o", str(OUT / f"_pp_{n}.so")]
        procs.append((n, subprocess.Popen(cmd, stderr=subprocess.PIPE, text=True)))
    for n, p in procs:
        err = p.communicate()[1]
        if p.returncode:
            raise SystemExit(f"{n}: {err[-3000:]}")
        print("built", n, flush=True)


def stamps(a):
    """Per-section cycle counts of K-tiles 10-11 (s_memtime) for 3 workgroups of gate_up."""
    import numpy as np
    import torch
    from localai_amd import ops
    from scripts.gq_bench import SHAPES, rand_qweight
    dev = torch.device("cuda:0")
    L = ctypes.CDLL(str(OUT / "_pp_stamp.so"))
    L.la_gemm_pp.argtypes = ops.lib().la_gemm_pp.argtypes
    L.la_gemm_pp_dbg.argtypes = [ctypes.c_void_p]
    for name in a.shapes.split(","):
        parts, K = SHAPES[name]
        n_, t_ = parts[0]
        w = rand_qweight(n_, K, t_, 0)
        for M in a.m:
            x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            out = torch.empty(M, w.N, dtype=torch.bfloat16, device=dev)
            dbg = torch.zeros(3 * 8 * 8 * 6, dtype=torch.int64, device=dev)
            assert L.la_gemm_pp_dbg(dbg.data_ptr()) == 0
            p0, p1, g = ops._pp_planes(w)
            for _ in range(3):
                assert L.la_gemm_pp(w.fmt, p0, p1, g, w.N, K, x.data_ptr(), K, M, 1, out.data_ptr(), w.N, 0, 1,
                                    ops._stream()) == 0
            torch.cuda.synchronize()
            d = dbg.cpu().numpy().reshape(3, 8, 8, 6).astype(np.int64)
            print(f"== {name} M={M}: cycles per section, mean over tiles 10-11 (rows: wave; cols: phase "
                  f"MEM/BAR1/LGKM/MFMA/BAR2)", flush=True)
            for b in range(3):
                tot = d[b, :, 7, 5] - d[b, :, 0, 0]
                print(f" block {b}: 2 K-tiles took {tot.mean():.0f} cycles (min {tot.min()}, max {tot.max()})")
                for wv in range(8):
                    secs = []
                    for ph in range(4):
                        v = [(d[b, wv, tt * 4 + ph, k + 1] - d[b, wv, tt * 4 + ph, k]) for tt in range(2) for k in range(5)]
                        v = np.array(v).reshape(2, 5).mean(0)
                        secs.append("/".join(f"{x:.0f}" for x in v))
                    print(f"  w{wv}: " + "  ".join(f"p{ph}:{sx}" for ph, sx in enumerate(secs)))


def bench(a):
    import numpy as np
    import torch
    from localai_amd import ops
    from scripts.gq_bench import SHAPES, rand_qweight
    dev = torch.device("cuda:0")
    libs = {}
    for n in VARIANTS:
        p = OUT / f"_pp_{n}.so"
        if n == "stamp" or (a.only and n not in a.only.split(",")):
            continue
        if p.exists():
            L = ctypes.CDLL(str(p))
            L.la_gemm_pp.argtypes = ops.lib().la_gemm_pp.argtypes
            L.la_gemm_pp.restype = ctypes.c_int
            libs[n] = L
    cases = []
    for name in a.shapes.split(","):
        parts, K = SHAPES[name]
        if name == "bf16":
            continue
        n_, t_ = parts[0]
        cases.append((name, rand_qweight(n_, K, t_, 0), K))
    if a.bf16:
        K = 4096
        wf = (torch.randn(28672, K, device=dev) * 0.02).to(torch.bfloat16)
        cases.append(("gate_up_bf16", ops.QWeight.from_float(wf), K))
    for name, w, K in cases:
        for M in a.m:
            x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            out = torch.empty(M, w.N, dtype=torch.bfloat16, device=dev)
            p0, p1, g = ops._pp_planes(w)
            flops = 2.0 * M * w.N * K
            res = {n: [] for n in libs}
            ref = None
            for n, L in libs.items():   # correctness of every non-ablation variant first
                if n.startswith("abl"):
                    continue
                if ref is None:
                    ref = ops._run_scratch_blas(x, [w], w.N).float()
                out.zero_()
                assert L.la_gemm_pp(w.fmt, p0, p1, g, w.N, K, x.data_ptr(), K, M, 1, out.data_ptr(), w.N, 0, 1,
                                    ops._stream()) == 0
                err = ((out.float() - ref).norm() / ref.norm()).item()
                print(f"check {n} {name} M={M}: rel-L2 {err:.2e}", flush=True)
                assert err < 1e-2, n
            for _ in range(a.rounds):
                for n, L in libs.items():
                    def fn(L=L):
                        rc = L.la_gemm_pp(w.fmt, p0, p1, g, w.N, K, x.data_ptr(), K, M, 1, out.data_ptr(), w.N, 0, 1,
                                          ops._stream())
                        assert rc == 0, rc
                    fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(3):
                        fn()
                    e1.record()
                    e1.synchronize()
                    res[n].append(e0.elapsed_time(e1) * 1000 / 3)
            line = " ".join(f"{n}:{np.median(v):.0f}us({flops / np.median(v) / 1e6:.0f}TF)" for n, v in res.items())
            print(f"{name} M={M} N={w.N} K={K}: {line}", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--m", type=int, nargs="+", default=[8192])
    ap.add_argument("--shapes", default="gate_up,down6")
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--stamp", action="store_true")
    a = ap.parse_args()
    if a.build:
        build([n for n in VARIANTS if not a.only or n in a.only.split(",")])
    elif a.stamp:
        stamps(a)
    else:
        bench(a)

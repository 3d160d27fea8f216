"""Ablation timings of gemm_dq's 8-wave kernel at the gate_up shape (M=256): which part of the
per-K-step schedule sets the time.  bits: 1 no MFMA, 2 no dequant VALU, 4 no X DMA, 8 no W DMA,
16 no barrier."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from localai_amd import ops  # noqa: E402
from scripts.dq_bench import qw, timeit  # noqa: E402

DEV = torch.device("cuda:0")
L = ops.lib()
L.la_qgemm_dq_probe.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int] * 2 + [ctypes.c_void_p] + [ctypes.c_int] * 2 + \
    [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
L.la_qgemm_dq_probe.restype = ctypes.c_int
for name, N, K, S in (("gate_up", 28672, 4096, 1), ("down", 4096, 14336, 8)):
    M = 256
    w = qw(N, K, 5)
    qsw, ssw = w.dq_planes()
    x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    out = torch.empty(S, M, N, dtype=torch.float32, device=DEV)
    res = {}
    for abl in (0, 1, 2, 3, 4, 8, 12, 13, 14, 15, 16, 31):
        fn = lambda: L.la_qgemm_dq_probe(qsw.data_ptr(), ssw.data_ptr(), N, K, x.data_ptr(), M, S, out.data_ptr(),  # noqa
                                         abl, ops._stream())
        assert fn() == 0
        res[abl] = (timeit(fn), timeit(fn, reps=5) if False else None)
        # warm (weights in MALL) timing as well
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        res[abl] = (res[abl][0], e0.elapsed_time(e1) * 100)
    print(name, " ".join(f"abl{a}: cold {c:.1f} warm {w_:.1f}" for a, (c, w_) in res.items()))

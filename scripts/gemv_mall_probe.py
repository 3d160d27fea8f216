"""Batch-1 decode GEMV with weights cold (HBM) vs resident in the 256 MiB Infinity Cache (MALL):
is a cross-kernel weight prefetch worth building?  Prints us per launch for Llama-3-8B shapes."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType, quantize  # noqa: E402

DEV = torch.device("cuda:0")


def qw(N, K, t, seed):
    rng = np.random.default_rng(seed)
    w = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    return ops.QWeight.from_raw(quantize(w, t), t, (N, K), DEV)


def ev_time(fn, prep=None, reps=5):
    ts = []
    for _ in range(reps):
        if prep:
            prep()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000)
    return sorted(ts)[len(ts) // 2]


for name, N, K, t in (("qkv", 6144, 4096, GGMLType.Q4_K), ("o", 4096, 4096, GGMLType.Q4_K),
                      ("gate_up", 28672, 4096, GGMLType.Q4_K), ("down_q6", 4096, 14336, GGMLType.Q6_K)):
    w = qw(N, K, t, 3)
    x = torch.randn(1, K, device=DEV).to(torch.bfloat16)
    S = ops._gemv_splits([w], K, 1)
    out = torch.empty(S, 1, N, dtype=torch.float32, device=DEV)
    fn = lambda: ops.gemv_dp4(x, [w], S, out)  # noqa: E731
    fn()
    cold = ev_time(fn, prep=lambda: ops._cold_caches(DEV))
    warm = ev_time(fn, prep=fn)  # the previous launch left the weights in MALL / L2
    planes = [p for p in w.planes if p is not None]
    nbytes = sum(p.numel() * p.element_size() for p in planes)

    def touch():  # stream the planes once (what a prefetch kernel would cost)
        for p in planes:
            p.view(torch.uint8).max()
    tt = ev_time(touch, prep=lambda: ops._cold_caches(DEV))
    print(f"{name:8s} {nbytes / 1e6:6.1f} MB  S={S}  cold {cold:6.1f} us ({nbytes / cold / 1e6:4.2f} TB/s)  "
          f"warm {warm:6.1f} us ({nbytes / warm / 1e6:4.2f} TB/s)  touch-cold {tt:6.1f} us", flush=True)

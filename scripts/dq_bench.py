"""Cold-cache timing of the batch-decode GEMM candidates at Llama-3-8B Q4_K shapes:
hipBLASLt on the bf16 copy, qgemm_mid (best tile/split), qgemm_ws, and gemm_dq (wave tile x split).
Usage: python scripts/dq_bench.py [M]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType, quantize  # noqa: E402

DEV = torch.device("cuda:0")
M = int(sys.argv[1]) if len(sys.argv) > 1 else 256
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def qw(N, K, seed):
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal((N, K)).astype(np.float32) * 0.05)
    return ops.QWeight.from_raw(quantize(w, GGMLType.Q4_K), GGMLType.Q4_K, (N, K), DEV)


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
    return sorted(ts)[len(ts) // 2]


def main():
    print(f"M = {M}")
    for name, (N, K) in SHAPES.items():
        w = qw(N, K, hash(name) % 1000)
        x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
        ref = ops._run_blas(x, [w], N).float()
        res = {"blas": timeit(lambda: ops._run_blas(x, [w], N))}
        for S in (1, 2, 4, 8):
            if (K // 64) % S:
                continue
            out = torch.empty(S, M, N, dtype=torch.float32, device=DEV)
            for t in (42, 41, 22, 21):
                res[f"mid{t}/S{S}"] = timeit(lambda: ops._run_mid(x, [w], S, out, N, t))
            if ops._ws_ok([w], K, S):
                res[f"ws/S{S}"] = timeit(lambda: ops._run_ws(x, [w], S, out, N))
            for wnt in (1,):
                res[f"dq{wnt}/S{S}"] = timeit(lambda: ops._run_dq(x, [w], S, out, N, wnt))
                ops._run_dq(x, [w], S, out, N, wnt)
                err = (out.sum(0) - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                if err > 3e-2:
                    print(f"  !! dq{wnt}/S{S} max rel err {err:.3g}")
        ob = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        for wnt in (1,):
            res[f"dq{wnt}/bf16"] = timeit(lambda: ops._run_dq(x, [w], 1, ob, N, wnt))
        flop = 2.0 * M * N * K
        best = sorted(res.items(), key=lambda kv: kv[1])
        line = "  ".join(f"{k}={v:.1f}" for k, v in best[:8])
        print(f"{name:8s} N={N} K={K}: {line}")
        print(f"{'':8s} blas {res['blas']:.1f} us ({flop / res['blas'] / 1e6:.0f} TF/s); best {best[0][0]} "
              f"{best[0][1]:.1f} us ({flop / best[0][1] / 1e6:.0f} TF/s)")


if __name__ == "__main__":
    main()

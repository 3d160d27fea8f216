"""Batch-1/2 decode GEMV (gemv_dp4.hip) split-K sweep on the Llama-3-8B shapes, timed the way the
engine runs it: launches captured in a hipGraph, cycling through enough weight copies that every
launch streams cold weights from HBM; per-launch µs = graph time / launches.

    python scripts/gemv_sweep.py [--m 1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
SHAPES = {
    "qkv": ([(5120, GGMLType.Q4_K), (1024, GGMLType.Q6_K)], 4096),
    "o": ([(4096, GGMLType.Q4_K)], 4096),
    "gate_up": ([(14336, GGMLType.Q4_K), (14336, GGMLType.Q4_K)], 4096),
    "down4": ([(4096, GGMLType.Q4_K)], 14336),
    "down6": ([(4096, GGMLType.Q6_K)], 14336),
}
# Llama-3-70B (d 8192, 64 q / 8 kv heads, ffn 28672)
SHAPES_70B = {
    "qkv": ([(9216, GGMLType.Q4_K), (1024, GGMLType.Q6_K)], 8192),
    "o": ([(8192, GGMLType.Q4_K)], 8192),
    "gate_up": ([(28672, GGMLType.Q4_K), (28672, GGMLType.Q4_K)], 8192),
    "down4": ([(8192, GGMLType.Q4_K)], 28672),
    "down6": ([(8192, GGMLType.Q6_K)], 28672),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--mib", type=int, default=600, help="weight bytes cycled through per graph")
    ap.add_argument("--preset", default="8b", choices=["8b", "70b"])
    a = ap.parse_args()
    M = a.m
    shapes = SHAPES_70B if a.preset == "70b" else SHAPES
    print("| shape | bytes/launch (MB) | default S | S:µs (TB/s) |")
    print("|---|---:|---:|---|")
    for name, (parts, K) in shapes.items():
        one = sum(n * K * (0.5625 if t == GGMLType.Q4_K else 0.8203) for n, t in parts)
        copies = max(2, int(a.mib * 2 ** 20 // one))
        sets = [[rand_qweight(n, K, t, seed=100 * c + i) for i, (n, t) in enumerate(parts)] for c in range(copies)]
        x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
        Ntot = sum(n for n, _ in parts)
        nsb = K // 256
        S0 = ops._gemv_splits(sets[0], K, M)
        res = []
        for S in [s for s in range(1, nsb + 1) if nsb % s == 0]:
            if M * (K // S) * (1 + 4 / 16 + 4 / 32) > 65536:
                continue
            out = torch.empty(S, M, Ntot, dtype=torch.float32, device=DEV)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                ops.gemv_dp4(x, sets[0], S, out)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for ws in sets:
                    ops.gemv_dp4(x, ws, S, out)
            g.replay()
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1000 / copies)
            t = sorted(ts)[2]
            res.append(f"{S}:{t:.1f} ({one / t / 1e6:.2f})")
            del g
        print(f"| {name} | {one / 1e6:.1f} | {S0} | {' '.join(res)} |", flush=True)
        del sets


if __name__ == "__main__":
    main()

"""Decode-batch GEMM probe: does a K-split library GEMM (strided-batched hipBLASLt, one batch per
K-slice, fp32 or bf16 slabs summed by the consumer) beat the single GEMM at M = 256?

At M = 256 a 256x256 output tile leaves N/256 workgroups (gate_up: 112 on 256 CUs), so the
library falls back to narrower tiles that re-read the activations more often.  Splitting K
multiplies the tile count by S at the price of S slabs.  Weights come cold from HBM (384 MiB
read between calls), as in the engine.  Prints one line per (shape, variant) with the median us.
"""
import os
import sys

import torch

# lm_head (128256 x 4096) is left out: its K-split strided-batched view with bf16 output faulted
# inside the library GEMM on MI355X (illegal address, round 2); the single GEMM wins there anyway
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    M = int(os.environ.get("PROBE_M", 256))
    tune = os.environ.get("PROBE_TUNE", "0") == "1"
    if tune:
        import torch.cuda.tunable as tn
        tn.enable(True)
        tn.tuning_enable(True)
        tn.set_max_tuning_duration(30)
        tn.set_max_tuning_iterations(30)
        tn.set_rotating_buffer_size(512)
        tn.set_filename("/tmp/splitk_probe_tune.csv")
    dev = torch.device("cuda:0")
    flush = torch.ones(96 << 20, dtype=torch.float32, device=dev)

    def timeit(fn, reps=7):
        fn()
        ts = []
        for _ in range(reps):
            flush.sum()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000)
        return sorted(ts)[reps // 2]

    for name, (N, K) in SHAPES.items():
        W = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        ref = (x.float() @ W.float().t())
        base = timeit(lambda: torch.matmul(x, W.t()))
        fl = 2.0 * M * N * K
        print(f"{name:8s} N={N:6d} K={K:5d} single      {base:8.1f} us  {fl / base / 1e6:7.1f} TF", flush=True)
        for S in (2, 4, 8):
            if K % S:
                continue
            ks = K // S
            xs = x.view(M, S, ks).permute(1, 0, 2)         # [S, M, ks], strides (ks, K, 1)
            Ws = W.view(N, S, ks).permute(1, 2, 0)         # [S, ks, N], strides (ks, 1, K)
            for od in (torch.float32, torch.bfloat16):
                try:
                    if od == torch.float32:
                        fn = lambda: torch.bmm(xs, Ws, out_dtype=torch.float32)  # noqa: E731
                    else:
                        fn = lambda: torch.bmm(xs, Ws)  # noqa: E731
                    y = fn().float().sum(0)
                    err = float((y - ref).abs().max() / ref.abs().max())
                    t = timeit(fn)
                    slab = S * M * N * (4 if od == torch.float32 else 2)
                    # the consumer reads S slabs instead of one bf16 output: charge the extra bytes at 4 TB/s
                    extra = (slab - M * N * 2) / 4e6
                    print(f"{name:8s} N={N:6d} K={K:5d} splitK{S} {str(od)[6:]:8s} {t:8.1f} us (+{extra:5.1f} consumer)"
                          f"  {fl / (t + extra) / 1e6:7.1f} TF  err {err:.2e}", flush=True)
                except Exception as e:  # noqa: BLE001
                    print(f"{name} splitK{S} {od}: {type(e).__name__}: {str(e)[:160]}", flush=True)
        del W
        torch.cuda.empty_cache()
    if tune:
        tn.write_file()


if __name__ == "__main__":
    sys.exit(main())

"""Mid-M (64..512) projection GEMMs of Llama-3-8B: default hipBLASLt choice vs. split-K through
bmm with fp32 output vs. PyTorch TunableOp (exhaustive hipBLASLt/rocBLAS solution search).
Writes the TunableOp result table to gpurun_out/tunableop_results.csv."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, ".")
dev = torch.device("cuda:0")
SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)]
MS = [int(m) for m in os.environ.get("PROBE_MS", "128,256,512").split(",")]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


res = {}
W = {}
for name, N, K in SHAPES:
    W[name] = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
for name, N, K in SHAPES:
    w = W[name]
    for M in MS:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        r = {"shape": name, "M": M, "default_us": bench(lambda: torch.matmul(x, w.t()))}
        for s in (2, 4, 8):
            if K % (s * 256):
                continue
            xs = x.view(M, s, K // s).transpose(0, 1)
            ws = w.view(N, s, K // s).transpose(0, 1).transpose(1, 2)
            try:
                r[f"splitk{s}_us"] = bench(lambda: torch.bmm(xs, ws, out_dtype=torch.float32))
            except Exception as e:  # noqa: BLE001
                r[f"splitk{s}_err"] = str(e)[:80]
        res[(name, M)] = r

import torch.cuda.tunable as tun  # noqa: E402
os.makedirs("gpurun_out", exist_ok=True)
tun.enable(True)
tun.tuning_enable(True)
tun.set_filename("gpurun_out/tunableop_results.csv")
tun.set_max_tuning_duration(300)
tun.set_max_tuning_iterations(50)
for name, N, K in SHAPES:
    w = W[name]
    for M in MS:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        t0 = time.time()
        torch.matmul(x, w.t())
        torch.cuda.synchronize()
        r = res[(name, M)]
        r["tune_s"] = round(time.time() - t0, 1)
        r["tuned_us"] = bench(lambda: torch.matmul(x, w.t()))
        fl = 2.0 * M * N * K
        r["tuned_tflops"] = fl / r["tuned_us"] / 1e6
        r["default_tflops"] = fl / r["default_us"] / 1e6
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
tun.write_file()

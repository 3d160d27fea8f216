"""Prefill-chunk GEMMs (M = 8192 tokens, Llama-3-8B shapes, bf16 weights): hipBLASLt default
heuristic vs PyTorch TunableOp-tuned solutions."""
import os
import time
import torch
dev = "cuda:0"
M = int(os.environ.get("PF_M", "8192"))
shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
x = {K: torch.randn(M, K, device=dev).bfloat16() for K in (4096, 14336)}
W = {n: torch.randn(N, K, device=dev).bfloat16() for n, (N, K) in shapes.items()}
def t(fn, n=10):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / n * 1e6
base = {n: t(lambda n=n: torch.matmul(x[shapes[n][1]], W[n].t())) for n in shapes}
import torch.cuda.tunable as tn
tn.enable(True); tn.tuning_enable(True); tn.set_filename("/tmp/pf_tune.csv")
tn.set_max_tuning_duration(int(os.environ.get("PF_TUNE_MS", "30"))); tn.set_max_tuning_iterations(20)
t0 = time.time()
for n in shapes:
    torch.matmul(x[shapes[n][1]], W[n].t())
torch.cuda.synchronize()
tune_s = time.time() - t0
tn.tuning_enable(False)
tuned = {n: t(lambda n=n: torch.matmul(x[shapes[n][1]], W[n].t())) for n in shapes}
for n, (N, K) in shapes.items():
    fl = 2 * M * N * K
    print(f"{n:8s} M={M} N={N} K={K}: default {base[n]:8.1f} us ({fl / base[n] / 1e6:6.0f} TF/s)  tuned {tuned[n]:8.1f} us ({fl / tuned[n] / 1e6:6.0f} TF/s)")
print(f"tuning took {tune_s:.1f} s")

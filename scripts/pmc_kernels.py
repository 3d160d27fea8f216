"""Hot kernels of the two headline regimes, 20 launches each, for rocprofv3 --pmc passes:
batch-1 decode GEMV (gate_up, Q4_K), batch-256 decode attention (L = 384), batch-256 quantised
GEMM (down, Q4_K on qgemm_mid), batch-256 add+RMSNorm.  Weights / KV rotate through copies larger
than the MALL so the counters see HBM traffic as in the engine."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from localai_amd import ops
from localai_amd.gguf import GGMLType, random_q4_k_blocks

dev = torch.device("cuda:0")
rng = np.random.default_rng(0)
N_IT = 20


def q4(N, K):
    return ops.QWeight.from_raw(random_q4_k_blocks(rng, N * K // 256, 0.02), GGMLType.Q4_K, (N, K), dev)


# 1. GEMV gate_up M=1 (66 MB per copy, 8 copies)
gu = [q4(28672, 4096) for _ in range(8)]
x1 = torch.randn(1, 4096, device=dev).to(torch.bfloat16)
S = ops._gemv_splits(gu[:1], 4096, 1)
out = torch.empty(S, 1, 28672, dtype=torch.float32, device=dev)
for i in range(N_IT):
    ops.gemv_dp4(x1, [gu[i % 8]], S, out)
torch.cuda.synchronize()
del gu

# 2. decode attention B=256, L=384 (Llama-3-8B heads), 4 layer copies
Hq, Hkv, Dh, BS, B, L = 32, 8, 128, 32, 256, 384
nb = L // BS
kcs = [(torch.randn(B * nb, Hkv, BS, Dh, device=dev) * 0.5).to(torch.bfloat16) for _ in range(4)]
vcs = [ops.v_from_rows((torch.randn(B * nb, Hkv, BS, Dh, device=dev) * 0.5).to(torch.bfloat16)) for _ in range(4)]
bt = torch.randperm(B * nb, device=dev).to(torch.int32).view(B, nb)
sl = torch.full((B,), L, dtype=torch.int32, device=dev)
q = torch.randn(B, Hq, Dh, device=dev).to(torch.bfloat16)
ws = ops.decode_workspace(B, Hq, Hkv, Dh, 2048, dev, BS)
o = torch.empty(B, Hq, Dh, dtype=torch.bfloat16, device=dev)
for i in range(N_IT):
    ops.attn_decode(q, kcs[i % 4], vcs[i % 4], bt, sl, 0.088, 2048, out=o, workspace=ws)
torch.cuda.synchronize()
del kcs, vcs

# 3. qgemm_mid down M=256 (Q4_K 4096 x 14336, 33 MB per copy, 10 copies)
dn = [q4(4096, 14336) for _ in range(10)]
x3 = torch.randn(256, 14336, device=dev).to(torch.bfloat16)
S3 = ops.pick_mid_splits(4096, 14336, 256)
o3 = torch.empty(S3, 256, 4096, dtype=torch.float32, device=dev)
for i in range(N_IT):
    ops._run_mid(x3, [dn[i % 10]], S3, o3, 4096, 41)
torch.cuda.synchronize()

# 4. add + RMSNorm at batch 256 over 8 split-K slabs
res = torch.randn(256, 4096, device=dev)
add = ops.Partial(torch.randn(8, 256, 4096, device=dev))
w = torch.ones(4096, device=dev)
for i in range(N_IT):
    ops.add_norm(res, add, w, None, 1e-5)
torch.cuda.synchronize()
print("PMC_KERNELS_OK")

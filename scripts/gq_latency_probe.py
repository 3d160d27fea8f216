"""Per-K-step latency of the tile GEMM when few workgroups run (qkv-shaped 6144x4096 Q4_K, M=256):
tiles x split-K with ablation builds (no X DMA / no W DMA / no DMA / no compute)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight, timeit  # noqa: E402

DEV = torch.device("cuda:0")
w = rand_qweight(6144, 4096, GGMLType.Q4_K, 0)
p0, _, g = w.tile_planes()
x = (torch.randn(256, 4096, device=DEV) * 0.5).to(torch.bfloat16)
for tile in (8, 7, 12):
    for S in (1, 4, 16):
        out = torch.empty(S, 256, w.N, dtype=torch.float32, device=DEV)
        line = []
        for abl in (0, 4, 8, 12, 3, 15):
            def fn(abl=abl):
                if abl == 0:
                    ops._run_tile(x, [w], S, out, w.N, tile)
                else:
                    assert ops.lib().la_qgemm_tile_probe(p0, g, w.N, 4096, x.data_ptr(), 256, S, out.data_ptr(), tile,
                                                         abl, ops._stream()) == 0
            line.append("abl%d=%.1f" % (abl, timeit(fn)))
        ks = 64 // S
        print(f"tile {tile} S={S} ({ks} K-steps/WG, {ops._tile_grid(256, 6144, tile) * S} WGs): " + " ".join(line),
              flush=True)

"""Launch driver for counter runs of the tile GEMM (gemm_q.hip): gate_up 28672x4096 Q4_K at
M = 256 for the production tiles and two ablation builds, 10 launches each (warm)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd import ops  # noqa: E402
from localai_amd.gguf import GGMLType  # noqa: E402
from scripts.gq_bench import rand_qweight  # noqa: E402

DEV = torch.device("cuda:0")
w = rand_qweight(28672, 4096, GGMLType.Q4_K, 0)
p0, _, g = w.tile_planes()
x = (torch.randn(256, 4096, device=DEV) * 0.5).to(torch.bfloat16)
for tile, S in ((6, 2), (16, 2), (10, 2)):
    out = torch.empty(S, 256, w.N, dtype=torch.float32, device=DEV)
    for _ in range(10):
        ops._run_tile(x, [w], S, out, w.N, tile)
    for abl in (15, 3):
        for _ in range(10):
            assert ops.lib().la_qgemm_tile_probe(p0, g, w.N, 4096, x.data_ptr(), 256, S, out.data_ptr(), tile, abl,
                                                 ops._stream()) == 0
torch.cuda.synchronize()
print("done")

"""Driver for stream_probe.hip: HBM read rate of GEMV weight access patterns.

Build (CPU, in-tree):  hipcc --offload-arch=gfx950 -O3 -shared -fPIC scripts/stream_probe.hip -o scripts/_stream_probe.so
"""
import ctypes
import os
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "_stream_probe.so"))
P, I, LNG = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
L.stream_probe.argtypes = [I, I, P, LNG, I, I, I, P, P]
dev = torch.device("cuda:0")
N, K = 28672, 4096
rowbytes = K // 2
copies = [torch.randint(0, 255, (N * rowbytes,), dtype=torch.uint8, device=dev) for _ in range(10)]
out = torch.zeros(4, dtype=torch.int32, device=dev)
nsb = K // 256
for pat in (0, 1, 2, 3):
    for depth in (2, 4, 8):
        for splits in (1, 2, 4):
            def run(i):
                L.stream_probe(pat, depth, copies[i % len(copies)].data_ptr(), rowbytes, N, nsb, splits,
                               out.data_ptr(), torch.cuda.current_stream().cuda_stream)
            for i in range(3):
                run(i)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(30):
                    run(i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.replay()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / 30 * 1e6
            print(f"pat={pat} depth={depth} splits={splits}: {us:7.2f} us  {N * rowbytes / us / 1e6:5.2f} TB/s",
                  flush=True)

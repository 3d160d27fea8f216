"""Time the on-device sampler per configuration (B rows x 128256 vocab, Llama-3 size)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from localai_amd import ops


def params(B, **kw):
    p = np.zeros(B, dtype=ops.SAMPLE_ROW_DTYPE)
    p["temp"] = kw.get("temp", 0.0)
    p["top_p"] = kw.get("top_p", 1.0)
    p["min_p"] = kw.get("min_p", 0.0)
    p["typical_p"] = kw.get("typical_p", 1.0)
    p["tfs_z"] = kw.get("tfs_z", 1.0)
    p["top_k"] = kw.get("top_k", 0)
    p["mirostat"] = kw.get("mirostat", 0)
    p["tau"] = 5.0
    p["eta"] = 0.1
    p["seed"] = np.arange(B) + 1
    return p


def main():
    V = 128256
    cfgs = {"greedy": {}, "mirostat2": dict(temp=0.9, mirostat=2),
            "topk40_topp0.95": dict(temp=0.9, top_k=40, top_p=0.95),
            "topp0.95_only": dict(temp=0.9, top_p=0.95)}
    for B in (1, 256):
        l = torch.randn(B, V, device="cuda") * 3
        for name, kw in cfgs.items():
            p = params(B, **kw)
            mu = torch.full((B,), 10.0, device="cuda")
            pd = torch.from_numpy(p.view(np.uint8).copy()).cuda()
            for _ in range(3):
                ops.sample(l, p, mu=mu, params_dev=pd)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.sample(l, p, mu=mu, params_dev=pd)
            e1.record()
            e1.synchronize()
            print(f"sample B={B:4d} {name:18s} {e0.elapsed_time(e1) / 20 * 1000:9.1f} us", flush=True)


if __name__ == "__main__":
    main()

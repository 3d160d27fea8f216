"""Which module of a diffusion UNet is not bitwise deterministic on the GPU: the same inputs run
twice (eager), every leaf module's output hashed, the first differing module named.

    python scripts/determinism_probe.py [--size tiny-xl]
"""
import argparse
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from localai_amd.models import synth  # noqa: E402
from localai_amd.models.sd import StableDiffusion  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", default="tiny-xl")
    ap.add_argument("--deterministic", action="store_true", help="torch.backends.cudnn.deterministic (MIOpen)")
    a = ap.parse_args()
    if a.deterministic:
        torch.backends.cudnn.deterministic = True
    d = synth.write_sd_pipeline(os.path.join(tempfile.mkdtemp(), "p"), size=a.size)
    p = StableDiffusion(d, "cuda:0")
    p.use_graphs = False
    rec = []
    hooks = []
    for name, m in p.unet.named_modules():
        if len(list(m.children())) == 0 or name.endswith(("attn1", "attn2")):
            hooks.append(m.register_forward_hook(
                lambda mod, inp, out, name=name: rec.append((name, out.detach().clone()
                                                             if torch.is_tensor(out) else None))))
    calls = []
    orig = p._model

    def wrapped(*ins):
        calls.append(tuple(None if v is None else v.clone() for v in ins))
        return orig(*ins)
    p._model = wrapped
    p("determinism", steps=1, seed=3, width=64, height=64)
    ins = calls[0]
    outs = []
    for _ in range(2):
        rec.clear()
        with torch.inference_mode():
            y = orig(*ins)
        torch.cuda.synchronize()
        outs.append((y.clone(), list(rec)))
    (y0, r0), (y1, r1) = outs
    import time
    for h in hooks:
        h.remove()
    with torch.inference_mode():
        for _ in range(3):
            orig(*ins)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            orig(*ins)
        torch.cuda.synchronize()
    print(f"UNet eager forward {(time.perf_counter() - t0) / 20 * 1e3:.2f} ms (deterministic={a.deterministic})")
    print(f"UNet output equal: {torch.equal(y0, y1)}  max diff {float((y0.float() - y1.float()).abs().max()):.3e}")
    for (n0, t0), (n1, t1) in zip(r0, r1):
        if t0 is None or t1 is None:
            continue
        if not torch.equal(t0, t1):
            print(f"FIRST NONDETERMINISTIC: {n0} {type(dict(p.unet.named_modules())[n0]).__name__} "
                  f"shape {tuple(t0.shape)} dtype {t0.dtype} max diff {float((t0.float() - t1.float()).abs().max()):.3e}")
            break
    else:
        print("every module output bitwise equal")


if __name__ == "__main__":
    main()

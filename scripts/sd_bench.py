"""Stable Diffusion 1.5 text-to-image latency (the `diffusers` backend path, models/sd.py):
random-init SD-1.5 architecture (860M-parameter UNet, CLIP ViT-L/14 text encoder, KL VAE),
512x512, DDIM, classifier-free guidance (UNet batch 2).  Prints seconds per image and UNet
iterations per second.

    python scripts/sd_bench.py --steps 20
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--nchw", action="store_true", help="keep NCHW activations (default NHWC)")
    a = ap.parse_args()
    import torch
    from localai_amd.models import synth
    from localai_amd.models.sd import StableDiffusion
    cache = os.environ.get("LOCALAI_AMD_CACHE", "/tmp/localai_amd_cache")
    d = os.path.join(cache, "sd15")
    if not os.path.exists(os.path.join(d, "model_index.json")):
        synth.write_sd_pipeline(d, size="sd15")
    print("pipeline written", flush=True)
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    p = StableDiffusion(d, dev, channels_last=not a.nchw)
    p("warm up", "", a.size, a.size, steps=2, seed=1)
    best = None
    for r in range(a.runs):
        torch.cuda.synchronize() if dev != "cpu" else None
        t0 = time.perf_counter()
        p("a photograph of an astronaut riding a horse", "blurry", a.size, a.size, steps=a.steps, seed=r + 2)
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
        print(f"run {r}: {el:.3f} s", flush=True)
    print(json.dumps({"metric": "SD-1.5 txt2img, diffusers backend", "size": a.size, "steps": a.steps,
                      "s_per_image": round(best, 3), "unet_it_s": round(a.steps / best, 2), "cfg": True, "layout": "nchw" if a.nchw else "nhwc", "hipgraph": bool(p.use_graphs and p._graphs),
                      "dtype": str(p.dtype).replace("torch.", "")}), flush=True)


if __name__ == "__main__":
    main()

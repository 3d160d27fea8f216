"""LLaVA-1.6-Mistral-7B latency and throughput (BASELINE.json config 5: image_url chat on the CLIP
ViT-L/14-336 + projector path), engine mode: random-init Mistral-7B Q4_K_M with a random-init
LLaVA-1.6 mmproj (anyres grid pinpoints, so one 672x336 image becomes 3 tiles + image_newline
rows), C concurrent requests each carrying one image.  Prints p50 time to first token (vision tower
+ splice + prefill) and output tokens/s.

    python scripts/llava_bench.py --concurrency 16 --max-tokens 64
"""
import argparse
import io
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _png(seed: int, w: int = 672, h: int = 336) -> bytes:
    import numpy as np
    from PIL import Image
    rng = np.random.default_rng(seed)
    img = Image.fromarray(rng.integers(0, 255, size=(h, w, 3), dtype=np.uint8))
    b = io.BytesIO()
    img.save(b, format="PNG")
    return b.getvalue()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=16)
    ap.add_argument("--max-tokens", type=int, default=64)
    ap.add_argument("--waves", type=int, default=2)
    a = ap.parse_args()
    import torch
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.engine.sampling_params import SamplingParams
    from localai_amd.models import synth
    cache = os.environ.get("LOCALAI_AMD_CACHE", "/tmp/localai_amd_cache")
    os.makedirs(cache, exist_ok=True)
    txt = os.path.join(cache, "mistral-7b.gguf")
    if not os.path.exists(txt):
        synth.write_model(txt + ".partial", "mistral-7b")
        os.replace(txt + ".partial", txt)
    mm = os.path.join(cache, "llava16-mmproj.gguf")
    if not os.path.exists(mm):
        synth.write_mmproj(mm + ".partial", out_dim=4096,
                           pinpoints=[336, 672, 672, 336, 672, 672, 1008, 336, 336, 1008])
        os.replace(mm + ".partial", mm)
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    eng = LLMEngine(EngineConfig(model_path=txt, device=dev, context_size=4096, max_num_seqs=max(a.concurrency, 1),
                                 max_batched_tokens=8192, mmproj=mm))
    eng.warmup()
    best = None
    for w in range(a.waves + 1):
        # new images every wave: the prefix cache keys image positions by the image's hash, so a
        # repeated image would skip the vision tower and its prefill
        imgs = [_png(w * 1000 + i) for i in range(a.concurrency)]
        done, ttft, ntok = [0], [], [0]
        lock = threading.Lock()
        t0 = time.perf_counter()
        for i in range(a.concurrency):
            first = [True]

            def cb(ev, first=first):
                with lock:
                    if first[0] and (ev.text or ev.finished):
                        first[0] = False
                        ttft.append(time.perf_counter() - t0)
                    if ev.finished:
                        ntok[0] += ev.completion_tokens
                        done[0] += 1
            prompt = f"[INST] [img-0]\n({w}.{i}) Describe the image in detail. [/INST]"
            eng.add_request(prompt, SamplingParams(max_tokens=a.max_tokens, temperature=0.0, ignore_eos=True), cb,
                            images=[imgs[i]])
        while done[0] < a.concurrency:
            eng.step()
        el = time.perf_counter() - t0
        if w == 0:
            continue  # warm-up wave
        tt = sorted(ttft)
        res = (ntok[0] / el, tt[len(tt) // 2] * 1e3, el)
        if best is None or res[0] > best[0]:
            best = res
    n_img_tokens = eng.clip.embed_image(imgs[0]).shape[0]
    print(json.dumps({"metric": "LLaVA-1.6-Mistral-7B image chat, engine", "concurrency": a.concurrency,
                      "output_tok_s": round(best[0], 1), "p50_ttft_ms": round(best[1], 1), "wall_s": round(best[2], 3),
                      "image_tokens": int(n_img_tokens), "max_tokens": a.max_tokens}), flush=True)
    eng.shutdown()


if __name__ == "__main__":
    main()

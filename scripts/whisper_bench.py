"""Whisper transcription speed on the native worker (the reference's `whisper` backend, whisper.cpp):
a random-init whisper-base-sized GGML model (6+6 layers, width 512), 60 s of 16 kHz audio (two 30-s
windows), real-time factor = wall / audio seconds.  Random weights decode up to the per-window token
cap, so this is the worst-case decode length."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from localai_amd.models import synth
    from localai_amd.models.whisper import WhisperModel
    cache = os.environ.get("LOCALAI_AMD_CACHE", "/tmp/localai_amd_cache")
    os.makedirs(cache, exist_ok=True)
    p = os.path.join(cache, "ggml-base-random.bin")
    if not os.path.exists(p):
        synth.write_whisper(p + ".partial", n_audio_state=512, n_audio_head=8, n_audio_layer=6, n_text_state=512,
                            n_text_head=8, n_text_layer=6)
        os.replace(p + ".partial", p)
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    m = WhisperModel(p, dev)
    rng = np.random.default_rng(0)
    audio = (0.1 * rng.standard_normal(16000 * 60)).astype(np.float32)
    m.transcribe(audio[:16000 * 5], language="en")  # warm-up
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    segs, text = m.transcribe(audio, language="en")
    if dev.startswith("cuda"):
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"metric": "whisper-base (random-init) transcription", "audio_s": 60, "wall_s": round(el, 3),
                      "rtf": round(el / 60, 4), "segments": len(segs)}), flush=True)


if __name__ == "__main__":
    main()

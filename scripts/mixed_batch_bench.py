"""Decode throughput of a 256-stream engine wave when ONE stream needs host-side sampling work:
all plain (device multi-step decode), 1 repeat-penalised + 255 plain (penalty ring inside the
decode graph), 1 GBNF-constrained (`[a-z ]+`) + 255 plain (the batch drops to one device
step per host round trip: the grammar row is masked on the host, the other 255 rows keep device
sampling).  Llama-3-8B Q4_K_M shapes, random init, 128-token prompts, 128 generated tokens."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
from localai_amd.engine.sampling_params import SamplingParams
from localai_amd.models import synth

C, PLEN, NGEN = 256, 128, 128
path = os.path.join(os.environ.get("LOCALAI_AMD_CACHE", "/tmp/la_cache"), "llama3-8b.gguf")
os.makedirs(os.path.dirname(path), exist_ok=True)
if not os.path.exists(path):
    synth.write_model(path, "llama3-8b")
eng = LLMEngine(EngineConfig(model_path=path, device="cuda:0", context_size=2048, max_num_seqs=C,
                             max_kv_tokens=C * (PLEN + NGEN + 64) + 4096))
eng.warmup()
words = "the model server token request graph kernel memory stream batch".split()


def wave(tag, special):
    done, toks = [0], [0]

    def cb(ev):
        if ev.finished:
            done[0] += 1
            toks[0] += ev.completion_tokens
    for i in range(C):
        prompt = f"{tag} {i}: " + " ".join(words[(i + j) % len(words)] for j in range(PLEN - 8))
        sp = SamplingParams(max_tokens=NGEN, temperature=0.0, ignore_eos=True)
        if i == 0 and special == "penalty":
            sp = SamplingParams(max_tokens=NGEN, temperature=0.0, ignore_eos=True, repeat_penalty=1.1)
        elif i == 0 and special == "grammar":
            # a grammar that never completes, so the constrained stream lasts the whole wave
            sp = SamplingParams(max_tokens=NGEN, temperature=0.0, ignore_eos=True, grammar='root ::= [a-z ]+')
        eng.add_request(prompt, sp, cb)
    # time the decode phase only: from the step after the last prefill to the end
    t_first = None
    while done[0] < C:
        eng.step()
        if t_first is None and eng.sched.num_waiting == 0 and not any(
                r.n_gen == 0 for r in eng.requests.values()):
            t_first, tok0 = time.perf_counter(), sum(r.n_gen for r in eng.requests.values())
    el = time.perf_counter() - t_first
    return (toks[0] - tok0) / el


wave("warm", "")
eng.k1_reasons.clear()
eng.k_hist.clear()
for special in ("", "penalty", "grammar", ""):
    eng.k1_reasons.clear()
    eng.k_hist.clear()
    eng.k_log.clear()
    r = wave(f"w{time.time():.0f}", special)
    print(f"{special or 'plain':8s} decode {r:9.1f} tok/s", flush=True)
    if special == "grammar":
        m = eng.metrics
        print(f"  grammar runs {m['grammar_runs']} rows {m['grammar_run_rows']} tokens {m['grammar_run_tokens']} "
              f"hit-rate {dict((k[:20], round(v, 3)) for k, v in eng._ghit.items())} "
              f"single-step reasons {dict(eng.k1_reasons)} runs by (K, constrained rows) {dict(eng.k_hist)}",
              flush=True)
        print("  run sequence (K, constrained, batch, waiting):", list(eng.k_log), flush=True)
    eng.k1_reasons.clear()
    eng.k_hist.clear()

"""Function-calling throughput (BASELINE.json config 4's "+ GBNF function-calling" half): C concurrent
streaming /v1/chat/completions requests with a forced tool (`tool_choice` naming the function, so
every token is sampled under the GBNF grammar generated from its JSON schema), through the real
gateway on the native HTTP server, on random-init Llama-3-8B Q4_K_M.  Prints tokens/s and checks
that a non-streaming request returns a tool call whose arguments parse under the schema.

    python scripts/fc_bench.py --concurrency 32 [--waves 8 --max-tokens 256]

Measurement (same engine, same box): WAVES forced-tool waves, WAVES plain waves and WAVES plain
waves with the FC wave's per-request lengths, interleaved so drift hits all alike; each request asks for MAX_TOKENS (256).  The
throughput tool's schema ends in an open string field ("notes"), so a random-init model keeps
sampling under the grammar's string state until max_tokens (the enum fields before it exercise
the bounded states); plain waves use ignore_eos.  Reported: median tokens/s of each kind and
their ratio.  The validity checks use the all-enum tool, whose calls close on their own.
"""
import argparse
import json
import os
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TOOLS = [{"type": "function", "function": {
    "name": "get_weather", "description": "current weather for a city",
    "parameters": {"type": "object", "properties": {
        "location": {"type": "string", "enum": ["paris", "tokyo", "lima", "oslo"]},
        "unit": {"type": "string", "enum": ["celsius", "fahrenheit"]},
        "days": {"type": "string", "enum": ["1", "3", "7"]}}, "required": ["location", "unit", "days"]}}}]
CHOICE = {"type": "function", "function": {"name": "get_weather"}}
# throughput tool: bounded fields first, then an open string the model fills until max_tokens
TOOLS_TP = [{"type": "function", "function": {
    "name": "log_weather", "description": "record a weather observation",
    "parameters": {"type": "object", "properties": {
        "location": {"type": "string", "enum": ["paris", "tokyo", "lima", "oslo"]},
        "unit": {"type": "string", "enum": ["celsius", "fahrenheit"]},
        "notes": {"type": "string"}}, "required": ["location", "unit", "notes"]}}}]
CHOICE_TP = {"type": "function", "function": {"name": "log_weather"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=32)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--preset", default="llama3-8b")
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--checks", type=int, default=8, help="non-streaming requests whose tool call is validated")
    a = ap.parse_args()
    from localai_amd.utils.loadgen import LoadGen
    lg = LoadGen(2)  # client processes first: nothing forks after the GPU is initialised
    import torch
    from localai_amd.engine.llm_engine import EngineConfig, LLMEngine
    from localai_amd.gateway.app import create_app_for_engine
    from localai_amd.gateway.native_server import NativeHTTPServer
    from localai_amd.models import synth
    cache = os.environ.get("LOCALAI_AMD_CACHE", "/tmp/localai_amd_cache")
    os.makedirs(cache, exist_ok=True)
    path = os.path.join(cache, f"{a.preset}.gguf")
    if not os.path.exists(path):
        synth.write_model(path + ".partial", a.preset)
        os.replace(path + ".partial", path)
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    eng = LLMEngine(EngineConfig(model_path=path, device=dev, context_size=2048, max_num_seqs=max(a.concurrency, 1),
                                 max_batched_tokens=8192))
    eng.warmup()
    eng.start()
    app, name = create_app_for_engine(eng, name="llama3-8b-instruct")
    srv = NativeHTTPServer(app, "127.0.0.1", 0)
    import threading
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    while not srv.started:
        time.sleep(0.05)
    url = f"http://127.0.0.1:{srv.port}/v1/chat/completions"
    extra = {"tools": TOOLS, "tool_choice": CHOICE, "temperature": 0}
    msgs = [f"(q{i}) What is the weather like in city number {i} for the next few days?" for i in range(a.concurrency)]
    extra_tp = {"tools": TOOLS_TP, "tool_choice": CHOICE_TP, "temperature": 0}
    lg.wave(url, name, msgs[:2], 8, extra=extra)  # warm the grammar paths
    lg.wave(url, name, msgs[:2], 8, extra=extra_tp)
    import statistics
    fc_r, pl_r, pm_r, fc_tok = [], [], [], []
    plain_extra = {"temperature": 0, "ignore_eos": True}
    for w in range(a.waves):
        t0 = time.perf_counter()
        _, tok = lg.wave(url, name, [f"[{w}] " + m for m in msgs], a.max_tokens, extra=extra_tp)
        fc_r.append(tok / (time.perf_counter() - t0))
        fc_tok.append(tok)
        per = list(lg.last_per)
        # same concurrency and token budget without the grammar, on the same engine (same box)
        t0 = time.perf_counter()
        _, tok = lg.wave(url, name, [f"[p{w}] " + m for m in msgs], a.max_tokens, extra=plain_extra)
        pl_r.append(tok / (time.perf_counter() - t0))
        # ... and with the FC wave's per-request lengths (a tool call that closes early leaves the
        # batch thinner at the tail: the matched wave isolates the grammar's own cost)
        t0 = time.perf_counter()
        _, tok = lg.wave(url, name, [f"[m{w}] " + m for m in msgs], [max(1, v) for v in per], extra=plain_extra)
        pm_r.append(tok / (time.perf_counter() - t0))
        print(f"wave {w}: fc {fc_r[-1]:.1f} tok/s ({fc_tok[-1]} tokens)  plain {pl_r[-1]:.1f} tok/s  "
              f"plain-matched {pm_r[-1]:.1f} tok/s ({tok} tokens)", file=sys.stderr, flush=True)
    fc_med, pl_med, pm_med = statistics.median(fc_r), statistics.median(pl_r), statistics.median(pm_r)

    def check(content):
        body = json.dumps({"model": name, "max_tokens": a.max_tokens, "messages": [{"role": "user", "content": content}],
                           **extra}).encode()
        req = urllib.request.Request(url, data=body, headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=600) as r:
            doc = json.loads(r.read())
        msg = doc["choices"][0]["message"]
        calls = msg.get("tool_calls") or []
        ok = False
        if calls:
            fn = calls[0]["function"]
            try:
                args = json.loads(fn["arguments"])
                ok = fn["name"] == "get_weather" and args.get("unit") in ("celsius", "fahrenheit") and \
                    args.get("days") in ("1", "3", "7") and args.get("location") in ("paris", "tokyo", "lima", "oslo")
            except (ValueError, TypeError):
                ok = False
        if not ok:
            print(f"INVALID tool call for {content!r}: finish={doc['choices'][0]['finish_reason']} "
                  f"usage={doc.get('usage')} message={json.dumps(msg)[:600]}", file=sys.stderr, flush=True)
        return ok, doc, msg, calls
    n_ok = 0
    for i in range(a.checks):
        ok, d_, m_, c_ = check(msgs[i % len(msgs)])
        n_ok += int(ok)
        if i == 0:
            ok0, doc, msg, calls = ok, d_, m_, c_
    ok = ok0
    m = eng.metrics
    print(f"grammar runs {m['grammar_runs']} rows {m['grammar_run_rows']} tokens {m['grammar_run_tokens']} "
          f"hit-rate {[round(v, 3) for v in eng._ghit.values()]}", file=sys.stderr, flush=True)
    print(json.dumps({"metric": "function-calling output tokens/s (forced tool, GBNF-constrained)",
                      "value": round(fc_med, 1), "plain_value": round(pl_med, 1),
                      "fc_over_plain": round(fc_med / pl_med, 3), "plain_matched_value": round(pm_med, 1),
                      "fc_over_plain_matched": round(fc_med / pm_med, 3), "waves": a.waves,
                      "fc_waves": [round(v, 1) for v in fc_r], "plain_waves": [round(v, 1) for v in pl_r],
                      "fc_tokens_per_wave": fc_tok, "preset": a.preset, "concurrency": a.concurrency,
                      "max_tokens": a.max_tokens, "finish_reason": doc["choices"][0]["finish_reason"],
                      "tool_call_valid": ok, "valid_calls": f"{n_ok}/{a.checks}",
                      "sample_call": calls[0]["function"] if calls else msg.get("content"),
                      "k1_reasons": dict(eng.k1_reasons)}),
          flush=True)
    lg.close()
    srv.shutdown()
    th.join(timeout=10)
    eng.shutdown()


if __name__ == "__main__":
    main()

"""Per-request gateway cost on the CPU (no GPU): the real app (routes, config merge, Go-template
chat rendering, servicer, Llama-3 BPE tokenisation) in front of an engine stub that finishes
every request at once, driven through the native HTTP server by the out-of-process load
generator.  Prints requests/s for a 256-request burst and, with --profile, the top functions of
the gateway thread by cumulative time (cProfile)."""
import argparse
import os
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class StubEngine:
    """Tokenises like the engine (caller thread), then ends the request after one token."""

    def __init__(self, tokenizer, model_path):
        import torch
        from localai_amd.engine.llm_engine import Event
        self.Event, self.tokenizer, self.device = Event, tokenizer, torch.device("cpu")
        self.n = 0

        class C:
            context_size = 4096
        C.model_path = model_path
        self.cfg = C()

    def tokenize(self, s, add_bos=None):
        return self.tokenizer.encode(s, add_bos=add_bos)

    def add_request(self, prompt, params, cb, req_id=None, sink=None, images=None):
        toks = self.tokenize(prompt) if isinstance(prompt, str) else list(prompt)
        self.n += 1
        if sink is not None:
            sink.set_prompt_tokens(len(toks))
            sink.push(b" x", 1)
        cb(self.Event(text=b"" if sink is not None else b" x", finished=True, finish_reason="length",
                      prompt_tokens=len(toks), completion_tokens=1))
        return self.n

    def abort(self, rid):
        pass

    def shutdown(self):
        pass


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--clients", type=int, default=4)
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    from localai_amd.gguf import GGUFReader
    from localai_amd.gateway.app import create_app_for_engine
    from localai_amd.gateway.native_server import NativeHTTPServer
    from localai_amd.models import synth
    from localai_amd.tokenizer import Tokenizer
    from localai_amd.utils.loadgen import LoadGen
    lg = LoadGen(a.clients)  # before anything heavy
    path = os.path.join(tempfile.gettempdir(), "gw_profile_llama3_tok.gguf")
    if not os.path.exists(path):
        synth.write_model(path, "tiny-llama", n_vocab=128256, tokenizer="llama3")
    tok = Tokenizer.from_gguf(GGUFReader(path))
    eng = StubEngine(tok, path)
    app, name = create_app_for_engine(eng, name="llama3-8b-instruct")
    srv = NativeHTTPServer(app, "127.0.0.1", 0)
    prof = None
    if a.profile:  # the gateway runs on the server thread: profile that thread
        import cProfile
        prof = cProfile.Profile()

        def run():
            prof.enable()
            try:
                srv.run()
            finally:
                prof.disable()
    th = threading.Thread(target=run if prof is not None else srv.run, daemon=True)
    th.start()
    while not srv.started:
        time.sleep(0.05)
    url = f"http://127.0.0.1:{srv.port}/v1/chat/completions"
    words = "the model server token request graph kernel memory stream batch latency context".split()
    msgs = [f"(wave 0) Request {i}: " + " ".join(words[(i + j) % len(words)] for j in range(100))
            for i in range(a.requests)]
    lg.wave(url, name, msgs[:16], 1, extra={"temperature": 0, "ignore_eos": True, "mirostat": 0})
    import psutil

    def srv_cpu():  # CPU seconds of the server thread (the gateway's event loop)
        return sum(t.user_time + t.system_time for t in psutil.Process().threads() if t.id == th.native_id)
    c0 = srv_cpu()
    t0 = time.perf_counter()
    ttft, _ = lg.wave(url, name, msgs, 1, extra={"temperature": 0, "ignore_eos": True, "mirostat": 0})
    el = time.perf_counter() - t0
    cpu = srv_cpu() - c0
    print(f"{a.requests} requests in {el * 1e3:.1f} ms: {a.requests / el:.0f} req/s, "
          f"{el / a.requests * 1e3:.3f} ms per request; p50 ttft {sorted(ttft)[len(ttft) // 2] * 1e3:.1f} ms; "
          f"gateway thread CPU {cpu / a.requests * 1e3:.3f} ms per request")
    lg.close()
    srv.shutdown()
    th.join(10)
    if prof is not None:
        import pstats
        pstats.Stats(prof).sort_stats(os.environ.get("SORT", "tottime")).print_stats(30)
        if os.environ.get("PROF_OUT"):
            prof.dump_stats(os.environ["PROF_OUT"])


if __name__ == "__main__":
    main()

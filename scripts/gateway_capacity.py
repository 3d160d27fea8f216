"""Gateway capacity probe (CPU only): a fake engine that emits one token per active stream
every `--step-ms`, served through the real gateway, driven by the out-of-process load
generator.  Reports delivered tokens/s vs. what the fake engine produced, i.e. how many
streamed tokens/s the HTTP layer can carry before it becomes the bottleneck."""
import argparse
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class FakeEngine:
    def __init__(self, step_ms: float):
        import torch
        from localai_amd.engine.llm_engine import Event
        self.Event = Event
        self.device = torch.device("cpu")
        self.step_s = step_ms / 1000.0
        self.lock = threading.Lock()
        self.reqs = {}
        self.next = 1
        self.busy = False
        self.produced = 0

        class C:
            context_size = 4096
            model_path = "fake.gguf"
        self.cfg = C()
        threading.Thread(target=self._loop, daemon=True).start()

    def tokenize(self, s, add_bos=None):
        return list(range(len(s.split())))

    def add_request(self, prompt, params, cb, sink=None):
        with self.lock:
            rid = self.next
            self.next += 1
            self.reqs[rid] = [cb, params.max_tokens, 0, sink]
        if sink is not None:
            sink.set_prompt_tokens(10)
        return rid

    def abort(self, rid):
        with self.lock:
            self.reqs.pop(rid, None)

    def _loop(self):
        while True:
            t0 = time.perf_counter()
            with self.lock:
                items = list(self.reqs.items())
            for rid, r in items:
                cb, mx, n, sink = r
                r[2] = n + 1
                self.produced += 1
                if r[2] >= mx:
                    with self.lock:
                        self.reqs.pop(rid, None)
                    cb(self.Event(text=b" tok", finished=True, finish_reason="length", prompt_tokens=10,
                                  completion_tokens=r[2]))
                elif sink is not None:
                    if not sink.push(b" tok", r[2]):
                        with self.lock:
                            self.reqs.pop(rid, None)
                else:
                    cb(self.Event(text=b" tok"))
            dt = time.perf_counter() - t0
            time.sleep(max(0.0, self.step_s - dt))

    def shutdown(self):
        pass


def main():
    sys.setswitchinterval(float(os.environ.get("SWITCH", "0.005")))
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=256)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--step-ms", type=float, default=10.0)
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--server", default="native", choices=["native", "uvicorn"])
    a = ap.parse_args()
    import socket
    import uvicorn
    from localai_amd.gateway.app import create_app_for_engine
    from localai_amd.utils.loadgen import LoadGen
    eng = FakeEngine(a.step_ms)
    app, name = create_app_for_engine(eng, name="fake")
    if a.server == "native":
        from localai_amd.gateway.native_server import NativeHTTPServer
        srv = NativeHTTPServer(app, "127.0.0.1", 0)
        port = srv.port
    else:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning", access_log=False))
    threading.Thread(target=srv.run, daemon=True).start()
    while not srv.started:
        time.sleep(0.05)
    lg = LoadGen(a.clients)
    url = f"http://127.0.0.1:{port}/v1/chat/completions"
    msgs = [f"hello {i}" for i in range(a.concurrency)]
    lg.wave(url, name, msgs[:8], 4)
    t0 = time.perf_counter()
    p0 = eng.produced
    ttft, tok = lg.wave(url, name, msgs, a.max_tokens)
    el = time.perf_counter() - t0
    ideal = a.concurrency * 1000.0 / a.step_ms
    print(f"C={a.concurrency} step={a.step_ms}ms: delivered {tok / el:.0f} tok/s (engine ideal {ideal:.0f}), "
          f"produced {(eng.produced - p0) / el:.0f}/s, wall {el:.2f}s, p50 ttft {sorted(ttft)[len(ttft) // 2] * 1e3:.1f}ms")
    lg.close()


if __name__ == "__main__":
    main()

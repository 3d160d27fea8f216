"""Engine event timeline (SURVEY §5.1 "MI355X plan": per-step batch size, prefill/decode time,
queue wait; correlation IDs end to end).

The reference has no tracing: `X-Correlation-ID` is read by the gateway but never reaches the
backend (`core/backend/options.go:180-229` drops it), and the C++ server only logs per-slot
timings when a slot is released (`grpc-server.cpp:305-359`).  Here:

* `LOCALAI_AMD_TRACE=/path/trace.json` records a Chrome/Perfetto trace of the engine: one
  complete event per prefill / decode step (batch, tokens, device steps per host round trip),
  counters for running / waiting sequences and KV blocks, and per request an arrival instant,
  a first-token instant and a request span -- all tagged with the request's correlation ID.
  The file is (re)written every `LOCALAI_AMD_TRACE_FLUSH` seconds (default 5) and at shutdown.
* `LOCALAI_AMD_ROCTX=1` additionally brackets prefill / decode / graph replays with roctx
  ranges (torch.cuda.nvtx is roctx on ROCm), visible in `rocprofv3 --marker-trace`.
"""
from __future__ import annotations

import json
import os
import threading
import time
from contextlib import contextmanager
from typing import Optional

_T0 = time.perf_counter()


def _us(t: float) -> float:
    return (t - _T0) * 1e6


class Tracer:
    def __init__(self, path: str, flush_every_s: float = 5.0, max_events: int = 2_000_000):
        self.path = path
        self.flush_every_s = flush_every_s
        self.max_events = max_events
        self._ev = []
        self._lock = threading.Lock()
        self._last_flush = time.perf_counter()
        self.pid = os.getpid()
        self._dropped = 0

    def _add(self, ev: dict):
        with self._lock:
            if len(self._ev) >= self.max_events:
                self._dropped += 1
                return
            self._ev.append(ev)
        if time.perf_counter() - self._last_flush > self.flush_every_s:
            self.flush()

    def complete(self, name: str, t0: float, t1: float, cat: str = "engine", tid: int = 0, **args):
        self._add({"name": name, "cat": cat, "ph": "X", "ts": _us(t0), "dur": max(0.0, (t1 - t0) * 1e6),
                   "pid": self.pid, "tid": tid, "args": args})

    def instant(self, name: str, t: float, cat: str = "engine", tid: int = 0, **args):
        self._add({"name": name, "cat": cat, "ph": "i", "s": "t", "ts": _us(t), "pid": self.pid, "tid": tid,
                   "args": args})

    def counter(self, name: str, t: float, **values):
        self._add({"name": name, "ph": "C", "ts": _us(t), "pid": self.pid, "args": values})

    def flush(self):
        with self._lock:
            evs = list(self._ev)
            dropped = self._dropped
            self._last_flush = time.perf_counter()
        doc = {"traceEvents": evs, "displayTimeUnit": "ms",
               "otherData": {"producer": "localai_amd", "dropped_events": dropped}}
        tmp = f"{self.path}.tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(doc, f)
        os.replace(tmp, self.path)


_TRACER: Optional[Tracer] = None
_INIT = False


def get_tracer() -> Optional[Tracer]:
    """The process tracer when LOCALAI_AMD_TRACE names an output file, else None."""
    global _TRACER, _INIT
    if not _INIT:
        _INIT = True
        path = os.environ.get("LOCALAI_AMD_TRACE")
        if path:
            _TRACER = Tracer(path, float(os.environ.get("LOCALAI_AMD_TRACE_FLUSH", "5")))
    return _TRACER


def reset_for_tests():
    global _TRACER, _INIT
    _TRACER, _INIT = None, False


_ROCTX = os.environ.get("LOCALAI_AMD_ROCTX") == "1"


@contextmanager
def roctx(name: str):
    """roctx range (torch.cuda.nvtx maps to roctx on ROCm); no-op unless LOCALAI_AMD_ROCTX=1."""
    if not _ROCTX:
        yield
        return
    import torch
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()

"""Test-only fault injection (SURVEY §5.3 "MI355X plan": kill a rank, drop the gRPC stream, make
hipMalloc fail).  The reference has none (§5.3 "No fault injection anywhere").

    LOCALAI_AMD_FAULT="engine_step:3,grpc_stream_drop:1,kv_alloc,worker_exit:2"

Each entry `site[:n]` fires ONCE, on the n-th time (default 1st) the code passes that site:

    engine_step       LLMEngine.step raises a fatal device error -> in-flight requests fail,
                      the engine reports unhealthy, the model manager respawns it
    kv_alloc          KV-cache allocation fails like hipMalloc -> LoadModel returns an error
    grpc_stream_drop  PredictStream dies after its first message -> the gateway ends the SSE
                      stream with an error and the engine frees the sequence
    worker_exit       the out-of-process worker exits (os._exit) when serving its n-th request
                      -> the gateway sees the dead process and respawns it
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional, Tuple

_lock = threading.Lock()
_spec: Optional[Dict[str, Tuple[int, int]]] = None  # site -> (fire_at, seen)


class InjectedFault(RuntimeError):
    """Raised by an armed fault site."""


def _load() -> Dict[str, Tuple[int, int]]:
    global _spec
    if _spec is None:
        spec = {}
        for part in os.environ.get("LOCALAI_AMD_FAULT", "").split(","):
            part = part.strip()
            if not part:
                continue
            name, _, n = part.partition(":")
            spec[name.strip()] = (int(n) if n.strip() else 1, 0)
        _spec = spec
    return _spec


def hit(site: str) -> bool:
    """True exactly once: the n-th time `site` is reached (n from LOCALAI_AMD_FAULT)."""
    spec = _load()
    if site not in spec:
        return False
    with _lock:
        at, seen = spec[site]
        seen += 1
        spec[site] = (at, seen)
        return seen == at


def armed(site: str) -> bool:
    return site in _load()


def reset():
    """Re-read LOCALAI_AMD_FAULT (tests)."""
    global _spec
    _spec = None

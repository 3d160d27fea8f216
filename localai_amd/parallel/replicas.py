"""In-server data parallelism: one model served by N engine replicas (one per GPU, or per TP
group), behind ONE backend handle that the gateway uses like any other.

Reference: the reference scales a model over GPUs/hosts only by running more LocalAI instances
behind its federated load balancer (`core/p2p/federated_server.go:36-107`, least-used worker
selection in `core/p2p/federated.go` SelectLeastUsedServer) or by vLLM's own replicas
(`backend/python/vllm/backend.py:102-103`).  Here one gateway process owns the replicas:

  * dispatch: least in-flight requests first (the federated server's least-used rule, counted
    per request instead of per TCP connection), ties broken round-robin;
  * prefix affinity: requests whose prompt shares its first `affinity_chars` characters (system
    prompt, chat-template header, few-shot block) prefer the replica that served that prefix
    last, so its prefix cache hits -- unless that replica carries `affinity_slack` more
    in-flight requests than the least-loaded one;
  * stateful RPCs (Stores*) always go to replica 0 (one store, not N diverging copies);
    LoadModel / Free / health / close go to every replica;
  * Status / GetMetrics report the replica that is busiest (the one a caller polls for).

Each replica is any handle with the backend.proto call surface (`grpc.rpc.GRPCBackend` for
worker processes, `EmbeddedBackend` for in-process engines)."""
from __future__ import annotations

import contextvars
import hashlib
import itertools
import threading
from typing import List, Optional, Sequence

from ..grpc import backend_pb as pb

# replica chosen by pick_native() for this task's next streaming call (a remote one)
_PINNED: contextvars.ContextVar = contextvars.ContextVar("localai_amd_replica_pin", default=None)
STREAM_RPCS = {r for r, _, _, s in pb.RPCS if s}
STICKY_RPCS = {"StoresSet", "StoresDelete", "StoresGet", "StoresFind"}
BROADCAST_RPCS = {"LoadModel", "Free"}
OBSERVE_RPCS = {"Status", "GetMetrics"}


def _prompt_key(req, chars: int) -> Optional[str]:
    """Affinity key of a PredictOptions: its prompt (or first messages) prefix."""
    text = getattr(req, "Prompt", "") or ""
    if not text:
        msgs = getattr(req, "Messages", None)
        if msgs:
            text = "".join(f"{getattr(m, 'role', '')}:{getattr(m, 'content', '')}" for m in list(msgs)[:2])
    if not text or len(text) < chars // 4:
        return None
    return hashlib.blake2b(text[:chars].encode("utf-8", "ignore"), digest_size=8).hexdigest()


class ReplicaBackend:
    """N replica handles behind one backend.proto call surface."""

    def __init__(self, replicas: Sequence, names: Optional[Sequence[str]] = None, affinity_chars: int = 512,
                 affinity_slack: int = 8, affinity_entries: int = 4096):
        if not replicas:
            raise ValueError("ReplicaBackend needs at least one replica")
        self.replicas: List = list(replicas)
        self.names = list(names) if names else [getattr(r, "addr", str(i)) for i, r in enumerate(self.replicas)]
        self.addr = ",".join(self.names)
        self.inflight = [0] * len(self.replicas)
        self.served = [0] * len(self.replicas)
        self._rr = itertools.count()
        self._lock = threading.Lock()
        self.affinity_chars = affinity_chars
        self.affinity_slack = affinity_slack
        self._affinity: dict = {}
        self._aff_cap = affinity_entries

    # ------------------------------------------------------------------ selection
    def pick(self, req=None) -> int:
        """Replica index for a request: least in-flight, prefix-affine when cheap enough."""
        with self._lock:
            n = len(self.replicas)
            start = next(self._rr) % n
            order = [(start + i) % n for i in range(n)]
            best = min(order, key=lambda i: self.inflight[i])
            key = _prompt_key(req, self.affinity_chars) if req is not None else None
            if key is not None:
                pref = self._affinity.get(key)
                if pref is not None and self.inflight[pref] <= self.inflight[best] + self.affinity_slack:
                    best = pref
                else:
                    if len(self._affinity) >= self._aff_cap:
                        self._affinity.pop(next(iter(self._affinity)))
                    self._affinity[key] = best
            self.inflight[best] += 1
            self.served[best] += 1
            return best

    def _done(self, i: int) -> None:
        with self._lock:
            self.inflight[i] = max(0, self.inflight[i] - 1)

    def pick_native(self, request):
        """Replica choice for the gateway's native SSE fast path (openai_routes._native_stream),
        which hands tokens to an in-process engine without the RPC surface.  Returns (i, servicer)
        for an in-process replica -- counted in flight until `_done(i)` -- or (i, None) for a
        remote one, which is then pinned for this task's next streaming RPC so the generic path
        sends the request exactly where the balancer chose."""
        i = self.pick(request)
        sv = vars(self.replicas[i]).get("servicer")
        if sv is not None and getattr(sv, "engine", None) is not None:
            return i, sv
        with self._lock:
            self.inflight[i] -= 1
            self.served[i] -= 1
        _PINNED.set(i)
        return i, None

    def _pick_stream(self, request) -> int:
        i = _PINNED.get()
        if i is None:
            return self.pick(request)
        _PINNED.set(None)
        with self._lock:
            self.inflight[i] += 1
            self.served[i] += 1
        return i

    # ------------------------------------------------------------------ call surface
    def __getattr__(self, rpc):
        if rpc.startswith("_") or rpc not in {r for r, _, _, _ in pb.RPCS}:
            raise AttributeError(rpc)
        if rpc in STREAM_RPCS:
            def call_stream(request, timeout=None):
                i = self._pick_stream(request)
                return self._stream(i, rpc, request, timeout)
            return call_stream
        if rpc in BROADCAST_RPCS:
            async def call_all(request, timeout=None):
                res = None
                for h in self.replicas:
                    r = await getattr(h, rpc)(request, timeout=timeout)
                    if res is None or (hasattr(r, "success") and not r.success):
                        res = r
                return res
            return call_all
        if rpc in STICKY_RPCS:
            async def call_first(request, timeout=None):
                return await getattr(self.replicas[0], rpc)(request, timeout=timeout)
            return call_first
        if rpc in OBSERVE_RPCS:
            async def call_busiest(request, timeout=None):
                i = max(range(len(self.replicas)), key=lambda j: self.inflight[j])
                return await getattr(self.replicas[i], rpc)(request, timeout=timeout)
            return call_busiest

        async def call(request, timeout=None):
            i = self.pick(request)
            try:
                return await getattr(self.replicas[i], rpc)(request, timeout=timeout)
            finally:
                self._done(i)
        return call

    async def _stream(self, i: int, rpc: str, request, timeout):
        try:
            async for rep in getattr(self.replicas[i], rpc)(request, timeout=timeout):
                yield rep
        finally:
            self._done(i)

    async def health(self, timeout: float = 5.0) -> bool:
        for h in self.replicas:
            if hasattr(h, "health") and not await h.health(timeout=timeout):
                return False
        return True

    async def close(self):
        for h in self.replicas:
            if hasattr(h, "close"):
                await h.close()

    def stats(self) -> dict:
        with self._lock:
            return {"replicas": self.names, "inflight": list(self.inflight), "served": list(self.served)}

"""Federated request-level load balancer (`core/p2p/federated_server.go`, `federated.go`,
`core/cli/federated.go`): one front door that forwards each HTTP request to one of N LocalAI
instances (e.g. one per MI355X node, or one per GPU when running data-parallel replicas) and
streams the response back.  Worker choice: an explicit target, least active requests (the
reference's SelectLeastUsedServer), or random.  Instead of libp2p discovery the worker list is
static (`--workers` / LOCALAI_FEDERATED_WORKERS) plus runtime registration via
POST /federated/workers; unhealthy workers (failed /readyz) are skipped until they recover.
"""
from __future__ import annotations

import asyncio
import logging
import random
import time
from typing import Dict, List, Optional

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response, StreamingResponse

log = logging.getLogger("localai_amd.federated")

HOP_HEADERS = {"connection", "keep-alive", "proxy-authenticate", "proxy-authorization", "te", "trailers",
               "transfer-encoding", "upgrade", "host", "content-length"}


class Worker:
    def __init__(self, url: str):
        self.url = url.rstrip("/")
        self.active = 0
        self.served = 0
        self.healthy = True
        self.last_check = 0.0


class FederatedBalancer:
    def __init__(self, workers: List[str], strategy: str = "least-used", target: str = ""):
        self.workers: Dict[str, Worker] = {w.rstrip("/"): Worker(w) for w in workers if w}
        self.strategy = strategy
        self.target = target.rstrip("/")

    def pick(self) -> Optional[Worker]:
        live = [w for w in self.workers.values() if w.healthy] or list(self.workers.values())
        if not live:
            return None
        if self.target and self.target in self.workers:
            return self.workers[self.target]
        if self.strategy == "random":
            return random.choice(live)
        return min(live, key=lambda w: (w.active, w.served))

    async def health_loop(self, session, interval: float = 10.0):
        while True:
            for w in list(self.workers.values()):
                try:
                    async with session.get(w.url + "/readyz", timeout=5) as r:
                        w.healthy = r.status == 200
                except Exception:
                    w.healthy = False
                w.last_check = time.time()
            await asyncio.sleep(interval)


def create_federated_app(balancer: FederatedBalancer) -> FastAPI:
    import aiohttp
    state = {"session": None, "task": None}
    from contextlib import asynccontextmanager

    @asynccontextmanager
    async def lifespan(app):
        state["session"] = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=None, sock_connect=10))
        state["task"] = asyncio.get_running_loop().create_task(balancer.health_loop(state["session"]))
        yield
        state["task"].cancel()
        await state["session"].close()

    app = FastAPI(title="LocalAI federated", lifespan=lifespan)

    @app.get("/federated/workers")
    async def list_workers():
        return [{"url": w.url, "active": w.active, "served": w.served, "healthy": w.healthy}
                for w in balancer.workers.values()]

    @app.post("/federated/workers")
    async def add_worker(request: Request):
        b = await request.json()
        url = str(b.get("url", "")).rstrip("/")
        if not url:
            return JSONResponse({"error": "url required"}, status_code=400)
        balancer.workers.setdefault(url, Worker(url))
        return {"ok": True}

    @app.get("/api/p2p")
    async def p2p_nodes():
        return {"nodes": [{"id": w.url, "online": w.healthy} for w in balancer.workers.values()]}

    @app.api_route("/{path:path}", methods=["GET", "POST", "PUT", "DELETE", "PATCH"])
    async def proxy(path: str, request: Request):
        w = balancer.pick()
        if w is None:
            return JSONResponse({"error": {"code": 503, "message": "no federated workers"}}, status_code=503)
        body = await request.body()
        headers = {k: v for k, v in request.headers.items() if k.lower() not in HOP_HEADERS}
        url = f"{w.url}/{path}"
        if request.url.query:
            url += "?" + request.url.query
        sess = state["session"]
        w.active += 1
        w.served += 1
        try:
            resp = await sess.request(request.method, url, data=body, headers=headers)
        except Exception as e:
            w.active -= 1
            w.healthy = False
            return JSONResponse({"error": {"code": 502, "message": f"worker {w.url}: {e}"}}, status_code=502)
        out_headers = {k: v for k, v in resp.headers.items() if k.lower() not in HOP_HEADERS}

        async def body_iter():
            try:
                async for chunk in resp.content.iter_any():
                    yield chunk
            finally:
                resp.release()
                w.active -= 1
        if "text/event-stream" in resp.headers.get("content-type", ""):
            return StreamingResponse(body_iter(), status_code=resp.status, headers=out_headers)
        data = await resp.read()
        resp.release()
        w.active -= 1
        return Response(data, status_code=resp.status, headers=out_headers)

    return app

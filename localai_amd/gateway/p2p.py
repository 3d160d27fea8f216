"""`run --p2p`: network membership, node census and the p2p API/UI of a LocalAI instance.

Reference: `core/cli/run.go` (P2P token generation and start), `core/p2p/p2p.go:31-438` (join a
network, announce services, discover nodes), `core/p2p/node.go:13-66` (NodeData, 40-s liveness,
per-service node registry), `core/http/endpoints/localai/p2p.go` (`GET /api/p2p`,
`GET /api/p2p/token`), `core/http/routes/ui.go:89-118` (`/p2p` page and its htmx fragments).

The reference joins an edgevpn/libp2p network named by a token.  Here the transport between
instances is plain HTTP and the intra-node data plane is RCCL (`parallel/`), so a network token
is the explorer's token (`gateway/explorer.py`): base64 of {network_id, federated: [balancer
URLs], workers: [instance URLs]}.  With `--p2p`:
  - no token given: one is generated naming this instance as the network's first worker, and
    logged (the reference prints its generated token the same way);
  - a token given: this instance announces itself to every federated balancer the token lists
    (`POST /federated/workers`), which is what makes a balancer route requests to it.
A census thread then probes the token's balancers (their worker lists) and workers (`/readyz`)
every `interval` seconds and records NodeData with LastSeen, so `/api/p2p` reports online nodes
with the reference's 40-second rule.
"""
from __future__ import annotations

import html
import json
import logging
import os
import socket
import threading
import time
import urllib.error
import urllib.request
from dataclasses import dataclass
from datetime import datetime, timezone
from typing import Callable, Dict, List, Optional

from fastapi import APIRouter
from fastapi.responses import HTMLResponse, PlainTextResponse

from .explorer import decode_network_token, make_network_token

log = logging.getLogger("localai_amd.p2p")

WORKER_ID = "worker"          # core/p2p/node.go:10
FEDERATED_ID = "federated"    # core/p2p/federated.go
ONLINE_S = 40.0               # NodeData.IsOnline (node.go:21-25)


def network_service_id(network_id: str, service: str) -> str:
    """`p2p.NetworkID`: "<network>_<service>" or the bare service name."""
    return f"{network_id}_{service}" if network_id else service


@dataclass
class NodeData:
    Name: str
    ID: str
    TunnelAddress: str = ""
    ServiceID: str = ""
    LastSeen: float = 0.0

    def is_online(self, now: Optional[float] = None) -> bool:
        return ((now or time.time()) - self.LastSeen) < ONLINE_S

    def to_json(self) -> dict:
        return {"Name": self.Name, "ID": self.ID, "TunnelAddress": self.TunnelAddress, "ServiceID": self.ServiceID,
                "LastSeen": datetime.fromtimestamp(self.LastSeen, timezone.utc).isoformat()}


class NodeRegistry:
    """Per-service node tables (node.go:27-66)."""

    def __init__(self):
        self._mu = threading.Lock()
        self._nodes: Dict[str, Dict[str, NodeData]] = {}

    def add(self, service_id: str, node: NodeData) -> None:
        with self._mu:
            self._nodes.setdefault(service_id or "services", {})[node.ID] = node

    def available(self, service_id: str) -> List[NodeData]:
        with self._mu:
            return list(self._nodes.get(service_id or "services", {}).values())


def advertise_url(address: str) -> str:
    """This instance's URL as other instances reach it: LOCALAI_ADVERTISE_URL, or the bind
    address with a wildcard host replaced by the host name."""
    env = os.environ.get("LOCALAI_ADVERTISE_URL", "").rstrip("/")
    if env:
        return env
    host, _, port = address.rpartition(":")
    if host in ("", "0.0.0.0", "::", "[::]"):
        host = socket.gethostname()
    return f"http://{host}:{port or '8080'}"


def _get_json(url: str, timeout: float):
    with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310 (network members' URLs)
        return json.loads(r.read() or b"null")


def _probe(url: str, timeout: float) -> bool:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310
            return r.status == 200
    except (urllib.error.URLError, OSError, ValueError):
        return False


def _announce(balancer: str, me: str, timeout: float) -> bool:
    req = urllib.request.Request(balancer.rstrip("/") + "/federated/workers", method="POST",
                                 data=json.dumps({"url": me}).encode(), headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:  # noqa: S310
            return r.status == 200
    except (urllib.error.URLError, OSError, ValueError):
        return False


class P2PNode:
    """Network membership of one instance: token, announce, periodic census."""

    def __init__(self, token: str, network_id: str, self_url: str, interval: float = 10.0, timeout: float = 5.0,
                 get_json: Callable[[str, float], object] = _get_json, probe: Callable[[str, float], bool] = _probe,
                 announce: Callable[[str, str, float], bool] = _announce):
        self.self_url = self_url.rstrip("/")
        if not token:
            token = make_network_token(workers=[self.self_url], network_id=network_id)
            log.info("p2p: generated network token (share it with --p2ptoken / the explorer): %s", token)
        self.token = token
        self.net = decode_network_token(token)  # ValueError on a malformed token
        self.network_id = network_id or self.net["network_id"]
        self.registry = NodeRegistry()
        self.interval, self.timeout = interval, timeout
        self._get_json, self._probe, self._announce = get_json, probe, announce
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None

    def worker_service(self) -> str:
        return network_service_id(self.network_id, WORKER_ID)

    def federated_service(self) -> str:
        return network_service_id(self.network_id, FEDERATED_ID)

    def census_once(self) -> None:
        now = time.time()
        for bal in self.net["federated"]:
            base = bal.rstrip("/")
            if self.self_url not in self.net["workers"]:
                self._announce(base, self.self_url, self.timeout)  # (re-)join: balancers may restart
            try:
                doc = self._get_json(base + "/federated/workers", self.timeout)
            except (urllib.error.URLError, OSError, ValueError):
                continue
            self.registry.add(self.federated_service(), NodeData(Name=base, ID=base, TunnelAddress=base,
                                                                 ServiceID=self.federated_service(), LastSeen=now))
            for w in doc if isinstance(doc, list) else []:
                if isinstance(w, dict) and w.get("healthy") and w.get("url"):
                    u = str(w["url"]).rstrip("/")
                    self.registry.add(self.worker_service(), NodeData(Name=u, ID=u, TunnelAddress=u,
                                                                      ServiceID=self.worker_service(), LastSeen=now))
        for u in self.net["workers"]:
            u = u.rstrip("/")
            if u == self.self_url or self._probe(u + "/readyz", self.timeout):
                self.registry.add(self.worker_service(), NodeData(Name=u, ID=u, TunnelAddress=u,
                                                                  ServiceID=self.worker_service(), LastSeen=now))

    def start(self) -> None:
        def loop():
            while not self._stop.is_set():
                try:
                    self.census_once()
                except Exception:  # noqa: BLE001 - the census must outlive a bad peer
                    log.exception("p2p census failed")
                self._stop.wait(self.interval)
        self._th = threading.Thread(target=loop, name="p2p-census", daemon=True)
        self._th.start()

    def stop(self) -> None:
        self._stop.set()

    def nodes(self) -> dict:
        """`schema.P2PNodesResponse`: every known node of each service (online or not; the UI
        marks them), as the reference's GetAvailableNodes does."""
        return {"nodes": [n.to_json() for n in self.registry.available(self.worker_service())],
                "federated_nodes": [n.to_json() for n in self.registry.available(self.federated_service())]}


def _boxes(nodes: List[NodeData]) -> str:
    now = time.time()
    out = []
    for n in nodes:
        on = n.is_online(now)
        out.append(f"<div class='node'><b>{html.escape(n.Name)}</b> "
                   f"<span class='{'on' if on else 'off'}'>{'online' if on else 'offline'}</span>"
                   f"<div class='muted'>last seen {int(now - n.LastSeen)} s ago</div></div>")
    return "".join(out) or "<p class='muted'>No nodes yet.</p>"


def _stats(nodes: List[NodeData]) -> str:
    on = sum(1 for n in nodes if n.is_online())
    return f"<b>{on}</b>/<b>{len(nodes)}</b>"


def build_router(node: Optional[P2PNode]) -> APIRouter:
    """`/api/p2p`, `/api/p2p/token` (p2p builds only in the reference: here when --p2p is on) and
    the `/p2p` page with its htmx fragment routes."""
    r = APIRouter()
    if node is None:
        return r

    @r.get("/api/p2p")
    async def p2p_nodes():
        return node.nodes()

    @r.get("/api/p2p/token")
    async def p2p_token():
        return PlainTextResponse(node.token)

    @r.get("/p2p/ui/workers")
    async def ui_workers():
        return HTMLResponse(_boxes(node.registry.available(node.worker_service())))

    @r.get("/p2p/ui/workers-federation")
    async def ui_fed():
        return HTMLResponse(_boxes(node.registry.available(node.federated_service())))

    @r.get("/p2p/ui/workers-stats")
    async def ui_workers_stats():
        return HTMLResponse(_stats(node.registry.available(node.worker_service())))

    @r.get("/p2p/ui/workers-federation-stats")
    async def ui_fed_stats():
        return HTMLResponse(_stats(node.registry.available(node.federated_service())))

    @r.get("/p2p")
    async def p2p_page():
        from .webui import _page
        body = (
            "<h2>Distributed inference</h2>"
            "<p class='muted'>Instances that share this network token form one network: a federated balancer "
            "(<code>local-ai federated</code>) routes requests across them, and each node runs its own "
            "tensor-parallel group over RCCL/xGMI inside the machine.</p>"
            "<h3>Network token</h3><pre id='tok' style='white-space:pre-wrap;word-break:break-all'></pre>"
            "<p class='muted'>Start another instance with <code>local-ai run --p2p --p2ptoken &lt;token&gt;</code>, "
            "or add the token to an explorer.</p>"
            "<h3>Workers <span id='ws'></span></h3><div id='workers'></div>"
            "<h3>Federated balancers <span id='fs'></span></h3><div id='fed'></div>")
        script = ("async function load(u,id){const r=await fetch(u);document.getElementById(id).innerHTML=await r.text();}"
                  "async function tok(){const r=await fetch('/api/p2p/token');"
                  "document.getElementById('tok').textContent=await r.text();}"
                  "function refresh(){load('/p2p/ui/workers','workers');load('/p2p/ui/workers-federation','fed');"
                  "load('/p2p/ui/workers-stats','ws');load('/p2p/ui/workers-federation-stats','fs');}"
                  "tok();refresh();setInterval(refresh,5000);")
        return _page("LocalAI - P2P", body, script)

    return r

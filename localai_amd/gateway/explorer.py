"""Network explorer: a directory of LocalAI deployments and a discovery loop that keeps it
current.  Reference: `core/cli/explorer.go:12-49` (command and flags),
`core/explorer/database.go:15-125` (flock-guarded JSON token database),
`core/explorer/discovery.go:16-213` (per-token connect, cluster census, failure threshold,
deletion) and `core/http/endpoints/explorer/dashboard.go:12-102` + `routes/explorer.go:9-13`
(`GET /`, `POST /network/add`, `GET /networks`).

The reference's tokens name libp2p/edgevpn networks and discovery reads their ledger.  This
framework replaces p2p with RCCL tensor parallelism inside a node and the federated HTTP
balancer across nodes (`gateway/federated.py`), so a *network token* here is base64 of either
  - a JSON document ``{"network_id": str, "federated": [url, ...], "workers": [url, ...]}``, or
  - a bare URL of a federated balancer.
Discovery asks each federated balancer for its worker list (`GET /federated/workers`, the
analogue of the ledger's federated service entries) and probes each listed worker's `/readyz`
(the analogue of a worker node's liveness), giving the same ClusterData{Workers, Type,
NetworkID} census the reference stores.  A token whose network shows no online worker gains a
failure; past `--connection-error-threshold` failures it is removed, as in the reference.
"""
from __future__ import annotations

import base64
import binascii
import fcntl
import html
import json
import logging
import os
import threading
import time
import urllib.error
import urllib.request
from dataclasses import asdict, dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

from fastapi import FastAPI, Request
from fastapi.responses import HTMLResponse, JSONResponse

log = logging.getLogger("localai_amd.explorer")


@dataclass
class ClusterData:
    Workers: List[str] = field(default_factory=list)
    Type: str = ""
    NetworkID: str = ""


@dataclass
class TokenData:
    name: str = ""
    description: str = ""
    Clusters: List[ClusterData] = field(default_factory=list)
    Failures: int = 0

    @staticmethod
    def from_json(d: dict) -> "TokenData":
        cl = [ClusterData(Workers=list(c.get("Workers") or []), Type=c.get("Type", ""),
                          NetworkID=c.get("NetworkID", "")) for c in (d.get("Clusters") or [])]
        return TokenData(name=d.get("name", ""), description=d.get("description", ""), Clusters=cl,
                         Failures=int(d.get("Failures", 0)))


class Database:
    """JSON file keyed by token.  Every operation takes an exclusive `flock` on `<path>.lock`
    (other processes: an explorer running `--only-sync` beside the web server) and a mutex
    (threads of this process), re-reads the file, and writes it back after a change."""

    def __init__(self, path: str):
        self.path = path
        self._mu = threading.Lock()
        self.data: Dict[str, TokenData] = {}
        with self._locked():
            pass

    def _locked(self):
        db = self

        class _Ctx:
            def __enter__(self_):
                db._mu.acquire()
                d = os.path.dirname(os.path.abspath(db.path))
                os.makedirs(d, exist_ok=True)
                self_.fd = os.open(db.path + ".lock", os.O_CREAT | os.O_RDWR, 0o644)
                fcntl.flock(self_.fd, fcntl.LOCK_EX)
                db._load()
                return db

            def __exit__(self_, *exc):
                try:
                    fcntl.flock(self_.fd, fcntl.LOCK_UN)
                    os.close(self_.fd)
                finally:
                    db._mu.release()
                return False
        return _Ctx()

    def _load(self) -> None:
        if not os.path.exists(self.path):
            self.data = {}
            return
        with open(self.path) as f:
            raw = f.read()
        doc = json.loads(raw) if raw.strip() else {}
        self.data = {k: TokenData.from_json(v) for k, v in doc.items()}

    def _save(self) -> None:
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump({k: asdict(v) for k, v in self.data.items()}, f)
        os.replace(tmp, self.path)

    def get(self, token: str) -> Tuple[TokenData, bool]:
        with self._locked():
            t = self.data.get(token)
            return (t if t is not None else TokenData()), t is not None

    def set(self, token: str, t: TokenData) -> None:
        with self._locked():
            self.data[token] = t
            self._save()

    def delete(self, token: str) -> None:
        with self._locked():
            self.data.pop(token, None)
            self._save()

    def token_list(self) -> List[str]:
        with self._locked():
            return sorted(self.data)


# ---- network tokens -------------------------------------------------------------------------

def make_network_token(federated: Optional[List[str]] = None, workers: Optional[List[str]] = None,
                       network_id: str = "") -> str:
    doc = {"network_id": network_id, "federated": list(federated or []), "workers": list(workers or [])}
    return base64.b64encode(json.dumps(doc, separators=(",", ":")).encode()).decode()


def decode_network_token(token: str) -> dict:
    """Token -> {"network_id", "federated", "workers"}; raises ValueError when the token is not
    base64 of a network document or of an http(s) URL."""
    try:
        raw = base64.b64decode(token.encode(), validate=True).decode()
    except (binascii.Error, UnicodeDecodeError, ValueError) as e:
        raise ValueError("invalid token") from e
    raw = raw.strip()
    if raw.startswith(("http://", "https://")):
        return {"network_id": "", "federated": [raw], "workers": []}
    try:
        doc = json.loads(raw)
    except json.JSONDecodeError as e:
        raise ValueError("invalid token") from e
    if not isinstance(doc, dict):
        raise ValueError("invalid token")
    fed = [str(u) for u in doc.get("federated") or []]
    wk = [str(u) for u in doc.get("workers") or []]
    if not fed and not wk:
        raise ValueError("token names no federated server or worker")
    return {"network_id": str(doc.get("network_id", "")), "federated": fed, "workers": wk}


def _http_json(url: str, timeout: float):
    with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310 (operator-supplied URLs)
        return r.status, json.loads(r.read() or b"null")


def _http_ok(url: str, timeout: float) -> bool:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310
            return r.status == 200
    except (urllib.error.URLError, OSError, ValueError):
        return False


class DiscoveryServer:
    """Keeps the database in step with the networks (`discovery.go:43-134`): one token at a
    time, each bounded by `connection_timeout`; a token whose network has online workers gets
    its clusters replaced and its failure count reset, any other token gains a failure, and
    tokens past `error_threshold` failures are deleted at the end of the pass."""

    def __init__(self, db: Database, connection_timeout: float = 50.0, error_threshold: int = 3,
                 fetch_json: Optional[Callable[[str, float], tuple]] = None,
                 probe: Optional[Callable[[str, float], bool]] = None):
        self.db = db
        self.connection_timeout = connection_timeout or 50.0
        self.error_threshold = error_threshold or 3
        self._fetch_json = fetch_json or _http_json
        self._probe = probe or _http_ok
        self._mu = threading.Lock()

    def census(self, token: str) -> List[ClusterData]:
        net = decode_network_token(token)
        deadline = time.monotonic() + self.connection_timeout
        left = lambda: max(0.5, min(10.0, deadline - time.monotonic()))  # noqa: E731
        clusters: List[ClusterData] = []
        for url in net["federated"]:
            base = url.rstrip("/")
            try:
                status, doc = self._fetch_json(base + "/federated/workers", left())
            except (urllib.error.URLError, OSError, ValueError):
                continue
            if status != 200 or not isinstance(doc, list):
                continue
            online = [str(w.get("url")) for w in doc if isinstance(w, dict) and w.get("healthy") and w.get("url")]
            if online:
                clusters.append(ClusterData(Workers=online, Type="federated", NetworkID=net["network_id"]))
        workers = [u.rstrip("/") for u in net["workers"] if time.monotonic() < deadline
                   and self._probe(u.rstrip("/") + "/readyz", left())]
        if workers:
            clusters.append(ClusterData(Workers=workers, Type="worker", NetworkID=net["network_id"]))
        return clusters

    def run_once(self) -> None:
        for token in self.db.token_list():
            try:
                clusters = self.census(token)
            except ValueError as e:
                log.warning("explorer: token %s...: %s", token[:12], e)
                clusters = []
            with self._mu:
                data, _ = self.db.get(token)
                if any(c.Workers for c in clusters):
                    data.Clusters = clusters
                    data.Failures = 0
                else:
                    data.Failures += 1
                self.db.set(token, data)
        self.delete_failed()

    def delete_failed(self) -> None:
        with self._mu:
            for t in self.db.token_list():
                data, _ = self.db.get(t)
                if data.Failures > self.error_threshold:
                    log.info("explorer: token %s... removed after %d failures", t[:12], data.Failures)
                    self.db.delete(t)

    def start(self, keep_running: bool = True, stop: Optional[threading.Event] = None,
              idle_sleep: float = 5.0) -> None:
        while stop is None or not stop.is_set():
            if not self.db.token_list():
                time.sleep(idle_sleep)  # nothing to watch yet (discovery.go:44-47)
            else:
                self.run_once()
            if not keep_running:
                return


# ---- HTTP app -------------------------------------------------------------------------------

_PAGE = """<!doctype html><html><head><meta charset='utf-8'><title>{title}</title>
<style>body{{font-family:system-ui,sans-serif;margin:0;background:#0f1115;color:#e6e6e6}}
main{{max-width:980px;margin:1.2em auto;padding:0 1em}}h1{{color:#ff7a45}}
.card{{background:#171a21;border:1px solid #2a2f3a;border-radius:8px;padding:1em;margin:.8em 0}}
input,textarea,button{{background:#1f2430;color:#e6e6e6;border:1px solid #39404f;border-radius:6px;padding:.45em .7em;width:100%;margin:.2em 0}}
button{{cursor:pointer;width:auto}}.muted{{color:#8a93a5;font-size:.9em}}code{{word-break:break-all}}</style></head>
<body><main><h1>LocalAI network explorer</h1><p class='muted'>{version}: deployments and their online workers</p>
<div class='card'><b>Add a network</b>
<input id='name' placeholder='name'><input id='desc' placeholder='description'>
<textarea id='token' placeholder='network token (base64)'></textarea>
<button id='add'>Add</button> <span id='msg' class='muted'></span></div>
<div id='nets'></div></main>
<script>
function el(tag, cls, text){{const e=document.createElement(tag);if(cls)e.className=cls;if(text!==undefined)e.textContent=text;return e;}}
async function refresh(){{
  const r=await fetch('/networks');const nets=await r.json();const root=document.getElementById('nets');root.replaceChildren();
  if(!nets.length){{root.appendChild(el('p','muted','No network with online workers yet.'));return;}}
  for(const n of nets){{const c=el('div','card');c.appendChild(el('b','',n.name));c.appendChild(el('p','muted',n.description));
    for(const cl of n.Clusters){{c.appendChild(el('div','',cl.Type+(cl.NetworkID?' ('+cl.NetworkID+')':'')+': '+cl.Workers.length+' online'));
      for(const w of cl.Workers)c.appendChild(el('div','muted',' - '+w));}}
    const t=el('code','muted',n.token);c.appendChild(t);root.appendChild(c);}}
}}
document.getElementById('add').onclick=async()=>{{
  const body={{name:document.getElementById('name').value,description:document.getElementById('desc').value,token:document.getElementById('token').value.trim()}};
  const r=await fetch('/network/add',{{method:'POST',headers:{{'Content-Type':'application/json'}},body:JSON.stringify(body)}});
  const j=await r.json();document.getElementById('msg').textContent=j.message||j.error;refresh();
}};
refresh();setInterval(refresh,10000);
</script></body></html>"""


def create_explorer_app(db: Database):
    """`core/http/explorer.go:13-45` + `routes/explorer.go:9-13`."""
    from .. import __version__

    app = FastAPI(title="LocalAI explorer")
    title = f"LocalAI API - {__version__}"

    @app.get("/")
    async def dashboard(request: Request):
        accept = request.headers.get("accept", "")
        if request.headers.get("content-type", "") == "application/json" or "html" not in accept:
            return {"Title": title, "Version": __version__}
        return HTMLResponse(_PAGE.format(title=html.escape(title), version=html.escape(__version__)))

    @app.get("/networks")
    async def networks():
        out = []
        for tok in db.token_list():
            data, ok = db.get(tok)
            if ok and any(c.Workers for c in data.Clusters):
                d = asdict(data)
                d["token"] = tok
                out.append(d)
        out.sort(key=lambda d: len(d["Clusters"]), reverse=True)  # most clusters first (dashboard.go:57-60)
        return out

    @app.post("/network/add")
    async def add_network(request: Request):
        try:
            req = await request.json()
            if not isinstance(req, dict):
                raise ValueError
        except ValueError:
            return JSONResponse({"error": "Cannot parse JSON"}, status_code=400)
        token, name, desc = (str(req.get(k) or "") for k in ("token", "name", "description"))
        for v, what in ((token, "Token"), (name, "Name"), (desc, "Description")):
            if not v:
                return JSONResponse({"error": f"{what} is required"}, status_code=400)
        try:
            decode_network_token(token)
        except ValueError:
            return JSONResponse({"error": "Invalid token"}, status_code=400)
        if db.get(token)[1]:
            return JSONResponse({"error": "Token already exists"}, status_code=400)
        try:
            db.set(token, TokenData(name=name, description=desc))
        except OSError:
            return JSONResponse({"error": "Cannot add token"}, status_code=500)
        return {"message": "Token added"}

    return app


def parse_duration(s: str) -> float:
    """Go `time.ParseDuration` subset: "2m", "50s", "1h30m", "500ms", bare seconds."""
    s = s.strip()
    try:
        return float(s)
    except ValueError:
        pass
    units = {"ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}
    total, num = 0.0, ""
    i = 0
    while i < len(s):
        ch = s[i]
        if ch.isdigit() or ch == ".":
            num += ch
            i += 1
            continue
        u = "ms" if s.startswith("ms", i) else ch
        if u not in units or not num:
            raise ValueError(f"invalid duration {s!r}")
        total += float(num) * units[u]
        num = ""
        i += len(u)
    if num:
        raise ValueError(f"invalid duration {s!r}")
    return total

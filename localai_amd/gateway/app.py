"""HTTP application factory (`core/http/app.go`): middleware chain + route registration.

Middleware order mirrors the reference: metrics (api_call histogram) -> API-key auth
(Authorization: Bearer / x-api-key / xi-api-key; GET exemptions) -> CORS -> routes; errors are
`{"error": {"code", "message"}}` JSON, or bare status codes with `opaque_errors`.
"""
from __future__ import annotations

import hmac
import json
import logging
import os
import re
import time
from typing import Optional, Tuple

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response

from ..config.app_config import ApplicationConfig
from ..config.backend_config import BackendConfig
from .openai_routes import APIError
from .state import AppState

log = logging.getLogger("localai_amd.http")


def _extract_key(request: Request) -> str:
    auth = request.headers.get("authorization", "")
    if auth:
        if auth[:7].lower() == "bearer ":
            return auth[7:].strip()
        return ""
    return request.headers.get("x-api-key", "") or request.headers.get("xi-api-key", "")


class AuthMiddleware:
    """API-key check as a plain ASGI middleware (no per-chunk body re-streaming)."""

    def __init__(self, app, state: AppState):
        self.app = app
        self.state = state
        self.exempt = [re.compile(p) for p in state.cfg.http_get_exempted_endpoints]

    def _keys(self):
        # static keys + dynamic api_keys.json (kept current by startup.ConfigWatcher)
        return self.state.cfg.api_keys

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        keys = self._keys()
        if keys:
            cfg = self.state.cfg
            request = Request(scope)
            skip = cfg.disable_api_key_requirement_for_http_get and request.method == "GET" and \
                any(rx.search(request.url.path) for rx in self.exempt)
            if not skip:
                k = _extract_key(request)
                if cfg.use_subtle_key_comparison:
                    good = any(hmac.compare_digest(k.encode(), v.encode()) for v in keys)
                else:
                    good = k in keys
                if not good:
                    resp = Response(status_code=403) if cfg.opaque_errors else \
                        Response("missing or malformed API Key", status_code=403)
                    return await resp(scope, receive, send)
        return await self.app(scope, receive, send)


class CSRFMiddleware:
    """Double-submit CSRF protection behind --csrf / LOCALAI_CSRF (reference:
    core/http/app.go:146-148, fiber's csrf.New() defaults).  A safe request (GET, HEAD, OPTIONS,
    TRACE) is issued a token in the `csrf_` cookie (SameSite=Lax, 1 h); a state-changing request
    must echo that token in the X-Csrf-Token header, and the token must be one this server
    issued and has not expired -- otherwise 403 Forbidden before any handler runs."""

    SAFE = frozenset({"GET", "HEAD", "OPTIONS", "TRACE"})
    COOKIE, HEADER, TTL = "csrf_", "x-csrf-token", 3600.0
    MAX_TOKENS = 65536   # live-token cap: the least recently used token is dropped first

    def __init__(self, app, max_tokens: Optional[int] = None):
        from collections import OrderedDict
        self.app = app
        self.max_tokens = max_tokens or self.MAX_TOKENS
        self.tokens: "OrderedDict[str, float]" = OrderedDict()   # token -> expiry, LRU order

    def _valid(self, tok: str, now: float) -> bool:
        exp = self.tokens.get(tok)
        if exp is None:
            return False
        if exp < now:
            self.tokens.pop(tok, None)
            return False
        return True

    def _touch(self, tok: str, now: float):
        self.tokens[tok] = now + self.TTL
        self.tokens.move_to_end(tok)
        while len(self.tokens) > self.max_tokens:   # bounded under unauthenticated GET floods
            self.tokens.popitem(last=False)

    def _issue(self, now: float) -> str:
        import secrets
        tok = secrets.token_urlsafe(24)
        self._touch(tok, now)
        return tok

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http":
            return await self.app(scope, receive, send)
        request = Request(scope)
        now = time.monotonic()
        cookie = request.cookies.get(self.COOKIE, "")
        if request.method.upper() not in self.SAFE:
            header = request.headers.get(self.HEADER, "")
            if not header or not cookie or not hmac.compare_digest(header, cookie) or not self._valid(cookie, now):
                return await Response("Forbidden", status_code=403)(scope, receive, send)
            return await self.app(scope, receive, send)
        tok = cookie if cookie and self._valid(cookie, now) else self._issue(now)
        self._touch(tok, now)   # a token in use is refreshed
        set_cookie = f"{self.COOKIE}={tok}; Path=/; Max-Age={int(self.TTL)}; SameSite=Lax".encode()

        async def send_wrap(msg):
            if msg["type"] == "http.response.start":
                msg = dict(msg)
                msg["headers"] = list(msg.get("headers", [])) + [(b"set-cookie", set_cookie)]
            await send(msg)
        return await self.app(scope, receive, send_wrap)


class MetricsMiddleware:
    """api_call{method,path} histogram (time to response start, like fiber's middleware)."""

    def __init__(self, app, state: AppState):
        self.app = app
        self.state = state

    async def __call__(self, scope, receive, send):
        if scope["type"] != "http" or scope.get("path") == "/metrics":
            return await self.app(scope, receive, send)
        t0 = time.perf_counter()
        done = False

        async def send_wrap(msg):
            nonlocal done
            if not done and msg["type"] == "http.response.start":
                done = True
                self.state.metrics.api_call.labels(scope["method"], scope["path"]).observe(time.perf_counter() - t0)
            await send(msg)
        return await self.app(scope, receive, send_wrap)


def create_app(state: AppState) -> FastAPI:
    from contextlib import asynccontextmanager

    cfg = state.cfg
    p2p_node = None
    if cfg.p2p:
        from .p2p import P2PNode, advertise_url
        p2p_node = P2PNode(cfg.p2p_token, cfg.p2p_network_id, advertise_url(cfg.address))
        cfg.p2p_token = p2p_node.token  # a generated token is what /api/p2p/token serves

    @asynccontextmanager
    async def lifespan(app):
        state.manager.start_watchdog()
        if p2p_node is not None:
            p2p_node.start()
        yield
        if p2p_node is not None:
            p2p_node.stop()
        await state.manager.stop_all()

    app = FastAPI(title="LocalAI (MI355X)", lifespan=lifespan, docs_url="/swagger", openapi_url="/swagger/doc.json")

    @app.exception_handler(APIError)
    async def _api_err(request: Request, e: APIError):
        if cfg.opaque_errors:
            return Response(status_code=e.code)
        return JSONResponse({"error": {"code": e.code, "message": str(e), "type": ""}}, status_code=e.code)

    @app.exception_handler(Exception)
    async def _err(request: Request, e: Exception):
        log.exception("request failed: %s %s", request.method, request.url.path)
        if cfg.opaque_errors:
            return Response(status_code=500)
        return JSONResponse({"error": {"code": 500, "message": str(e), "type": ""}}, status_code=500)

    if not cfg.disable_metrics:
        app.add_middleware(MetricsMiddleware, state=state)
    app.add_middleware(AuthMiddleware, state=state)
    if cfg.csrf:
        log.debug("CSRF middleware enabled: state-changing requests need the X-Csrf-Token header")
        app.add_middleware(CSRFMiddleware)
    if cfg.cors:
        from starlette.middleware.cors import CORSMiddleware
        origins = [o for o in cfg.cors_allow_origins.split(",") if o] or ["*"]
        app.add_middleware(CORSMiddleware, allow_origins=origins, allow_methods=["*"], allow_headers=["*"])

    from . import openai_routes, localai_routes, files_routes, gallery_routes, p2p, webui
    oai = openai_routes.build_router(state)
    app.include_router(oai)
    app.include_router(files_routes.build_router(state))
    app.include_router(localai_routes.build_router(state))
    app.include_router(webui.build_router(state))
    app.include_router(p2p.build_router(p2p_node))
    if not cfg.disable_gallery_endpoint:
        app.include_router(gallery_routes.build_router(state))
    app.state.localai = state
    app.state.p2p = p2p_node
    # the streaming chat / completion routes on the native server skip Starlette's middleware
    # stack, router and FastAPI's endpoint wrapper (~0.25 of ~0.85 ms of gateway CPU per
    # request, scripts/gateway_profile.py): the same auth and metrics middleware and the same
    # exception handlers, composed around the endpoint.  Not with CSRF / CORS (stateful or
    # response-rewriting middleware stays on the one regular stack).
    if not (cfg.csrf or cfg.cors):
        fast = {}
        for path, ep in oai.native_fast.items():
            h = _FastEndpoint(ep, _api_err, _err)
            if not cfg.disable_metrics:
                h = MetricsMiddleware(h, state=state)
            fast[path] = AuthMiddleware(h, state=state)
        app.state.native_fast = fast
    return app


class _FastEndpoint:
    """ASGI app for an endpoint taking only the Request (see create_app: native_fast)."""

    def __init__(self, endpoint, api_err, err):
        self.endpoint, self.api_err, self.err = endpoint, api_err, err

    async def __call__(self, scope, receive, send):
        from starlette.exceptions import HTTPException
        request = Request(scope, receive)
        try:
            resp = await self.endpoint(request)
        except APIError as e:
            resp = await self.api_err(request, e)
        except HTTPException as e:
            from fastapi.exception_handlers import http_exception_handler
            resp = await http_exception_handler(request, e)
        except Exception as e:  # noqa: BLE001 - same catch-all as the app's handler
            resp = await self.err(request, e)
        if not isinstance(resp, Response):
            from fastapi.encoders import jsonable_encoder
            resp = JSONResponse(jsonable_encoder(resp))
        await resp(scope, receive, send)


LLAMA3_CHAT_MESSAGE = ("<|start_header_id|>{{ .RoleName }}<|end_header_id|>\n\n{{.Content }}<|eot_id|>")
LLAMA3_CHAT = "<|begin_of_text|>{{.Input }}\n<|start_header_id|>assistant<|end_header_id|>"


def create_app_for_engine(engine, name: str = "llama3-8b-instruct", models_path: Optional[str] = None,
                          app_config: Optional[ApplicationConfig] = None,
                          replicas: Optional[list] = None) -> Tuple[FastAPI, str]:
    """Serve an already-constructed LLMEngine under `name` (bench / embedding use).

    The model config is the one the reference's guesser produces for a Llama-3 GGUF
    (core/config/guesser.go LLaMa3 defaults), with mirostat disabled so the sampler chain is the
    plain top-k/top-p/temperature one."""
    import tempfile
    from ..grpc.rpc import EmbeddedBackend
    from ..grpc.servicer import EngineServicer
    from ..grpc import backend_pb as pb

    ac = app_config or ApplicationConfig()
    ac.models_path = models_path or tempfile.mkdtemp(prefix="localai_models_")
    state = AppState(ac)
    sv = EngineServicer(device=str(engine.device))
    sv.engine = engine
    sv.model_name = name
    sv.state = pb.StatusResponse.READY
    handle = EmbeddedBackend(sv)
    if replicas:
        # data-parallel replicas behind the one handle (this engine first, then the remote ones)
        from ..parallel.replicas import ReplicaBackend
        handle = ReplicaBackend([handle] + list(replicas), ["embedded"] + [r.addr for r in replicas])
    state.manager.register(name, "localai-amd" if not replicas else f"localai-amd-dp{1 + len(replicas)}", handle,
                           servicer=sv)
    bc = BackendConfig({
        "name": name, "backend": "localai-amd", "context_size": engine.cfg.context_size, "mirostat": 0,
        "parameters": {"model": os.path.basename(engine.cfg.model_path), "temperature": 0.8, "top_k": 40,
                       "top_p": 0.95},
        "template": {"chat_message": LLAMA3_CHAT_MESSAGE, "chat": LLAMA3_CHAT},
        "stopwords": ["<|eot_id|>"],
    })
    bc.set_defaults()
    state.configs.add(bc)
    app = create_app(state)
    app.state.bench_handle = handle
    return app, name

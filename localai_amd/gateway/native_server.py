"""Serve the ASGI gateway app on the native HTTP/1.1 server (native/http_server.cpp).

The C++ side owns sockets and HTTP parsing; this module turns each parsed request into an
ASGI `http` scope, runs the FastAPI app on the asyncio loop, and maps `send()` events onto
`respond` / `stream_start` / `stream_write` / `stream_end`.  Routes that can stream tokens
natively find `scope["localai.native"] = (server, conn_id)` and bind an SseSink to the
connection so tokens never pass through the event loop (see openai_routes._native_stream).
"""
from __future__ import annotations

import asyncio
import logging
from typing import Optional
from urllib.parse import unquote

from starlette.responses import Response

log = logging.getLogger("localai_amd.http")



class NativeConn:
    """Handle a route uses to take over the connection (set `handled` when it does)."""
    __slots__ = ("srv", "conn", "handled")

    def __init__(self, srv, conn):
        self.srv, self.conn, self.handled = srv, conn, False


class NativeHandledResponse(Response):
    """ASGI response meaning 'a native sink owns this connection now' (sends nothing)."""

    def __init__(self):
        super().__init__(status_code=200)

    async def __call__(self, scope, receive, send):
        return None


class NativeHTTPServer:
    def __init__(self, app, host: str = "0.0.0.0", port: int = 8080):
        from ..native import http
        self.app = app
        # exact-path POST routes the app serves without its router (gateway/app.py native_fast)
        self.fast = dict(getattr(getattr(app, "state", None), "native_fast", None) or {})
        self.srv = http().Server(host, int(port))
        self.host = host
        self.port = self.srv.port
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self._stop: Optional[asyncio.Event] = None
        self.started = False
        self._lifespan_q: Optional[asyncio.Queue] = None
        import atexit
        atexit.register(self.srv.stop)  # join the I/O thread before interpreter teardown

    # ------------------------------------------------------------------ lifecycle
    async def _lifespan(self, phase: str):
        if self._lifespan_q is None:
            self._lifespan_q = asyncio.Queue()
            self._lifespan_done = asyncio.Queue()
            scope = {"type": "lifespan", "asgi": {"version": "3.0"}, "state": {}}

            async def receive():
                return await self._lifespan_q.get()

            async def send(msg):
                await self._lifespan_done.put(msg)

            async def run():
                try:
                    await self.app(scope, receive, send)
                except Exception:  # app without lifespan support
                    await self._lifespan_done.put({"type": "lifespan.unsupported"})
            self._lifespan_task = asyncio.get_running_loop().create_task(run())
        await self._lifespan_q.put({"type": f"lifespan.{phase}"})
        msg = await self._lifespan_done.get()
        if msg["type"].endswith(".failed"):
            raise RuntimeError(msg.get("message", f"lifespan {phase} failed"))

    async def serve(self):
        self.loop = asyncio.get_running_loop()
        self._stop = asyncio.Event()
        await self._lifespan("startup")
        self.loop.add_reader(self.srv.notify_fd, self._on_ready)
        self.srv.start()
        self.started = True
        try:
            await self._stop.wait()
        finally:
            self.loop.remove_reader(self.srv.notify_fd)
            await self._lifespan("shutdown")
            self.srv.stop()

    def run(self):
        asyncio.run(self.serve())

    def shutdown(self):
        if self.loop is not None and self._stop is not None:
            self.loop.call_soon_threadsafe(self._stop.set)

    # ------------------------------------------------------------------ requests
    def _on_ready(self):
        for req in self.srv.take_requests():
            self.loop.create_task(self._handle(*req))

    async def _handle(self, conn, method, target, version, headers, body, peer):
        srv = self.srv
        path, _, query = target.partition(b"?")
        host, _, cport = peer.rpartition(":")
        scope = {
            "type": "http", "asgi": {"version": "3.0", "spec_version": "2.3"},
            "http_version": version.split("/")[-1] if "/" in version else "1.1",
            "method": method, "scheme": "http", "path": unquote(path.decode("latin-1")), "raw_path": path,
            "query_string": query, "root_path": "", "headers": headers,
            "client": (host, int(cport or 0)), "server": (self.host, self.port),
            "localai.native": NativeConn(srv, conn),
        }
        sent_body = [False]
        st = {"status": 200, "headers": [], "streaming": False, "done": False}

        async def receive():
            if not sent_body[0]:
                sent_body[0] = True
                return {"type": "http.request", "body": body, "more_body": False}
            while srv.is_open(conn) and not st["done"]:
                await asyncio.sleep(0.25)
            return {"type": "http.disconnect"}

        def hdrs(raw):
            return [(k.decode("latin-1"), v.decode("latin-1")) for k, v in raw]

        async def send(msg):
            t = msg["type"]
            if t == "http.response.start":
                st["status"] = msg["status"]
                st["headers"] = hdrs(msg.get("headers", []))
            elif t == "http.response.body":
                data = msg.get("body", b"")
                more = msg.get("more_body", False)
                if st["done"]:
                    return
                if not st["streaming"]:
                    if not more:
                        st["done"] = True
                        srv.respond(conn, st["status"], st["headers"], data)
                        return
                    st["streaming"] = True
                    srv.stream_start(conn, st["status"], st["headers"])
                if more:
                    if data and not srv.stream_write(conn, data):
                        raise ConnectionResetError("client disconnected")
                else:
                    st["done"] = True
                    srv.stream_end(conn, data)

        fast = self.fast.get(scope["path"]) if method == "POST" and self.fast else None
        if fast is not None:
            scope["app"] = self.app
        try:
            await (fast or self.app)(scope, receive, send)
        except Exception:
            log.exception("unhandled error serving %s %s", method, path)
            if not st["streaming"] and not st["done"]:
                st["done"] = True
                srv.respond(conn, 500, [("content-type", "application/json")],
                            b'{"error":{"code":500,"message":"internal error","type":""}}')
        if not st["done"] and not scope["localai.native"].handled:
            # app returned without a complete response
            if st["streaming"]:
                srv.stream_end(conn, b"")
            else:
                srv.respond(conn, 500, [], b"")

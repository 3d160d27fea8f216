"""gRPC transport for the backend contract: an asyncio server exposing any servicer object
(methods named like the RPCs) and a client with ONE persistent channel per backend (the
reference dials a new connection per call)."""
from __future__ import annotations

import asyncio
import logging
from typing import AsyncIterator, Optional

import grpc

from . import backend_pb as pb

log = logging.getLogger("localai_amd.grpc")
MAX_MSG = 64 * 1024 * 1024
_OPTS = [("grpc.max_send_message_length", MAX_MSG), ("grpc.max_receive_message_length", MAX_MSG)]


def _handler(servicer, rpc, req, resp, stream):
    impl = getattr(servicer, rpc, None)
    des = pb.M[req].FromString
    ser = pb.M[resp].SerializeToString

    if stream:
        async def call(request, context):
            try:
                async for r in impl(request, context):
                    yield r
            except NotImplementedError as e:
                await context.abort(grpc.StatusCode.UNIMPLEMENTED, str(e))
        return grpc.unary_stream_rpc_method_handler(call, request_deserializer=des, response_serializer=ser)

    async def call(request, context):
        if impl is None:
            await context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{rpc} not implemented")
        try:
            return await impl(request, context)
        except Exception as e:
            if type(e).__name__ == "Unimplemented":
                await context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{rpc} not implemented")
            if isinstance(e, grpc.aio.AbortError):
                raise
            log.exception("%s failed", rpc)
            await context.abort(grpc.StatusCode.INTERNAL, str(e))
    return grpc.unary_unary_rpc_method_handler(call, request_deserializer=des, response_serializer=ser)


async def serve(servicer, addr: str, max_workers: int = 0) -> grpc.aio.Server:
    server = grpc.aio.server(options=_OPTS)
    handlers = {rpc: _handler(servicer, rpc, req, resp, stream) for rpc, req, resp, stream in pb.RPCS}
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(pb.SERVICE, handlers),))
    server.add_insecure_port(addr)
    await server.start()
    return server


class GRPCBackend:
    """Client side of backend.proto (persistent channel)."""

    def __init__(self, addr: str):
        self.addr = addr
        self.channel = None
        self._calls = {}
        self._loop = None
        try:
            asyncio.get_running_loop()
            self._connect()
        except RuntimeError:
            pass  # built outside an event loop: connect on first use, on the loop that uses it

    def _connect(self):
        # a grpc.aio channel belongs to the event loop it was created on
        self._loop = asyncio.get_running_loop()
        self.channel = grpc.aio.insecure_channel(self.addr, options=_OPTS)
        self._calls = {}
        for rpc, req, resp, stream in pb.RPCS:
            mk = self.channel.unary_stream if stream else self.channel.unary_unary
            self._calls[rpc] = mk(pb.method_path(rpc), request_serializer=pb.M[req].SerializeToString,
                                  response_deserializer=pb.M[resp].FromString)

    def __getattr__(self, rpc):
        if any(r == rpc for r, _, _, _ in pb.RPCS):
            if self.__dict__.get("channel") is None:
                self._connect()
            return self.__dict__["_calls"][rpc]
        raise AttributeError(rpc)

    async def health(self, timeout: float = 5.0) -> bool:
        try:
            r = await self.Health(pb.HealthMessage(), timeout=timeout)
            return r.message == b"OK"
        except Exception:
            return False

    async def close(self):
        if self.channel is not None:
            await self.channel.close()


class EmbeddedBackend:
    """In-process backend: calls the servicer directly (no sockets, no serialisation)."""

    def __init__(self, servicer):
        self.servicer = servicer
        self.addr = "embedded"

    def __getattr__(self, rpc):
        impl = getattr(self.__dict__["servicer"], rpc, None)
        if impl is None:
            raise AttributeError(rpc)
        stream = any(r == rpc and s for r, _, _, s in pb.RPCS)
        if stream:
            def call_stream(request, timeout=None):
                return impl(request, None)
            return call_stream

        async def call(request, timeout=None):
            return await impl(request, None)
        return call

    async def health(self, timeout: float = 5.0) -> bool:
        res = await self.servicer.Health(pb.HealthMessage(), None)
        return res.message == b"OK"

    async def close(self):
        pass

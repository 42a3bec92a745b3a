"""Generic grpc.aio server binding for the runtime-built service descriptors.

A service implementation is any object with `async def <Method>(self, request, context)` for
unary RPCs, or an async generator for server-streaming ones (e.g. AIRuntime.StreamInfer).
Missing methods answer UNIMPLEMENTED, like tonic's generated defaults.
"""
from __future__ import annotations

import asyncio
import logging
from typing import Dict, Iterable, Optional

import grpc

from .schema import message, service

log = logging.getLogger("aios.rpc")


def _handler(impl, md):
    req_cls = message(md.input_type.full_name)
    resp_cls = message(md.output_type.full_name)
    fn = getattr(impl, md.name, None)

    if md.server_streaming:
        async def stream(request, context):
            if fn is None:
                await context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{md.name} not implemented")
            async for item in fn(request, context):
                yield item

        return grpc.unary_stream_rpc_method_handler(stream, request_deserializer=req_cls.FromString,
                                                    response_serializer=resp_cls.SerializeToString)

    async def unary(request, context):
        if fn is None:
            await context.abort(grpc.StatusCode.UNIMPLEMENTED, f"{md.name} not implemented")
        resp = await fn(request, context)
        if resp is None:
            resp = resp_cls()
        return resp

    return grpc.unary_unary_rpc_method_handler(unary, request_deserializer=req_cls.FromString,
                                               response_serializer=resp_cls.SerializeToString)


def generic_handler(full_service_name: str, impl) -> grpc.GenericRpcHandler:
    sd = service(full_service_name)
    handlers = {md.name: _handler(impl, md) for md in sd.methods}
    return grpc.method_handlers_generic_handler(full_service_name, handlers)


def server_credentials(tls_dir: Optional[str] = None):
    """mTLS for every service when AIOS_TLS_DIR (or tls_dir) holds the node certificates made by the
    native TlsManager (agent-core/src/tls.rs -- generated but never used in the reference, whose
    gRPC is plaintext everywhere).  Clients must present a certificate signed by the node CA
    unless AIOS_TLS_CLIENT_AUTH=0.  Returns None for plaintext."""
    import os

    d = tls_dir if tls_dir is not None else os.environ.get("AIOS_TLS_DIR", "")
    if not d:
        return None
    from ..core import load as load_core

    mgr = load_core().TlsManager(d)
    mgr.generate_self_signed(os.environ.get("AIOS_TLS_SERVICE", "aios"))  # idempotent
    p = mgr.paths()
    read = lambda k: open(p[k], "rb").read()  # noqa: E731
    return grpc.ssl_server_credentials([(read("server_key"), read("server_cert"))], root_certificates=read("ca_cert"),
                                       require_client_auth=os.environ.get("AIOS_TLS_CLIENT_AUTH", "1") != "0")


class RpcServer:
    """grpc.aio server hosting one or more aiOS services on one address."""

    def __init__(self, address: str, services: Dict[str, object], options: Optional[Iterable] = None,
                 tls_dir: Optional[str] = None):
        self.address = address
        self.services = services
        self.server = grpc.aio.server(options=list(options or [
            ("grpc.max_receive_message_length", 64 * 1024 * 1024),
            ("grpc.max_send_message_length", 64 * 1024 * 1024),
        ]))
        for name, impl in services.items():
            self.server.add_generic_rpc_handlers((generic_handler(name, impl),))
        creds = server_credentials(tls_dir)
        self.tls = creds is not None
        self.port = self.server.add_secure_port(address, creds) if creds else self.server.add_insecure_port(address)
        if self.port == 0:
            raise RuntimeError(f"could not bind {address}")

    async def start(self):
        await self.server.start()
        log.info("serving %s on %s (port %d)", ", ".join(self.services), self.address, self.port)
        return self

    async def stop(self, grace: float = 1.0):
        await self.server.stop(grace)

    async def wait(self):
        await self.server.wait_for_termination()


async def serve_forever(address: str, services: Dict[str, object], stop_event: Optional[asyncio.Event] = None):
    srv = RpcServer(address, services)
    await srv.start()
    if stop_event is None:
        await srv.wait()
    else:
        await stop_event.wait()
        await srv.stop()
    return srv

"""Typed grpc.aio client stubs built from the runtime descriptors.

    stub = Stub(channel("127.0.0.1:50055"), "aios.runtime.AIRuntime")
    resp = await stub.Infer(pb.runtime.InferRequest(prompt="hi"), timeout=30)

Mirrors the reference's lazily-connected service clients (`agent-core/src/clients.rs:17-146`):
channels are created on first use, with keepalive, and calls default to a 300 s deadline.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import grpc

from .schema import SERVICES, message, service

DEFAULT_TIMEOUT = 300.0
_channels: Dict[str, grpc.aio.Channel] = {}


def channel_credentials(tls_dir: Optional[str] = None):
    """Client side of the node mTLS (see rpc.server.server_credentials): CA + this node's cert."""
    d = tls_dir if tls_dir is not None else os.environ.get("AIOS_TLS_DIR", "")
    if not d:
        return None
    p = {k: os.path.join(d, f) for k, f in (("ca", "ca.crt"), ("cert", "server.crt"), ("key", "server.key"))}
    read = lambda k: open(p[k], "rb").read()  # noqa: E731
    return grpc.ssl_channel_credentials(root_certificates=read("ca"), private_key=read("key"),
                                        certificate_chain=read("cert"))


def channel(address: str, fresh: bool = False, tls_dir: Optional[str] = None) -> grpc.aio.Channel:
    if fresh or address not in _channels:
        opts = [
            ("grpc.keepalive_time_ms", 10_000),
            ("grpc.keepalive_timeout_ms", 5_000),
            ("grpc.max_receive_message_length", 64 * 1024 * 1024),
        ]
        creds = channel_credentials(tls_dir)
        if creds is not None:
            # certificates carry SAN localhost / 127.0.0.1 / the service name
            opts.append(("grpc.ssl_target_name_override", os.environ.get("AIOS_TLS_SERVICE", "aios")))
            ch = grpc.aio.secure_channel(address, creds, options=opts)
        else:
            ch = grpc.aio.insecure_channel(address, options=opts)
        if fresh:
            return ch
        _channels[address] = ch
    return _channels[address]


async def close_all():
    for ch in list(_channels.values()):
        await ch.close()
    _channels.clear()


class Stub:
    def __init__(self, ch: grpc.aio.Channel, full_service_name: str, timeout: float = DEFAULT_TIMEOUT):
        self._sd = service(full_service_name)
        self._timeout = timeout
        for md in self._sd.methods:
            path = f"/{full_service_name}/{md.name}"
            req = message(md.input_type.full_name)
            resp = message(md.output_type.full_name)
            if md.server_streaming:
                call = ch.unary_stream(path, request_serializer=req.SerializeToString,
                                       response_deserializer=resp.FromString)
            else:
                call = ch.unary_unary(path, request_serializer=req.SerializeToString,
                                      response_deserializer=resp.FromString)
            setattr(self, md.name, self._wrap(call, md.server_streaming))

    def _wrap(self, call, streaming):
        default = self._timeout

        if streaming:
            def s(request, timeout: Optional[float] = None, **kw):
                return call(request, timeout=timeout or default, **kw)
            return s

        async def u(request, timeout: Optional[float] = None, **kw):
            return await call(request, timeout=timeout or default, **kw)
        return u


def default_address(full_service_name: str, host: str = "127.0.0.1") -> str:
    return f"{host}:{SERVICES[full_service_name]}"

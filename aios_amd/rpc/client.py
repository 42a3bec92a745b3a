"""Typed grpc.aio client stubs built from the runtime descriptors.

    stub = Stub(channel("127.0.0.1:50055"), "aios.runtime.AIRuntime")
    resp = await stub.Infer(pb.runtime.InferRequest(prompt="hi"), timeout=30)

Mirrors the reference's lazily-connected service clients (`agent-core/src/clients.rs:17-146`):
channels are created on first use, with keepalive, and calls default to a 300 s deadline.
"""
from __future__ import annotations

from typing import Dict, Optional

import grpc

from .schema import SERVICES, message, service

DEFAULT_TIMEOUT = 300.0
_channels: Dict[str, grpc.aio.Channel] = {}


def channel(address: str, fresh: bool = False) -> grpc.aio.Channel:
    if fresh or address not in _channels:
        ch = grpc.aio.insecure_channel(address, options=[
            ("grpc.keepalive_time_ms", 10_000),
            ("grpc.keepalive_timeout_ms", 5_000),
            ("grpc.max_receive_message_length", 64 * 1024 * 1024),
        ])
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

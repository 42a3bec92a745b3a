"""Leader -> worker command channel for the TP tier inside long-running servers.

The runtime daemon hosts several models and must not own a torch.distributed default group per
TP model, so the strategic tier's control plane is a loopback TCP fan-out: the leader (rank 0, in
the runtime process) accepts one connection per worker rank and broadcasts each engine command
once per call; at startup it gathers the workers' IPC handles.  Data never travels here --
partial sums move over xGMI inside the HIP all-reduce.

Safety: messages are JSON (bytes as tagged base64) -- nothing on this socket is ever executed or
unpickled; a worker must present the per-launch random token before it is accepted (constant-time
compare), and workers only dispatch to a fixed whitelist of engine methods (tp.py).
"""
from __future__ import annotations

import base64
import hmac
import json
import secrets
import socket
import struct
from typing import Any, List, Optional

_HDR = struct.Struct("!Q")
MAX_MSG = 256 << 20


def _enc(o: Any) -> Any:
    if isinstance(o, (bytes, bytearray)):
        return {"__b64__": base64.b64encode(bytes(o)).decode()}
    if isinstance(o, (list, tuple)):
        return [_enc(x) for x in o]
    if isinstance(o, dict):
        return {str(k): _enc(v) for k, v in o.items()}
    return o


def _dec(o: Any) -> Any:
    if isinstance(o, dict):
        if set(o) == {"__b64__"}:
            return base64.b64decode(o["__b64__"])
        return {k: _dec(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_dec(x) for x in o]
    return o


def pack(obj: Any) -> bytes:
    data = json.dumps(_enc(obj), separators=(",", ":")).encode()
    return _HDR.pack(len(data)) + data


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("TP channel closed")
        buf += chunk
    return bytes(buf)


def recv_msg(sock: socket.socket) -> Any:
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    if n > MAX_MSG:
        raise ValueError("TP channel message too large")
    return _dec(json.loads(_recv_exact(sock, n)))


class LeaderChannel:
    def __init__(self, world: int, host: str = "127.0.0.1", port: int = 0, timeout: float = 600.0):
        self.world = world
        self.token = secrets.token_hex(16)
        self.srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.srv.bind((host, port))
        self.srv.listen(world)
        self.srv.settimeout(timeout)
        self.address = f"{host}:{self.srv.getsockname()[1]}"
        self.peers: List[Optional[socket.socket]] = [None] * world

    def accept_all(self):
        while any(p is None for p in self.peers[1:]):
            s, _ = self.srv.accept()
            s.settimeout(30)
            try:
                hello = recv_msg(s)
                rank, tok = int(hello["rank"]), str(hello["token"])
            except Exception:
                s.close()
                continue
            if not hmac.compare_digest(tok, self.token) or not 0 < rank < self.world or self.peers[rank]:
                s.close()
                continue
            s.settimeout(None)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.peers[rank] = s

    def gather(self, mine: Any) -> List[Any]:
        out = [mine] + [None] * (self.world - 1)
        for r in range(1, self.world):
            out[r] = recv_msg(self.peers[r])
        return out

    def broadcast(self, obj: Any):
        msg = pack(obj)
        for s in self.peers[1:]:
            s.sendall(msg)

    def close(self):
        for s in self.peers[1:]:
            if s is not None:
                s.close()
        self.srv.close()


class WorkerChannel:
    def __init__(self, address: str, rank: int, token: str, timeout: float = 600.0):
        host, port = address.rsplit(":", 1)
        self.sock = socket.create_connection((host, int(port)), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.sock.settimeout(None)
        self.rank = rank
        self.sock.sendall(pack({"rank": rank, "token": token}))

    def send(self, obj: Any):
        self.sock.sendall(pack(obj))

    def recv(self) -> Any:
        return recv_msg(self.sock)

    def close(self):
        self.sock.close()

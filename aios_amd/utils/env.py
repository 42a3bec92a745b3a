"""Service addresses, data paths and env helpers shared by the daemons.

Ports follow the code of the reference, not its README: orchestrator 50051,
tools 50052, memory 50053, api-gateway 50054, runtime 50055, management console 9090.
"""
from __future__ import annotations

import logging
import os

DEFAULT_ADDRS = {
    "orchestrator": ("AIOS_ORCHESTRATOR_ADDR", "127.0.0.1:50051"),
    "tools": ("AIOS_TOOLS_ADDR", "127.0.0.1:50052"),
    "memory": ("AIOS_MEMORY_ADDR", "127.0.0.1:50053"),
    "api-gateway": ("AIOS_API_GATEWAY_ADDR", "127.0.0.1:50054"),
    "runtime": ("AIOS_RUNTIME_ADDR", "127.0.0.1:50055"),
}


def addr(service: str) -> str:
    env, default = DEFAULT_ADDRS[service]
    a = os.environ.get(env, default)
    for p in ("http://", "https://"):
        if a.startswith(p):
            a = a[len(p):]
    if a.startswith("[::]") or a.startswith("0.0.0.0"):
        a = "127.0.0.1" + a[a.rfind(":"):]
    return a


def listen_addr(service: str, port: int) -> str:
    env = {"orchestrator": "AIOS_ORCHESTRATOR_LISTEN", "tools": "AIOS_TOOLS_LISTEN",
           "memory": "AIOS_MEMORY_LISTEN", "api-gateway": "AIOS_API_GATEWAY_LISTEN"}.get(service, "")
    return os.environ.get(env, f"0.0.0.0:{port}") if env else f"0.0.0.0:{port}"


def data_dir() -> str:
    return os.environ.get("AIOS_DATA_DIR", "/var/lib/aios")


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.strip().lower() in ("1", "true", "yes", "on")


def setup_logging(name: str):
    logging.basicConfig(level=os.environ.get("AIOS_LOG", "INFO"),
                        format=f"%(asctime)s %(levelname)s {name} %(name)s: %(message)s")
    return logging.getLogger(name)

"""aios-tools daemon: `aios.tools.ToolRegistry` on :50052 over the native tool core.

Reference: `tools/src/main.rs` (ListTools/GetTool/Execute/Rollback/Register/Deregister,
`:40-301`), with the execution pipeline -- validate, capability check, rate limit, backup,
handler, audit -- living in C++ (`aios_amd/native/tools_core.cpp`).  Execution releases the GIL
and runs on a thread pool, so slow tools (network, package managers, sandboxed plugins) never
block the event loop and independent calls overlap (the reference held one Mutex across every
Execute, `main.rs:103`).

Differences from the reference, on purpose:
* externally registered tools (`Register` with a `handler_address`) are executed by forwarding
  the ExecuteRequest to the ToolRegistry at that address (the reference stored the address and
  never used it), after the local capability check;
* a plugin scan every 30 s picks up plugins written by other processes.
"""
from __future__ import annotations

import argparse
import asyncio
import concurrent.futures as cf
import json
import logging
import os
import signal
from typing import Optional

import grpc

from ..core import load as load_core
from ..rpc.client import Stub, channel
from ..rpc.schema import pb
from ..rpc.server import RpcServer
from ..utils.env import data_dir, setup_logging

log = logging.getLogger("aios.tools")
PLUGIN_SCAN_INTERVAL = 30.0


def tooldef_to_pb(d: dict):
    return pb.tools.ToolDefinition(
        name=d["name"], namespace=d["namespace"], version=d["version"], description=d["description"],
        required_capabilities=d["required_capabilities"], risk_level=d["risk_level"],
        requires_confirmation=d["requires_confirmation"], idempotent=d["idempotent"],
        reversible=d["reversible"], timeout_ms=d["timeout_ms"], rollback_tool=d["rollback_tool"])


class ToolRegistryService:
    def __init__(self, data: Optional[str] = None, source_dir: str = "", workers: int = 16):
        core = load_core()
        self.data_dir = data or data_dir()
        os.makedirs(self.data_dir, exist_ok=True)
        self.core = core.ToolService(self.data_dir, source_dir or os.environ.get("AIOS_SOURCE_DIR", ""))
        self.pool = cf.ThreadPoolExecutor(max_workers=workers, thread_name_prefix="tool")
        log.info("tool registry: %d tools (data dir %s)", self.core.tool_count(), self.data_dir)

    async def _run(self, fn, *args):
        return await asyncio.get_running_loop().run_in_executor(self.pool, fn, *args)

    # ---------------------------------------------------------------- RPCs
    async def ListTools(self, req, ctx):
        return pb.tools.ListToolsResponse(tools=[tooldef_to_pb(d) for d in self.core.list_tools(req.namespace)])

    async def GetTool(self, req, ctx):
        d = self.core.get_tool(req.name)
        if d is None:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"Tool not found: {req.name}")
        return tooldef_to_pb(d)

    async def Execute(self, req, ctx):
        d = self.core.get_tool(req.tool_name)
        if d is not None and d["handler_address"]:
            return await self._forward(req, d)
        r = await self._run(self.core.execute, req.tool_name, req.agent_id, req.task_id,
                            req.input_json or b"{}", req.reason)
        if not r["success"]:
            log.info("tool %s (agent %s) failed: %s", req.tool_name, req.agent_id, r["error"])
        return pb.tools.ExecuteResponse(success=r["success"], output_json=r["output_json"], error=r["error"],
                                        execution_id=r["execution_id"], duration_ms=r["duration_ms"],
                                        backup_id=r["backup_id"])

    async def _forward(self, req, d):
        chk = self.core.check(req.agent_id, req.tool_name)
        if not chk["allowed"]:
            return pb.tools.ExecuteResponse(success=False, error=f"Capability denied: {chk['reason']}")
        try:
            stub = Stub(channel(d["handler_address"]), "aios.tools.ToolRegistry")
            return await stub.Execute(req, timeout=max(1.0, d["timeout_ms"] / 1000.0))
        except grpc.aio.AioRpcError as e:
            return pb.tools.ExecuteResponse(success=False, error=f"remote handler {d['handler_address']}: {e.details()}")

    async def Rollback(self, req, ctx):
        ok, err = await self._run(self.core.rollback, req.execution_id)
        return pb.tools.RollbackResponse(success=ok, error=err)

    async def Register(self, req, ctx):
        if not req.HasField("tool"):
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "Missing tool definition")
        t = req.tool
        ok, err = self.core.register_tool({
            "name": t.name, "namespace": t.namespace or t.name.split(".")[0], "version": t.version or "1.0.0",
            "description": t.description, "required_capabilities": list(t.required_capabilities),
            "risk_level": t.risk_level or "medium", "requires_confirmation": t.requires_confirmation,
            "idempotent": t.idempotent, "reversible": t.reversible, "timeout_ms": t.timeout_ms or 30000,
            "rollback_tool": t.rollback_tool, "handler_address": req.handler_address})
        log.info("register %s -> %s (%s)", t.name, req.handler_address or "local", "ok" if ok else err)
        return pb.tools.RegisterToolResponse(accepted=ok, error=err)

    async def Deregister(self, req, ctx):
        ok = self.core.deregister_tool(req.tool_name)
        return pb.tools.Status(success=ok, message=f"Tool {req.tool_name} " + ("deregistered" if ok else "not found"))

    # ---------------------------------------------------------------- background
    async def plugin_scan_loop(self, stop: asyncio.Event):
        while not stop.is_set():
            try:
                n = await self._run(self.core.scan_plugins)
                if n:
                    log.info("plugin scan registered %d new plugin tools", n)
            except Exception as e:  # pragma: no cover - defensive
                log.warning("plugin scan failed: %s", e)
            try:
                await asyncio.wait_for(stop.wait(), PLUGIN_SCAN_INTERVAL)
            except asyncio.TimeoutError:
                pass

    def close(self):
        self.pool.shutdown(wait=False, cancel_futures=True)


async def amain(args):
    svc = ToolRegistryService(args.data_dir, args.source_dir)
    server = RpcServer(args.addr, {"aios.tools.ToolRegistry": svc})
    await server.start()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except NotImplementedError:
            pass
    await svc.plugin_scan_loop(stop)
    await server.stop()
    svc.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description="aiOS tool registry (aios.tools.ToolRegistry)")
    ap.add_argument("--addr", default=os.environ.get("AIOS_TOOLS_LISTEN", "0.0.0.0:50052"))
    ap.add_argument("--data-dir", default=data_dir())
    ap.add_argument("--source-dir", default=os.environ.get("AIOS_SOURCE_DIR", ""))
    args = ap.parse_args(argv)
    setup_logging("aios-tools")
    asyncio.run(amain(args))


if __name__ == "__main__":
    main()

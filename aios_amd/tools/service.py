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
import time
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
        reversible=d["reversible"], timeout_ms=d["timeout_ms"], rollback_tool=d["rollback_tool"],
        input_schema=d.get("input_schema", "").encode())


class PluginRuntime:
    """Hot reload + trigger dispatch for AI-authored plugins (one `tick()` per scan interval)."""

    def __init__(self, core_svc, data: str, triggers_db: Optional[str] = None):
        core = load_core()
        self.svc = core_svc
        self.plugin_dir = os.path.join(data, "plugins")
        os.makedirs(self.plugin_dir, exist_ok=True)
        self.watcher = core.PluginWatcher(self.plugin_dir)
        self.triggers = core.TriggerStore(triggers_db or os.path.join(data, "data", "plugin_triggers.db"))
        self.log_offsets: dict = {}
        self.fired: list = []

    def _metrics(self) -> dict:
        from ..utils import sysinfo

        try:
            return sysinfo.metric_snapshot()
        except Exception:  # pragma: no cover - platform specific
            return {}

    def _new_log_lines(self, path: str) -> list:
        try:
            size = os.path.getsize(path)
        except OSError:
            return []
        off = self.log_offsets.get(path)
        if off is None or off > size:  # first look: start at the end (only new lines fire)
            self.log_offsets[path] = size
            return []
        with open(path, "rb") as f:
            f.seek(off)
            data = f.read(min(size - off, 1 << 20))
        self.log_offsets[path] = off + len(data)
        return data.decode(errors="replace").splitlines()

    def tick(self, now: Optional[int] = None) -> dict:
        changes = self.watcher.poll()
        if changes["added"] or changes["changed"]:
            self.svc.scan_plugins()
        for name in changes["removed"]:
            self.svc.deregister_tool(f"plugin.{name}")
        trig = self.triggers.list()
        logs = {t["config"]["log_path"]: self._new_log_lines(t["config"]["log_path"])
                for t in trig if t["type"] == "log_pattern" and t["enabled"]}
        metrics = self._metrics() if any(t["type"] == "metric_threshold" for t in trig) else {}
        due = self.triggers.due(int(now if now is not None else time.time()), metrics, logs)
        for t in due:
            tool = t["plugin"] if t["plugin"].startswith("plugin.") else f"plugin.{t['plugin']}"
            payload = json.dumps({"trigger": {"id": t["id"], "type": t["type"], "config": t["config"]}})
            r = self.svc.execute(tool, "autonomy-loop", f"trigger-{t['id']}", payload.encode(), f"{t['type']} trigger")
            self.fired.append({"trigger": t["id"], "tool": tool, "success": r["success"]})
            log.info("trigger %s (%s) fired %s: %s", t["id"], t["type"], tool, "ok" if r["success"] else r["error"])
        return {"changes": changes, "fired": [t["id"] for t in due]}


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
            "rollback_tool": t.rollback_tool, "handler_address": req.handler_address,
            "input_schema": t.input_schema.decode(errors="replace") if t.input_schema else ""})
        log.info("register %s -> %s (%s)", t.name, req.handler_address or "local", "ok" if ok else err)
        return pb.tools.RegisterToolResponse(accepted=ok, error=err)

    async def Deregister(self, req, ctx):
        ok = self.core.deregister_tool(req.tool_name)
        return pb.tools.Status(success=ok, message=f"Tool {req.tool_name} " + ("deregistered" if ok else "not found"))

    # ---------------------------------------------------------------- background
    async def plugin_scan_loop(self, stop: asyncio.Event):
        """Plugin runtime (tools/src/plugin/mod.rs:107-219, events.rs, triggers.rs -- defined but
        never started in the reference): hot reload from the plugin directory (new / changed
        plugins are (re)registered, deleted ones deregistered) and trigger dispatch (cron,
        file_watch, log_pattern, metric_threshold) executing the plugin through the normal
        capability / audit pipeline as `autonomy-loop`."""
        runtime = PluginRuntime(self.core, self.data_dir)
        while not stop.is_set():
            try:
                await self._run(runtime.tick)
            except Exception as e:  # pragma: no cover - defensive
                log.warning("plugin runtime tick failed: %s", e)
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

"""Lazily connected clients for the orchestrator's downstream services + AI inference helpers.

Reference: `agent-core/src/clients.rs:17-146` (lazy channels, env addresses, 300 s request
timeout, optional discovery lookup with AIOS_USE_DISCOVERY=true) and the inference fallbacks of
`autonomy.rs:1058-1144` / `task_planner.rs:143-223` (gateway first, runtime second).
"""
from __future__ import annotations

import json
import logging
import os
from dataclasses import dataclass, field
from typing import List, Optional

import grpc

from ..rpc.client import Stub, channel
from ..rpc.schema import pb
from ..utils.env import addr, env_flag

log = logging.getLogger("aios.orchestrator.clients")

_SVC = {
    "tools": "aios.tools.ToolRegistry",
    "memory": "aios.memory.MemoryService",
    "api-gateway": "aios.api_gateway.ApiGateway",
    "runtime": "aios.runtime.AIRuntime",
}


@dataclass
class InferResult:
    success: bool
    text: str
    model_used: str = "none"
    tokens_used: int = 0
    backend: str = ""


class ServiceClients:
    def __init__(self, discovery=None, timeout: float = 300.0):
        self.discovery = discovery
        self.timeout = timeout
        self._stubs = {}

    def address(self, name: str) -> str:
        if self.discovery is not None and env_flag("AIOS_USE_DISCOVERY"):
            s = self.discovery.lookup(name)
            if s and s.get("port"):
                return f"{s['address']}:{s['port']}"
        return addr(name)

    def stub(self, name: str) -> Stub:
        a = self.address(name)
        key = (name, a)
        if key not in self._stubs:
            self._stubs[key] = Stub(channel(a), _SVC[name], timeout=self.timeout)
        return self._stubs[key]

    tools = property(lambda self: self.stub("tools"))
    memory = property(lambda self: self.stub("memory"))
    gateway = property(lambda self: self.stub("api-gateway"))
    runtime = property(lambda self: self.stub("runtime"))

    # ------------------------------------------------------------------ inference
    async def gateway_infer(self, prompt: str, system_prompt: str, max_tokens: int, temperature: float = 0.3,
                            provider: str = "", agent: str = "autonomy-loop", task_id: str = "") -> Optional[InferResult]:
        try:
            r = await self.gateway.Infer(pb.api_gateway.ApiInferRequest(
                prompt=prompt, system_prompt=system_prompt, max_tokens=max_tokens, temperature=temperature,
                preferred_provider=provider, requesting_agent=agent, task_id=task_id, allow_fallback=True))
            return InferResult(True, r.text, r.model_used, r.tokens_used, "api-gateway")
        except grpc.aio.AioRpcError as e:
            log.debug("gateway inference failed: %s", e.details())
            return None

    async def runtime_infer(self, prompt: str, system_prompt: str, max_tokens: int, temperature: float = 0.3,
                            level: str = "operational", agent: str = "autonomy-loop", task_id: str = "",
                            model: str = "") -> Optional[InferResult]:
        try:
            r = await self.runtime.Infer(pb.runtime.InferRequest(
                model=model, prompt=prompt, system_prompt=system_prompt, max_tokens=max_tokens,
                temperature=temperature, intelligence_level=level, requesting_agent=agent, task_id=task_id))
            return InferResult(True, r.text, r.model_used, r.tokens_used, "runtime")
        except grpc.aio.AioRpcError as e:
            log.debug("runtime inference failed: %s", e.details())
            return None

    async def infer_any(self, prompt: str, system_prompt: str, max_tokens: int, level: str, provider: str = "",
                        task_id: str = "", order: Optional[List[str]] = None) -> Optional[InferResult]:
        """Backends in `order` (default: gateway then runtime); None when all fail."""
        for b in order or ["api-gateway", "runtime"]:
            if b == "api-gateway":
                r = await self.gateway_infer(prompt, system_prompt, max_tokens, provider=provider, task_id=task_id)
            else:
                r = await self.runtime_infer(prompt, system_prompt, max_tokens, level=level, task_id=task_id)
            if r is not None:
                return r
        return None

    # ------------------------------------------------------------------ tools
    async def execute_tool(self, tool: str, input_obj, task_id: str, agent: str = "autonomy-loop") -> dict:
        """autonomy.rs:1619-1664: {tool, success, output, execution_id, duration_ms} or a failure dict."""
        data = input_obj if isinstance(input_obj, (bytes, bytearray)) else json.dumps(input_obj or {}).encode()
        try:
            r = await self.tools.Execute(pb.tools.ExecuteRequest(
                tool_name=tool, agent_id=agent, task_id=task_id, input_json=data,
                reason=f"Autonomy loop executing tool for task {task_id}"))
        except grpc.aio.AioRpcError as e:
            return {"tool": tool, "success": False, "error": f"Tool execution gRPC failed: {e.details()}"}
        if not r.success:
            return {"tool": tool, "success": False, "error": f"Tool '{tool}' failed: {r.error}"}
        try:
            out = json.loads(r.output_json) if r.output_json else {}
        except ValueError:
            out = r.output_json.decode("utf-8", "replace")
        return {"tool": tool, "success": True, "output": out, "execution_id": r.execution_id,
                "duration_ms": r.duration_ms}

    async def tool_catalog(self) -> str:
        """Live catalog grouped by namespace (autonomy.rs:988-1036), static fallback."""
        try:
            r = await self.tools.ListTools(pb.tools.ListToolsRequest(), timeout=5)
        except grpc.aio.AioRpcError:
            return STATIC_TOOL_CATALOG
        if not r.tools:
            return STATIC_TOOL_CATALOG
        by_ns = {}
        for t in r.tools:
            by_ns.setdefault(t.namespace or "other", []).append(f"{t.name} — {t.description}" if t.description
                                                                  else t.name)
        out = f"Available tools ({len(r.tools)} total):\n"
        for ns in sorted(by_ns):
            out += f"[{ns}] {', '.join(by_ns[ns])}\n"
        return out + "\n"

    async def memory_context(self, task: str, max_tokens: int = 2048) -> List[dict]:
        try:
            r = await self.memory.AssembleContext(pb.memory.ContextRequest(
                task_description=task, max_tokens=max_tokens, memory_tiers=["operational", "working", "long_term"]),
                timeout=5)
            return [{"source": c.source, "content": c.content} for c in r.chunks]
        except grpc.aio.AioRpcError:
            return []


STATIC_TOOL_CATALOG = (
    "Available tools you can call:\n"
    " - fs.read, fs.write, fs.list, fs.delete, fs.mkdir, fs.copy, fs.move, fs.stat, fs.search\n"
    " - process.list, process.kill, process.spawn, process.info\n"
    " - service.list, service.start, service.stop, service.restart, service.status\n"
    " - net.ping, net.dns, net.interfaces, net.http_get, net.port_scan\n"
    " - firewall.rules, firewall.add_rule, firewall.delete_rule\n"
    " - pkg.install, pkg.remove, pkg.list_installed, pkg.search, pkg.update\n"
    " - sec.check_perms, sec.audit_query\n"
    " - monitor.cpu, monitor.memory, monitor.disk, monitor.network, monitor.logs\n"
    " - web.http_request, web.scrape, web.webhook, web.download, web.api_call\n"
    " - git.init, git.clone, git.add, git.commit, git.push, git.pull, git.branch, git.status, git.log, git.diff\n"
    " - code.scaffold, code.generate\n"
    " - self.inspect, self.health, self.update, self.rebuild\n"
    " - plugin.create, plugin.list, plugin.delete, plugin.install_deps\n\n")

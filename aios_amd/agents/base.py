"""BaseAgent: the long-running Python worker every aiOS agent derives from.

Reference: `agent-core/python/aios_agent/base.py` -- lazy gRPC channels to
orchestrator / tools / memory / runtime, `call_tool`, memory helpers, `think()` (AIRuntime.Infer,
1024 tokens, T=0.3, the level string), registration, 10 s heartbeat, 2 s GetAssignedTask poll,
execute + ReportTaskResult, run/shutdown.

Same wire contract, different construction: typed stubs come from the runtime-built descriptor
pool (`aios_amd/rpc`), so there are no generated *_pb2 files and the orchestrator client speaks
real protobuf (the reference's OrchestratorClient sent JSON over a raw method, App. A).
Memory state is a per-agent key/value document (`store_memory` merges keys; the reference
overwrote the whole state on every call).  Subclasses implement `handle_task`, and may declare
`ACTIONS` (keyword -> coroutine) to get keyword dispatch for free, plus `background()` loops.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import re
import signal
import time
import uuid
from abc import ABC, abstractmethod
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Awaitable, Callable, Dict, List, Optional, Sequence, Tuple

import grpc

from ..rpc.client import Stub, channel
from ..rpc.schema import pb

logger = logging.getLogger("aios.agent")


class IntelligenceLevel(str, Enum):
    REACTIVE = "reactive"
    OPERATIONAL = "operational"
    TACTICAL = "tactical"
    STRATEGIC = "strategic"


@dataclass
class AgentConfig:
    orchestrator_addr: str = field(default_factory=lambda: os.getenv("AIOS_ORCHESTRATOR_ADDR", "127.0.0.1:50051"))
    tools_addr: str = field(default_factory=lambda: os.getenv("AIOS_TOOLS_ADDR", "127.0.0.1:50052"))
    memory_addr: str = field(default_factory=lambda: os.getenv("AIOS_MEMORY_ADDR", "127.0.0.1:50053"))
    runtime_addr: str = field(default_factory=lambda: os.getenv("AIOS_RUNTIME_ADDR", "127.0.0.1:50055"))
    heartbeat_interval_s: float = 10.0
    poll_interval_s: float = 2.0
    grpc_timeout_s: float = 30.0
    think_max_tokens: int = 1024
    think_temperature: float = 0.3
    extra: Dict[str, Any] = field(default_factory=dict)


def _host(addr: str) -> str:
    for p in ("http://", "https://"):
        if addr.startswith(p):
            addr = addr[len(p):]
    return addr.replace("localhost", "127.0.0.1")


def extract_json(text: str) -> Any:
    """First JSON value in an LLM answer (think tags / fences tolerated); None when absent."""
    text = re.sub(r"<think>.*?</think>", "", text or "", flags=re.S).strip()
    for cand in (text, *re.findall(r"```(?:json)?\s*(.*?)```", text, flags=re.S)):
        try:
            return json.loads(cand)
        except (ValueError, TypeError):
            pass
    for open_c, close_c in (("{", "}"), ("[", "]")):
        start = text.find(open_c)
        while start >= 0:
            depth, in_str, esc = 0, False, False
            for i in range(start, len(text)):
                ch = text[i]
                if in_str:
                    esc = (ch == "\\") and not esc
                    if ch == '"' and not esc:
                        in_str = False
                    continue
                if ch == '"':
                    in_str = True
                elif ch == open_c:
                    depth += 1
                elif ch == close_c:
                    depth -= 1
                    if depth == 0:
                        try:
                            return json.loads(text[start:i + 1])
                        except ValueError:
                            break
            start = text.find(open_c, start + 1)
    return None


Action = Callable[[Dict[str, Any]], Awaitable[Dict[str, Any]]]


class BaseAgent(ABC):
    AGENT_TYPE = "base"
    CAPABILITIES: Sequence[str] = ()
    # (keywords, method name); first entry whose keyword occurs in the task text wins
    ACTIONS: Sequence[Tuple[Sequence[str], str]] = ()

    def __init__(self, agent_id: Optional[str] = None, config: Optional[AgentConfig] = None):
        self.agent_id = agent_id or os.getenv("AIOS_AGENT_NAME") or f"{self.get_agent_type()}-{uuid.uuid4().hex[:8]}"
        self.config = config or AgentConfig()
        self.started = time.time()
        self.tasks_completed = 0
        self.tasks_failed = 0
        self.current_task_id: Optional[str] = None
        self._stop = asyncio.Event()
        self._stubs: Dict[str, Stub] = {}
        self._bg: List[asyncio.Task] = []

    # ------------------------------------------------------------------ identity
    def get_agent_type(self) -> str:
        return self.AGENT_TYPE

    def get_capabilities(self) -> List[str]:
        return list(self.CAPABILITIES)

    def tool_namespaces(self) -> List[str]:
        return sorted({c.split(".")[0] for c in self.get_capabilities() if "." in c})

    # ------------------------------------------------------------------ stubs
    def _stub(self, which: str) -> Stub:
        if which not in self._stubs:
            addr, svc = {
                "orchestrator": (self.config.orchestrator_addr, "aios.orchestrator.Orchestrator"),
                "tools": (self.config.tools_addr, "aios.tools.ToolRegistry"),
                "memory": (self.config.memory_addr, "aios.memory.MemoryService"),
                "runtime": (self.config.runtime_addr, "aios.runtime.AIRuntime"),
            }[which]
            self._stubs[which] = Stub(channel(_host(addr)), svc, timeout=self.config.grpc_timeout_s)
        return self._stubs[which]

    # ------------------------------------------------------------------ tools
    async def call_tool(self, name: str, input_json: Optional[Dict[str, Any]] = None, *, reason: str = "",
                        task_id: Optional[str] = None) -> Dict[str, Any]:
        req = pb.tools.ExecuteRequest(tool_name=name, agent_id=self.agent_id,
                                      task_id=task_id or self.current_task_id or "",
                                      input_json=json.dumps(input_json or {}, default=str).encode(),
                                      reason=reason or f"{self.agent_id} executing {name}")
        try:
            r = await self._stub("tools").Execute(req)
        except grpc.aio.AioRpcError as e:
            return {"success": False, "tool": name, "error": f"tools service: {e.details()}"}
        out: Any = {}
        if r.output_json:
            try:
                out = json.loads(r.output_json)
            except ValueError:
                out = {"raw": r.output_json.decode("utf-8", "replace")}
        res = {"success": r.success, "tool": name, "execution_id": r.execution_id, "duration_ms": r.duration_ms}
        if r.success:
            res.update(output=out, backup_id=r.backup_id)
        else:
            res["error"] = r.error
            logger.warning("tool %s failed: %s", name, r.error)
        return res

    async def call_tools(self, calls: Sequence[Tuple[str, Dict[str, Any]]]) -> List[Dict[str, Any]]:
        """Independent tool calls concurrently (the reference's asyncio.gather health checks)."""
        return list(await asyncio.gather(*(self.call_tool(n, i) for n, i in calls)))

    async def rollback_tool(self, execution_id: str, reason: str = "") -> Dict[str, Any]:
        r = await self._stub("tools").Rollback(pb.tools.RollbackRequest(execution_id=execution_id, reason=reason))
        return {"success": r.success, "error": r.error}

    async def list_tools(self, namespace: str = "") -> List[Dict[str, Any]]:
        r = await self._stub("tools").ListTools(pb.tools.ListToolsRequest(namespace=namespace))
        return [{"name": t.name, "namespace": t.namespace, "description": t.description, "risk_level": t.risk_level}
                for t in r.tools]

    # ------------------------------------------------------------------ memory
    async def _state(self) -> Dict[str, Any]:
        r = await self._stub("memory").GetAgentState(pb.memory.AgentStateRequest(agent_name=self.agent_id))
        try:
            st = json.loads(r.state_json) if r.state_json else {}
        except ValueError:
            st = {}
        return st if isinstance(st, dict) else {}

    async def store_memory(self, key: str, value: Any) -> None:
        st = await self._state()
        st[key] = value
        await self._stub("memory").StoreAgentState(pb.memory.AgentState(
            agent_name=self.agent_id, state_json=json.dumps(st, default=str).encode(), updated_at=int(time.time())))

    async def recall_memory(self, key: str, default: Any = None) -> Any:
        return (await self._state()).get(key, default)

    async def push_event(self, category: str, data: Dict[str, Any], *, critical: bool = False) -> None:
        await self._stub("memory").PushEvent(pb.memory.Event(
            id=uuid.uuid4().hex, timestamp=int(time.time()), category=category, source=self.agent_id,
            data_json=json.dumps(data, default=str).encode(), critical=critical))

    async def get_recent_events(self, count: int = 50, category: str = "", source: str = "") -> List[Dict[str, Any]]:
        r = await self._stub("memory").GetRecentEvents(pb.memory.RecentEventsRequest(count=count, category=category,
                                                                                      source=source))
        out = []
        for e in r.events:
            try:
                data = json.loads(e.data_json) if e.data_json else {}
            except ValueError:
                data = {}
            out.append({"id": e.id, "timestamp": e.timestamp, "category": e.category, "source": e.source,
                        "data": data, "critical": e.critical})
        return out

    async def update_metric(self, key: str, value: float) -> None:
        await self._stub("memory").UpdateMetric(pb.memory.MetricUpdate(key=key, value=float(value),
                                                                       timestamp=int(time.time())))

    async def get_metric(self, key: str) -> Optional[float]:
        r = await self._stub("memory").GetMetric(pb.memory.MetricRequest(key=key))
        return r.value if r.timestamp else None

    async def store_pattern(self, trigger: str, action: str, success_rate: float = 1.0) -> None:
        await self._stub("memory").StorePattern(pb.memory.Pattern(
            id=uuid.uuid4().hex, trigger=trigger, action=action, success_rate=success_rate, uses=1,
            last_used=int(time.time()), created_from=self.agent_id))

    async def find_pattern(self, trigger: str, min_success_rate: float = 0.5) -> Optional[Dict[str, Any]]:
        r = await self._stub("memory").FindPattern(pb.memory.PatternQuery(trigger=trigger,
                                                                          min_success_rate=min_success_rate))
        if not r.found:
            return None
        p = r.pattern
        return {"id": p.id, "trigger": p.trigger, "action": p.action, "success_rate": p.success_rate, "uses": p.uses}

    async def store_decision(self, context: str, options: List[str], chosen: str, reasoning: str,
                             level: str = "operational") -> None:
        await self._stub("memory").StoreDecision(pb.memory.Decision(
            id=uuid.uuid4().hex, context=context, options_json=json.dumps(options).encode(), chosen=chosen,
            reasoning=reasoning, intelligence_level=level, model_used=self.agent_id, timestamp=int(time.time())))

    async def semantic_search(self, query: str, collections: Sequence[str] = (), n: int = 5,
                              min_relevance: float = 0.0) -> List[Dict[str, Any]]:
        r = await self._stub("memory").SemanticSearch(pb.memory.SemanticSearchRequest(
            query=query, collections=list(collections), n_results=n, min_relevance=min_relevance))
        return [{"content": x.content, "relevance": x.relevance, "collection": x.collection, "id": x.id}
                for x in r.results]

    async def assemble_context(self, task: str, max_tokens: int = 2048, tiers: Sequence[str] = ()) -> str:
        r = await self._stub("memory").AssembleContext(pb.memory.ContextRequest(
            task_description=task, max_tokens=max_tokens, memory_tiers=list(tiers)))
        return "\n".join(f"[{c.source}] {c.content}" for c in r.chunks)

    # ------------------------------------------------------------------ inference
    async def think(self, prompt: str, level: IntelligenceLevel | str = IntelligenceLevel.OPERATIONAL, *,
                    system_prompt: str = "", max_tokens: Optional[int] = None, temperature: Optional[float] = None,
                    task_id: Optional[str] = None) -> str:
        level = IntelligenceLevel(level)
        system = system_prompt or (f"You are the {self.get_agent_type()} agent of aiOS, an AI-native operating "
                                   f"system on AMD Instinct GPUs. Agent ID: {self.agent_id}. Answer concisely.")
        r = await self._stub("runtime").Infer(pb.runtime.InferRequest(
            prompt=prompt, system_prompt=system, max_tokens=max_tokens or self.config.think_max_tokens,
            temperature=self.config.think_temperature if temperature is None else temperature,
            intelligence_level=level.value, requesting_agent=self.agent_id,
            task_id=task_id or self.current_task_id or ""))
        return r.text

    async def think_json(self, prompt: str, level: IntelligenceLevel | str = IntelligenceLevel.OPERATIONAL,
                         **kw) -> Any:
        """think() asking for JSON; parsed value or None (never raises on bad model output)."""
        try:
            text = await self.think(prompt + "\nRespond with ONLY a valid JSON object.", level, **kw)
        except grpc.aio.AioRpcError as e:
            logger.info("think unavailable: %s", e.details())
            return None
        return extract_json(text)

    async def analyze(self, prompt: str, level: IntelligenceLevel | str = IntelligenceLevel.TACTICAL, **kw) -> str:
        """think() for an analysis / advice paragraph; "" when the runtime is unavailable, so an
        agent's action still returns its tool results without the model's reading of them."""
        try:
            return (await self.think(prompt, level, **kw)).strip()
        except grpc.aio.AioRpcError as e:
            logger.info("think unavailable: %s", e.details())
            return ""

    async def safety_check(self, prompt: str, level: IntelligenceLevel | str = IntelligenceLevel.OPERATIONAL,
                           **kw) -> Optional[str]:
        """think() at a gate in front of a side effect (firewall rule, service restart, package
        install/remove, backup, restore): the model's answer, or None when the runtime is unreachable or
        answers nothing.  Callers fail closed on None -- the reference calls think() directly at these
        sites (agents/network.py:329, agents/system.py:238), so its RPC error fails the task."""
        try:
            text = (await self.think(prompt, level, **kw)).strip()
        except grpc.aio.AioRpcError as e:
            logger.warning("safety check unavailable: %s", e.details())
            return None
        return text or None

    @staticmethod
    def safety_unavailable(action: str, **extra) -> Dict[str, Any]:
        return {"success": False, "error": f"safety check unavailable: not {action} without the model's review",
                **extra}

    @staticmethod
    def advice_lines(text: str, n: int = 5) -> List[str]:
        """the first n non-empty lines of a model answer, list markers stripped"""
        return [ln.strip().lstrip("-*0123456789.) ").strip() for ln in (text or "").splitlines()
                if ln.strip().lstrip("-*0123456789.) ").strip()][:n]

    # ------------------------------------------------------------------ orchestrator
    async def register_with_orchestrator(self) -> bool:
        try:
            r = await self._stub("orchestrator").RegisterAgent(pb.common.AgentRegistration(
                agent_id=self.agent_id, agent_type=self.get_agent_type(), capabilities=self.get_capabilities(),
                tool_namespaces=self.tool_namespaces(), status="idle", registered_at=int(time.time())))
            return r.success
        except grpc.aio.AioRpcError as e:
            logger.error("registration failed: %s", e.details())
            return False

    async def unregister_from_orchestrator(self) -> bool:
        try:
            return (await self._stub("orchestrator").UnregisterAgent(pb.common.AgentId(id=self.agent_id))).success
        except grpc.aio.AioRpcError:
            return False

    async def send_heartbeat(self) -> bool:
        try:
            import resource

            mem_mb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
        except Exception:
            mem_mb = 0.0
        try:
            r = await self._stub("orchestrator").Heartbeat(pb.orchestrator.HeartbeatRequest(
                agent_id=self.agent_id, status="busy" if self.current_task_id else "idle",
                current_task_id=self.current_task_id or "", memory_usage_mb=mem_mb), timeout=5)
            if not r.success:  # orchestrator restarted and forgot us
                await self.register_with_orchestrator()
            return r.success
        except grpc.aio.AioRpcError as e:
            logger.warning("heartbeat failed: %s", e.details())
            return False

    async def request_capability(self, capabilities: List[str], reason: str = "", duration_hours: int = 24):
        r = await self._stub("orchestrator").RequestCapability(pb.orchestrator.CapabilityRequest(
            agent_id=self.agent_id, capabilities=capabilities, reason=reason, duration_hours=duration_hours))
        return {"granted": r.granted, "capabilities": list(r.capabilities), "expires_at": r.expires_at,
                "denial_reason": r.denial_reason}

    async def poll_once(self) -> bool:
        """GetAssignedTask -> execute -> ReportTaskResult.  True when a task was executed."""
        try:
            t = await self._stub("orchestrator").GetAssignedTask(pb.common.AgentId(id=self.agent_id), timeout=5)
        except grpc.aio.AioRpcError as e:
            if e.code() != grpc.StatusCode.UNAVAILABLE:
                logger.warning("GetAssignedTask failed: %s", e.code())
            return False
        if not t.id:
            return False
        task = {"id": t.id, "goal_id": t.goal_id, "description": t.description, "status": t.status,
                "intelligence_level": t.intelligence_level, "required_tools": list(t.required_tools),
                "depends_on": list(t.depends_on)}
        try:
            task["input"] = json.loads(t.input_json) if t.input_json else {}
        except ValueError:
            task["input"] = {}
        t0 = time.time()
        result = await self.execute_task(task)
        ok = bool(result.get("success", True)) and "error" not in result
        await self._stub("orchestrator").ReportTaskResult(pb.common.TaskResult(
            task_id=t.id, success=ok, output_json=json.dumps(result, default=str).encode(),
            error="" if ok else str(result.get("error", "task failed")),
            duration_ms=int((time.time() - t0) * 1000), model_used=self.agent_id))
        return True

    async def execute_task(self, task: Dict[str, Any]) -> Dict[str, Any]:
        self.current_task_id = task.get("id")
        try:
            out = await self.handle_task(task)
            if out.get("success", True) and "error" not in out:
                self.tasks_completed += 1
            else:
                self.tasks_failed += 1
            return out
        except Exception as e:
            logger.exception("task %s failed", task.get("id"))
            self.tasks_failed += 1
            return {"success": False, "error": f"{type(e).__name__}: {e}"}
        finally:
            self.current_task_id = None

    # ------------------------------------------------------------------ dispatch
    def match_action(self, text: str) -> Optional[str]:
        t = text.lower()
        for keywords, method in self.ACTIONS:
            if any(k in t for k in keywords):
                return method
        return None

    async def handle_task(self, task: Dict[str, Any]) -> Dict[str, Any]:
        """Keyword dispatch over ACTIONS; unmatched tasks go to `fallback` (LLM-assisted)."""
        text = f"{task.get('description', '')} {json.dumps(task.get('input', {}))}"
        method = task.get("input", {}).get("action") or self.match_action(text)
        if method and hasattr(self, method):
            return await getattr(self, method)(task)
        return await self.fallback(task)

    async def fallback(self, task: Dict[str, Any]) -> Dict[str, Any]:
        """Ask the model which of this agent's actions fits, then run it."""
        names = [m for _, m in self.ACTIONS]
        choice = await self.think_json(
            f"Task: {task.get('description', '')}\nChoose one action from {names} for the "
            f"{self.get_agent_type()} agent. JSON: {{\"action\": \"<name>\", \"reason\": \"...\"}}",
            IntelligenceLevel.OPERATIONAL)
        if isinstance(choice, dict) and choice.get("action") in names:
            return await getattr(self, choice["action"])(task)
        return {"success": False, "error": f"{self.get_agent_type()} agent cannot handle: {task.get('description')}"}

    # ------------------------------------------------------------------ lifecycle
    async def background(self) -> List[Awaitable]:
        """Subclass periodic loops (coroutines), started by run()."""
        return []

    async def periodic(self, interval_s: float, fn: Callable[[], Awaitable[Any]]):
        while not self._stop.is_set():
            try:
                await fn()
            except Exception as e:
                logger.debug("%s periodic task failed: %s", self.agent_id, e)
            try:
                await asyncio.wait_for(self._stop.wait(), interval_s)
            except asyncio.TimeoutError:
                pass

    async def heartbeat_loop(self):
        """Heartbeat every heartbeat_interval_s until shutdown (reference base.py:684)."""
        await self.periodic(self.config.heartbeat_interval_s, self.send_heartbeat)

    async def task_poll_loop(self):
        """Poll GetAssignedTask, execute, report, until shutdown (reference base.py:728)."""
        while not self._stop.is_set():
            try:
                busy = await self.poll_once()
            except Exception as e:
                logger.warning("poll error: %s", e)
                busy = False
            if busy:
                continue
            try:
                await asyncio.wait_for(self._stop.wait(), self.config.poll_interval_s)
            except asyncio.TimeoutError:
                pass

    async def run(self):
        for _ in range(30):
            if await self.register_with_orchestrator():
                break
            await asyncio.sleep(2)
        loop = asyncio.get_running_loop()
        for sig in (signal.SIGINT, signal.SIGTERM):
            try:
                loop.add_signal_handler(sig, self.shutdown)
            except (NotImplementedError, RuntimeError):
                pass
        coros = [self.heartbeat_loop(), self.task_poll_loop(), *(await self.background())]
        self._bg = [asyncio.ensure_future(c) for c in coros]
        await self._stop.wait()
        for t in self._bg:
            t.cancel()
        await self.unregister_from_orchestrator()

    def shutdown(self):
        self._stop.set()

    def uptime_seconds(self) -> int:
        return int(time.time() - self.started)

    def get_status(self) -> Dict[str, Any]:
        return {"agent_id": self.agent_id, "agent_type": self.get_agent_type(),
                "status": "busy" if self.current_task_id else "idle", "current_task_id": self.current_task_id or "",
                "tasks_completed": self.tasks_completed, "tasks_failed": self.tasks_failed,
                "uptime_seconds": self.uptime_seconds()}


def main_for(cls):
    """`python -m aios_amd.agents.<type>` entry point."""
    logging.basicConfig(level=os.environ.get("AIOS_LOG", "INFO"),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    asyncio.run(cls().run())

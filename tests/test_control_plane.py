"""End-to-end control plane on CPU: tools + memory + gateway + orchestrator services on ephemeral
ports, driven over real gRPC (mirrors the reference's service-level behaviour).

A scripted AIRuntime stands in for the GPU runtime (same role as the reference's fake/mocked
inference in its unit tests); an aiohttp server plays the OpenAI-compatible `local` provider.
"""
import asyncio
import json
import os
import time

import pytest

from aios_amd.rpc.client import Stub, channel, close_all
from aios_amd.rpc.schema import pb
from aios_amd.rpc.server import RpcServer


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


class ScriptedRuntime:
    """AIRuntime double: answers decomposition prompts with a JSON plan and task prompts with
    tool calls, recording every request."""

    def __init__(self, plan=None, calls=None):
        self.requests = []
        self.plan = plan
        self.calls = calls

    async def Infer(self, req, ctx):
        self.requests.append(req)
        if "Decompose this goal" in req.prompt:
            text = json.dumps(self.plan) if self.plan is not None else "no plan"
        elif "Previous tool results" in req.prompt:
            text = '{"done": true, "summary": "finished"}'
        else:
            text = "<think>hmm</think>" + json.dumps({"reasoning": "inspect", "tool_calls": self.calls or []})
        return pb.runtime.InferResponse(text=text, tokens_used=42, latency_ms=5, model_used="scripted")

    async def ListModels(self, req, ctx):
        return pb.runtime.ModelList(models=[pb.runtime.ModelStatus(model_name="mistral-7b", status="ready")])


async def _start(tmp, runtime=None, with_gateway=False):
    from aios_amd.memory.service import MemoryServiceImpl
    from aios_amd.orchestrator.clients import ServiceClients
    from aios_amd.orchestrator.service import OrchestratorService
    from aios_amd.orchestrator.state import OrchestratorState
    from aios_amd.tools.service import ToolRegistryService

    servers = {}
    tools = ToolRegistryService(str(tmp / "tools"))
    servers["tools"] = await RpcServer("127.0.0.1:0", {"aios.tools.ToolRegistry": tools}).start()
    mem = MemoryServiceImpl(str(tmp / "w.db"), str(tmp / "lt.db"), str(tmp / "kn.db"))
    servers["memory"] = await RpcServer("127.0.0.1:0", {"aios.memory.MemoryService": mem}).start()
    if runtime is not None:
        servers["runtime"] = await RpcServer("127.0.0.1:0", {"aios.runtime.AIRuntime": runtime}).start()
    addrs = {k: f"127.0.0.1:{s.port}" for k, s in servers.items()}
    addrs.setdefault("runtime", "127.0.0.1:1")
    addrs.setdefault("api-gateway", "127.0.0.1:1")
    clients = ServiceClients(timeout=10)
    clients.address = lambda name: addrs[name]
    st = OrchestratorState(str(tmp / "orch"), clients=clients)
    servers["orchestrator"] = await RpcServer("127.0.0.1:0", {"aios.orchestrator.Orchestrator":
                                                             OrchestratorService(st)}).start()
    addrs["orchestrator"] = f"127.0.0.1:{servers['orchestrator'].port}"
    return st, servers, addrs, tools


async def _stop(servers):
    for s in servers.values():
        await s.stop(0)
    await close_all()


def _orch(addrs):
    return Stub(channel(addrs["orchestrator"]), "aios.orchestrator.Orchestrator", timeout=10)


# ------------------------------------------------------------------------------------ tools over gRPC
def test_tools_service_grpc(tmp_path):
    async def go():
        st, servers, addrs, _ = await _start(tmp_path)
        try:
            t = Stub(channel(addrs["tools"]), "aios.tools.ToolRegistry", timeout=10)
            lst = await t.ListTools(pb.tools.ListToolsRequest(namespace="monitor"))
            assert {x.name for x in lst.tools} >= {"monitor.cpu", "monitor.memory", "monitor.disk"}
            d = await t.GetTool(pb.tools.GetToolRequest(name="fs.write"))
            assert d.reversible
            p = tmp_path / "f.txt"
            r = await t.Execute(pb.tools.ExecuteRequest(tool_name="fs.write", agent_id="task-agent",
                                                        input_json=json.dumps({"path": str(p), "content": "x"}).encode()))
            assert r.success and p.exists() and r.execution_id
            rb = await t.Rollback(pb.tools.RollbackRequest(execution_id=r.execution_id))
            assert rb.success and not p.exists()
            reg = await t.Register(pb.tools.RegisterToolRequest(
                tool=pb.tools.ToolDefinition(name="remote.echo", namespace="remote", description="echo",
                                             required_capabilities=[]), handler_address="127.0.0.1:1"))
            assert reg.accepted
            dr = await t.Deregister(pb.tools.DeregisterToolRequest(tool_name="remote.echo"))
            assert dr.success
        finally:
            await _stop(servers)
    run(go())


# ------------------------------------------------------------------------------------ memory over gRPC
def test_memory_service_grpc(tmp_path):
    async def go():
        st, servers, addrs, _ = await _start(tmp_path)
        M = pb.memory
        try:
            m = Stub(channel(addrs["memory"]), "aios.memory.MemoryService", timeout=10)
            await m.PushEvent(M.Event(id="e1", category="cpu", source="t", data_json=b'{"v": 1}'))
            ev = await m.GetRecentEvents(M.RecentEventsRequest(count=10))
            assert [e.id for e in ev.events] == ["e1"] and ev.events[0].timestamp > 0
            await m.UpdateMetric(M.MetricUpdate(key="cpu.usage", value=12.5))
            assert (await m.GetMetric(M.MetricRequest(key="cpu.usage"))).value == 12.5
            snap = await m.GetSystemSnapshot(M.Empty())
            assert snap.cpu_percent == 12.5
            await m.StoreGoal(M.GoalRecord(id="g1", description="rotate logs", status="in_progress", priority=3))
            assert [g.id for g in (await m.GetActiveGoals(M.Empty())).goals] == ["g1"]
            await m.StorePattern(M.Pattern(id="p1", trigger="disk full", action="clean", success_rate=0.9))
            pr = await m.FindPattern(M.PatternQuery(trigger="disk full"))
            assert pr.found and pr.pattern.id == "p1"
            assert not (await m.FindPattern(M.PatternQuery(trigger="zzz"))).found
            await m.StoreAgentState(M.AgentState(agent_name="a", state_json=b'{"k": 2}'))
            assert json.loads((await m.GetAgentState(M.AgentStateRequest(agent_name="a"))).state_json) == {"k": 2}
            await m.AddKnowledge(M.KnowledgeEntry(title="nginx", content="restart nginx via systemctl"))
            sr = await m.SearchKnowledge(M.SemanticSearchRequest(query="restart nginx", n_results=3))
            assert sr.results and "nginx" in sr.results[0].content
            await m.StoreProcedure(M.Procedure(id="pr", name="log rotation", description="rotate nginx logs"))
            ss = await m.SemanticSearch(M.SemanticSearchRequest(query="nginx logs", collections=["procedures"]))
            assert ss.results
            ctx = await m.AssembleContext(M.ContextRequest(task_description="restart nginx", max_tokens=500,
                                                           memory_tiers=["working", "knowledge"]))
            assert ctx.chunks and ctx.total_tokens <= 500
        finally:
            await _stop(servers)
    run(go())


# ------------------------------------------------------------------------------------ goal -> plan -> execute
def test_goal_heuristic_path_completes(tmp_path):
    """A reactive goal runs through the heuristic executor and the real tool service."""
    async def go():
        from aios_amd.orchestrator.autonomy import AutonomyLoop

        st, servers, addrs, _ = await _start(tmp_path)
        try:
            o = _orch(addrs)
            gid = (await o.SubmitGoal(pb.orchestrator.SubmitGoalRequest(description="report cpu usage status",
                                                                        priority=3))).id
            s = await o.GetGoalStatus(pb.common.GoalId(id=gid))
            assert len(s.tasks) == 1 and s.tasks[0].intelligence_level == "reactive"
            loop = AutonomyLoop(st)
            for _ in range(40):
                await loop.tick()
                await asyncio.sleep(0.05)
                if st.goal_engine.goal(gid)["status"] == "completed":
                    break
            s = await o.GetGoalStatus(pb.common.GoalId(id=gid))
            assert s.goal.status == "completed", (s, st.goal_engine.messages(gid, 20))
            out = json.loads(s.tasks[0].output_json)
            assert out["tool_results"][0]["tool"].startswith("monitor.")
            assert s.progress_percent == 100.0
        finally:
            await _stop(servers)
    run(go())


def test_goal_ai_decomposition_and_reasoning(tmp_path):
    """Tactical goal: AI plan from the runtime, then a reasoning round with real tool calls."""
    plan = [{"description": "gather cpu metrics for the report", "tools": ["monitor"]},
            {"description": "summarise memory use for the report", "tools": ["monitor"]}]
    rt = ScriptedRuntime(plan=plan, calls=[{"tool": "monitor.memory", "input": {}}])

    async def go():
        from aios_amd.orchestrator.autonomy import AutonomyLoop

        st, servers, addrs, _ = await _start(tmp_path, runtime=rt)
        try:
            o = _orch(addrs)
            t0 = time.perf_counter()
            gid = (await o.SubmitGoal(pb.orchestrator.SubmitGoalRequest(
                description="prepare a report on resource usage of this machine", priority=5))).id
            plan_ms = (time.perf_counter() - t0) * 1000
            s = await o.GetGoalStatus(pb.common.GoalId(id=gid))
            assert [t.description for t in s.tasks] == [p["description"] for p in plan]
            assert list(s.tasks[1].depends_on) == [s.tasks[0].id]
            assert plan_ms < 5000
            loop = AutonomyLoop(st)
            for _ in range(100):
                await loop.tick()
                await asyncio.sleep(0.05)
                if st.goal_engine.goal(gid)["status"] in ("completed", "failed"):
                    break
            g = st.goal_engine.goal(gid)
            assert g["status"] == "completed", st.goal_engine.messages(gid, 50)
            prompts = [r.prompt for r in rt.requests]
            assert any("Available tools" in p for p in prompts)           # live catalog from the tool service
            assert any("Previous tool results" in p for p in prompts)     # multi-round reasoning (tactical)
            msgs = [m["content"] for m in st.goal_engine.messages(gid, 50)]
            assert any("monitor.memory" in m for m in msgs)
        finally:
            await _stop(servers)
    run(go())


def test_ai_unavailable_fails_task(tmp_path):
    async def go():
        from aios_amd.orchestrator.autonomy import AutonomyLoop

        st, servers, addrs, _ = await _start(tmp_path)
        try:
            g = st.goal_engine.submit("compose a haiku about kernels", 5, "user", [], b"")
            st.goal_engine.add_tasks(g["id"], [{"id": "t1", "description": "compose a haiku about kernels",
                                                "status": "pending", "intelligence_level": "operational",
                                                "required_tools": [], "depends_on": []}])
            loop = AutonomyLoop(st)
            for _ in range(40):
                await loop.tick()
                await asyncio.sleep(0.05)
                if st.goal_engine.task("t1")["status"] == "failed":
                    break
            assert st.goal_engine.task("t1")["status"] == "failed"
            assert st.goal_engine.goal(g["id"])["status"] == "failed"
        finally:
            await _stop(servers)
    run(go())


def test_agent_dispatch_and_report(tmp_path):
    async def go():
        from aios_amd.orchestrator.autonomy import AutonomyLoop

        st, servers, addrs, _ = await _start(tmp_path)
        try:
            o = _orch(addrs)
            C = pb.common
            await o.RegisterAgent(C.AgentRegistration(agent_id="sys-1", agent_type="system",
                                                      tool_namespaces=["service", "process", "monitor"]))
            assert [a.agent_id for a in (await o.ListAgents(C.Empty())).agents] == ["sys-1"]
            assert (await o.Heartbeat(pb.orchestrator.HeartbeatRequest(agent_id="sys-1", status="idle"))).success
            gid = (await o.SubmitGoal(pb.orchestrator.SubmitGoalRequest(description="restart the nginx service now"))).id
            await AutonomyLoop(st).tick()
            t = await o.GetAssignedTask(C.AgentId(id="sys-1"))
            assert t.id and t.goal_id == gid
            r = await o.ReportTaskResult(C.TaskResult(task_id=t.id, success=True, output_json=b'{"ok": true}'))
            assert r.success
            s = await o.GetGoalStatus(C.GoalId(id=gid))
            if len(s.tasks) == 1:
                assert s.goal.status == "completed"
            assert not (await o.GetAssignedTask(C.AgentId(id="nobody"))).id
            sysst = await o.GetSystemStatus(C.Empty())
            assert sysst.active_agents == 1 and sysst.memory_total_mb > 0
        finally:
            await _stop(servers)
    run(go())


def test_schedule_cluster_capability_rpcs(tmp_path):
    async def go():
        st, servers, addrs, tools = await _start(tmp_path)
        O, C = pb.orchestrator, pb.common
        try:
            o = _orch(addrs)
            sid = (await o.CreateSchedule(O.CreateScheduleRequest(cron_expr="*/5 * * * *", goal_template="rotate logs",
                                                                  priority=4))).schedule_id
            assert [e.id for e in (await o.ListSchedules(C.Empty())).schedules] == [sid]
            assert (await o.DeleteSchedule(O.DeleteScheduleRequest(schedule_id=sid))).success
            await o.RegisterNode(O.NodeRegistration(node_id="n2", hostname="h2", address="10.0.0.2:50051", max_tasks=4))
            assert (await o.NodeHeartbeat(O.NodeStatus(node_id="n2", cpu_usage=10.0, active_tasks=1))).success
            assert [n.node_id for n in (await o.ListNodes(O.ListNodesRequest())).nodes] == ["n2"]
            cr = await o.RequestCapability(O.CapabilityRequest(agent_id="web-agent", capabilities=["git_read"],
                                                               reason="clone docs"))
            assert cr.granted and cr.expires_at
            assert tools.core.check("web-agent", "git.status")["allowed"]
            deny = await o.RequestCapability(O.CapabilityRequest(agent_id="web-agent", capabilities=["self_update"]))
            assert not deny.granted and "critical" in deny.denial_reason
            gid = (await o.SubmitGoal(O.SubmitGoalRequest(description="check disk usage"))).id
            assert (await o.CancelGoal(C.GoalId(id=gid))).success
            lst = await o.ListGoals(O.ListGoalsRequest(status_filter="cancelled"))
            assert lst.total == 1
        finally:
            await _stop(servers)
    run(go())


# ------------------------------------------------------------------------------------ gateway
def test_gateway_local_provider_cache_stream_budget(tmp_path, monkeypatch):
    from aiohttp import web

    calls = {"n": 0}

    async def completions(req):
        body = await req.json()
        calls["n"] += 1
        if body.get("stream"):
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
            await resp.prepare(req)
            for piece in ["hel", "lo"]:
                await resp.write(f"data: {json.dumps({'choices': [{'delta': {'content': piece}}]})}\n\n".encode())
            await resp.write(b"data: [DONE]\n\n")
            return resp
        assert body["response_format"] == {"type": "json_object"}  # prompt asks for a JSON object
        return web.json_response({"model": "mistral-7b", "choices": [{"message": {"content": '{"ok": 1}'}}],
                                  "usage": {"prompt_tokens": 10, "completion_tokens": 5, "total_tokens": 15}})

    async def go():
        app = web.Application()
        app.router.add_post("/v1/chat/completions", completions)
        runner = web.AppRunner(app)
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        port = site._server.sockets[0].getsockname()[1]
        for k in ("CLAUDE_API_KEY", "OPENAI_API_KEY", "QWEN3_API_KEY"):
            monkeypatch.delenv(k, raising=False)
        monkeypatch.setenv("LOCAL_LLM_URL", f"http://127.0.0.1:{port}")
        from aios_amd.gateway.core import _Http
        from aios_amd.gateway.service import ApiGatewayService

        svc = ApiGatewayService.from_env(str(tmp_path / "usage.db"))
        srv = await RpcServer("127.0.0.1:0", {"aios.api_gateway.ApiGateway": svc}).start()
        try:
            g = Stub(channel(f"127.0.0.1:{srv.port}"), "aios.api_gateway.ApiGateway", timeout=10)
            req = pb.api_gateway.ApiInferRequest(prompt="reply with a JSON object", max_tokens=16, allow_fallback=True)
            r1 = await g.Infer(req)
            r2 = await g.Infer(req)
            assert r1.text == '{"ok": 1}' and r2.text == r1.text and calls["n"] == 1   # second one from cache
            chunks = [c async for c in g.StreamInfer(pb.api_gateway.ApiInferRequest(prompt="hi"))]
            assert "".join(c.text for c in chunks) == "hello" and chunks[-1].done and chunks[0].provider == "local"
            b = await g.GetBudget(pb.common.Empty())
            assert b.claude_monthly_budget_usd == 100 and b.openai_monthly_budget_usd == 50 and not b.budget_exceeded
            u = await g.GetUsage(pb.api_gateway.UsageRequest(provider="local", days=1))
            assert u.total_requests == 2 and u.records[0].input_tokens == 10
        finally:
            await srv.stop(0)
            await _Http.close()
            await runner.cleanup()
            await close_all()
    run(go())


def test_gateway_router_selection_and_fallback():
    from aios_amd.gateway.core import BudgetManager, Completion, Provider, ProviderError, RequestRouter

    class P(Provider):
        def __init__(self, name, avail=True, fail=False):
            self.name, self.avail, self.fail, self.n = name, avail, fail, 0

        def available(self):
            return self.avail

        async def infer(self, prompt, system_prompt, max_tokens, temperature):
            self.n += 1
            if self.fail:
                raise ProviderError(f"{self.name} down")
            return Completion(f"from {self.name}", 10, 1, self.name, 5, 5, self.name)

    provs = {"claude": P("claude", fail=True), "openai": P("openai", avail=False), "qwen3": P("qwen3"),
             "local": P("local")}
    r = RequestRouter(provs, BudgetManager())
    assert r.select("") == "claude"
    req = pb.api_gateway.ApiInferRequest(prompt="x", allow_fallback=True)
    c = asyncio.run(r.route(req))
    assert c.text == "from qwen3" and r.stats["fallbacks"] == 1
    req2 = pb.api_gateway.ApiInferRequest(prompt="y", allow_fallback=False)
    with pytest.raises(ProviderError):
        asyncio.run(r.route(req2))
    # cache: oldest evicted at capacity
    r.max_entries = 2
    for i in range(3):
        asyncio.run(r.route(pb.api_gateway.ApiInferRequest(prompt=f"p{i}", preferred_provider="local")))
    assert len(r.cache) == 2


# ------------------------------------------------------------------------------------ remote tools
def test_remote_tool_execution_on_cluster_node(tmp_path):
    """A tool call that names another cluster node runs on THAT node's tool service
    (RemoteExecutor.execute_remote_tool, reference agent-core/src/remote_exec.rs:75-102); an
    unknown node is a failed call, not a crash; goal forwarding uses the same executor."""
    from aios_amd.orchestrator.autonomy import AutonomyLoop
    from aios_amd.orchestrator.remote import tools_address_of
    from aios_amd.tools.service import ToolRegistryService

    async def go():
        st, servers, addrs, local_tools = await _start(tmp_path)
        class CountingTools(ToolRegistryService):
            seen = []

            async def Execute(self, req, ctx):
                self.seen.append(req.input_json)
                return await super().Execute(req, ctx)

        remote_tools = CountingTools(str(tmp_path / "remote_tools"))
        servers["remote_tools"] = await RpcServer("127.0.0.1:0", {"aios.tools.ToolRegistry": remote_tools}).start()
        try:
            st.cluster.register_node({"node_id": "worker-2", "hostname": "w2", "address": addrs["orchestrator"],
                                      "metadata": {"tools_address": f"127.0.0.1:{servers['remote_tools'].port}"},
                                      "max_tasks": 4})
            assert tools_address_of({"address": "10.0.0.7:50051"}) == "10.0.0.7:50052"
            loop = AutonomyLoop(st)
            p_remote, p_local = tmp_path / "remote.txt", tmp_path / "local.txt"
            calls = [{"tool": "fs.write", "input": {"path": str(p_remote), "content": "r"}, "node": "worker-2"},
                     {"tool": "fs.write", "input": {"path": str(p_local), "content": "l"}}]
            results, ok = await loop.run_tools("task-1", calls)
            assert ok and p_remote.read_text() == "r" and p_local.read_text() == "l"
            assert results[0]["node"] == "worker-2" and results[0]["success"]
            # the remote node's tool service executed the first call only
            assert len(remote_tools.seen) == 1 and b"remote.txt" in remote_tools.seen[0]
            bad, ok2 = await loop.run_tools("task-2", [{"tool": "monitor.cpu", "input": {}, "node": "nope"}])
            assert not ok2 and "not registered" in bad[0]["error"]
            # cluster goal forwarding through the same executor (to this node's own orchestrator)
            rid = await loop.remote.submit_remote_goal(addrs["orchestrator"], "forwarded goal", 5, "cluster:t")
            assert rid
        finally:
            await _stop(servers)
    run(go())


# ------------------------------------------------------------------------------------ event bus
def test_event_bus_producers_create_goals(tmp_path):
    """Events now have producers: a service whose health probes fail 3 times emits
    service_unhealthy (critical), which the default subscription turns into a recovery goal
    (source event_bus:service_unhealthy); its recovery emits service_recovered; failed agent
    tasks and goal completion are published too (reference bus: agent-core/src/event_bus.rs)."""
    from aios_amd.orchestrator.loops import EventQueue, HealthChecker
    from aios_amd.orchestrator.state import OrchestratorState

    async def go():
        st = OrchestratorState(str(tmp_path / "orch"), in_memory=True)
        st.event_queue = EventQueue(st)
        subs = st.install_default_subscriptions()
        assert len(subs) == 2
        stop = asyncio.Event()
        runner = asyncio.ensure_future(st.event_queue.run(stop))
        # a "service" on a port nobody listens on, then a real listener on the same port
        import socket
        s0 = socket.socket()
        s0.bind(("127.0.0.1", 0))
        port = s0.getsockname()[1]
        s0.close()
        hc = HealthChecker({"memory": f"127.0.0.1:{port}"}, timeout=0.5, grace=0,
                           on_change=lambda n, up, s: st.emit("service_recovered" if up else "service_unhealthy", n,
                                                              {"failures": s.consecutive_failures},
                                                              "info" if up else "critical"))
        for _ in range(3):
            await hc.check_all()
        srv = await asyncio.start_server(lambda r, w: w.close(), "127.0.0.1", port)
        await hc.check_all()
        srv.close()
        st.emit("task_failed", "agent-x", {"task_id": "t1"}, "warning")
        for _ in range(100):
            goals, _ = st.goal_engine.list("", 50, 0)
            if goals and st.event_queue.q.empty():
                break
            await asyncio.sleep(0.05)
        await asyncio.sleep(0.1)
        stop.set()
        await runner
        kinds = [e["event_type"] for e in st.events.recent(10)]
        assert "service_unhealthy" in kinds and "service_recovered" in kinds and "task_failed" in kinds
        assert kinds.count("service_unhealthy") == 1  # debounced: one event per outage
        goals, _ = st.goal_engine.list("", 50, 0)
        assert len(goals) == 1 and "memory" in goals[0]["description"]
        assert goals[0]["source"] == "event_bus:service_unhealthy" and goals[0]["priority"] == 9
    run(go())

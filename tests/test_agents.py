"""Python agents against the real control plane (CPU): registration, task polling, tool calls
through the capability checker, result reporting, DAG execution, orchestrator client."""
import asyncio
import json

import pytest

from aios_amd.agents import AGENT_REGISTRY
from aios_amd.agents.base import AgentConfig, extract_json
from aios_amd.agents.task import validate_plan
from aios_amd.rpc.client import close_all

from test_control_plane import _start, _stop, run


def test_registry_and_namespaces():
    assert set(AGENT_REGISTRY) == {"system", "task", "network", "security", "package", "storage", "monitoring",
                                   "learning", "creator", "web"}
    for t in AGENT_REGISTRY:
        a = AGENT_REGISTRY[t](agent_id=f"{t}-agent")
        assert a.get_agent_type() == t and a.get_capabilities()
        for _, method in a.ACTIONS:
            assert hasattr(a, method), (t, method)


def test_extract_json_and_plan_validation():
    assert extract_json('<think>x</think>```json\n{"a": [1, {"b": "}"}]}\n```') == {"a": [1, {"b": "}"}]}
    assert extract_json("steps: [1, 2] done") == [1, 2]
    assert extract_json("nothing") is None
    plan = validate_plan([{"id": "a", "depends_on": ["b"]}, {"id": "b", "depends_on": ["a"]},
                          {"id": "c", "depends_on": ["a", "zzz"]}] + [{"id": f"x{i}"} for i in range(30)])
    assert len(plan) == 20
    ids = [s["id"] for s in plan]
    pos = {s: i for i, s in enumerate(ids)}
    for s in plan:  # topological and acyclic
        assert all(pos[d] < pos[s["id"]] for d in s["depends_on"])
    assert plan[ids.index("c")]["depends_on"] == ["a"]


def _cfg(addrs):
    return AgentConfig(orchestrator_addr=addrs["orchestrator"], tools_addr=addrs["tools"],
                       memory_addr=addrs["memory"], runtime_addr=addrs["runtime"], grpc_timeout_s=10)


def test_system_agent_end_to_end(tmp_path):
    async def go():
        from aios_amd.orchestrator.autonomy import AutonomyLoop
        from aios_amd.agents.system import SystemAgent

        st, servers, addrs, _ = await _start(tmp_path)
        try:
            agent = SystemAgent(agent_id="system-agent", config=_cfg(addrs))
            assert await agent.register_with_orchestrator()
            assert await agent.send_heartbeat()
            g = await st.submit_goal("report cpu and memory usage metrics", 3, "user")
            tasks = st.goal_engine.tasks_for_goal(g["id"])
            assert tasks and "monitor" in tasks[0]["required_tools"]
            await AutonomyLoop(st).tick()
            assert st.goal_engine.task(tasks[0]["id"])["assigned_agent"] == "system-agent"
            assert await agent.poll_once()
            t = st.goal_engine.task(tasks[0]["id"])
            assert t["status"] == "completed", t
            out = json.loads(t["output_json"])
            assert out["success"] and 0 <= out["cpu_percent"] <= 100 and out["overall"] in ("ok", "warning",
                                                                                             "critical")
            assert agent.tasks_completed == 1
            assert not await agent.poll_once()  # nothing left
            # memory helpers round-trip through the memory service
            await agent.store_memory("k", {"v": 1})
            await agent.store_memory("k2", 2)
            assert await agent.recall_memory("k") == {"v": 1} and await agent.recall_memory("k2") == 2
            assert await agent.get_metric("system.cpu_percent") is not None
        finally:
            await _stop(servers)
    run(go())


def test_task_agent_runs_dag_with_tools(tmp_path):
    async def go():
        from aios_amd.agents.task import TaskAgent

        st, servers, addrs, tools = await _start(tmp_path)
        try:
            tools.core.grant("task-agent-x", ["monitor_read", "fs_read", "fs_write"])
            agent = TaskAgent(agent_id="task-agent-x", config=_cfg(addrs))
            f = tmp_path / "note.txt"
            plan = [{"id": "cpu", "tool": "monitor.cpu", "input": {}},
                    {"id": "mem", "tool": "monitor.memory", "input": {}},
                    {"id": "write", "tool": "fs.write", "input": {"path": str(f), "content": "ok"},
                     "depends_on": ["cpu", "mem"]},
                    {"id": "bad", "tool": "fs.read", "input": {"path": str(tmp_path / "missing")},
                     "depends_on": ["write"], "can_fail": True}]
            r = await agent.execute_task({"id": "t1", "description": "collect", "input": {"plan": plan}})
            assert r["success"], r
            assert f.read_text() == "ok"
            assert set(r["results"]) == {"cpu", "mem", "write", "bad"} and not r["results"]["bad"]["success"]
            plan[3]["can_fail"] = False
            r2 = await agent.execute_task({"id": "t2", "description": "collect", "input": {"plan": plan}})
            assert not r2["success"]
        finally:
            await _stop(servers)
    run(go())


def test_orchestrator_client(tmp_path):
    async def go():
        from aios_amd.agents.orchestrator_client import OrchestratorClient

        st, servers, addrs, _ = await _start(tmp_path)
        try:
            c = OrchestratorClient(addrs["orchestrator"], timeout=10)
            gid = await c.submit_goal("check disk usage", priority=2, metadata={"preferred_provider": "local"})
            s = await c.get_goal_status(gid)
            assert s["goal"]["id"] == gid and s["tasks"]
            assert st.preferred_provider(gid) == "local"
            assert (await c.list_goals())["total"] == 1
            assert await c.register_agent("w-1", "web", ["web.scrape"])
            assert [a["agent_id"] for a in await c.list_agents()] == ["w-1"]
            assert await c.cancel_goal(gid)
            done = await c.wait_for_goal(gid, timeout=5, poll_interval=0.1)
            assert done["goal"]["status"] == "cancelled"
            sysst = await c.get_system_status()
            assert sysst["memory_total_mb"] > 0
        finally:
            await _stop(servers)
    run(go())

"""CPU tests for the native control-plane core (aios_amd/native -> aios_amd._core).

Mirrors the reference's in-crate unit tests: tools/src/{registry,capabilities,
audit,rate_limit,backup,sandbox}.rs, memory/src/*.rs, agent-core/src/{goal_engine,task_planner,
autonomy,agent_router,cluster,scheduler,event_bus,decision_logger}.rs.
"""
import json
import os
import sqlite3
import time

import pytest

from aios_amd.core import load

c = load()


def _exec(svc, tool, agent="task-agent", **inp):
    r = svc.execute(tool, agent, "t", json.dumps(inp).encode(), "test")
    out = json.loads(r["output_json"]) if r["output_json"] else None
    return r, out


@pytest.fixture
def svc(tmp_path):
    return c.ToolService(str(tmp_path / "data"), "/root/repo")


# ------------------------------------------------------------------------------------ tools
def test_registry_has_all_builtin_tools(svc):
    names = {d["name"] for d in svc.list_tools("")}
    assert svc.tool_count() == len(names) == 88
    per_ns = {}
    for n in names:
        per_ns[n.split(".")[0]] = per_ns.get(n.split(".")[0], 0) + 1
    assert per_ns == {"fs": 13, "process": 6, "service": 5, "net": 5, "firewall": 3, "pkg": 5, "sec": 10,
                      "monitor": 7, "hw": 1, "web": 5, "git": 10, "code": 2, "self": 4, "plugin": 5,
                      "container": 6, "email": 1}
    fsw = svc.get_tool("fs.write")
    assert fsw["reversible"] and fsw["risk_level"] == "medium"
    assert svc.get_tool("nope.nothing") is None


def test_capabilities_per_principal(svc):
    assert len(c.ToolService.all_capabilities()) == 30
    assert svc.check("autonomy-loop", "fs.delete")["allowed"]
    assert svc.check("monitoring-agent", "monitor.cpu")["allowed"]
    d = svc.check("monitoring-agent", "fs.delete")
    assert not d["allowed"] and d["missing"]
    assert not svc.check("stranger", "fs.read")["allowed"]
    svc.grant("stranger", ["fs_read"])
    assert svc.check("stranger", "fs.read")["allowed"]
    assert svc.revoke("stranger", ["fs_read"]) == 1
    assert not svc.check("stranger", "fs.read")["allowed"]


def test_fs_write_read_and_rollback(svc, tmp_path):
    p = tmp_path / "hello.txt"
    r, out = _exec(svc, "fs.write", path=str(p), content="hi there")
    assert r["success"], r["error"]
    assert p.read_text() == "hi there"
    r2, out2 = _exec(svc, "fs.read", path=str(p))
    assert r2["success"] and out2["content"] == "hi there"
    ok, err = svc.rollback(r["execution_id"])
    assert ok, err
    assert not p.exists()  # file created by the tool is removed on rollback


def test_rollback_restores_previous_content(svc, tmp_path):
    p = tmp_path / "cfg.txt"
    p.write_text("original")
    r, _ = _exec(svc, "fs.write", path=str(p), content="changed")
    assert r["success"] and r["backup_id"]
    assert p.read_text() == "changed"
    ok, err = svc.rollback(r["execution_id"])
    assert ok, err
    assert p.read_text() == "original"


def test_denied_and_unknown_tools_fail_cleanly(svc):
    r, _ = _exec(svc, "fs.delete", agent="monitoring-agent", path="/tmp/x")
    assert not r["success"] and "denied" in r["error"].lower()
    r, _ = _exec(svc, "no.such_tool")
    assert not r["success"]
    r, _ = _exec(svc, "fs.read")  # missing required field
    assert not r["success"] and "path" in r["error"]


def test_audit_chain_verifies_and_detects_tampering(svc, tmp_path):
    for i in range(5):
        _exec(svc, "fs.stat", path=str(tmp_path))
    assert svc.audit_count() >= 5
    assert svc.audit_verify()
    rows = svc.audit_query(tool="fs.stat", limit=10)
    assert len(rows) == 5 and all(r["tool_name"] == "fs.stat" for r in rows)
    db = tmp_path / "data" / "ledger" / "audit.db"
    con = sqlite3.connect(db)
    con.execute("UPDATE audit_log SET agent_id = 'evil' WHERE rowid = (SELECT MIN(rowid) FROM audit_log)")
    con.commit()
    con.close()
    fresh = c.ToolService(str(tmp_path / "data"), "")
    assert not fresh.audit_verify()


def test_rate_limit_agent_burst(svc, tmp_path):
    # agent bucket: 10 rps with a burst of 2x -> a tight loop of 40 calls must see denials
    denied = 0
    for _ in range(40):
        r, _ = _exec(svc, "fs.stat", agent="monitoring-agent", path=str(tmp_path))
        denied += (not r["success"]) and "rate" in r["error"].lower()
    assert 10 <= denied <= 25


def test_monitor_and_hw_tools(svc):
    r, out = _exec(svc, "monitor.cpu", agent="monitoring-agent")
    assert r["success"], r["error"]
    assert 0.0 <= out["percent"] <= 100.0 and out["cores"] >= 1 and len(out["load_avg"]) == 3
    r, out = _exec(svc, "monitor.memory", agent="monitoring-agent")
    assert r["success"] and out["total_mb"] > 0
    r, out = _exec(svc, "process.list", agent="monitoring-agent")
    assert r["success"] and any(p["pid"] == 1 for p in out["processes"])
    r, out = _exec(svc, "hw.info")
    assert r["success"] and out["cores"] >= 1 and out["ram_mb"] > 0 and "gpus" in out


def test_plugin_create_execute_and_chain(svc, tmp_path):
    code = "def main(input_data):\n    return {'doubled': input_data.get('x', 0) * 2}\n"
    r, out = _exec(svc, "plugin.create", name="doubler", description="x*2", code=code)
    assert r["success"], r["error"]
    assert out["tool_name"] == "plugin.doubler"
    assert svc.get_tool("plugin.doubler") is not None
    r, out = _exec(svc, "plugin.doubler", x=21)
    assert r["success"], r["error"]
    assert out["doubled"] == 42
    bad = c.plugin_validate("import os\nos.system('rm -rf /')\neval(x)\nos.setuid(0)\n")
    assert not bad["safe"] and bad["risk_score"] >= 70 and len(bad["findings"]) == 3
    mid = c.plugin_validate("import os\nos.system('ls')\n")
    assert mid["safe"] and mid["risk_score"] == 30
    good = c.plugin_validate(code)
    assert good["safe"]
    r, out = _exec(svc, "plugin.list")
    assert r["success"] and out["count"] == 1
    r, _ = _exec(svc, "plugin.delete", name="doubler")
    assert r["success"] and svc.get_tool("plugin.doubler") is None


def test_sandbox_limits():
    r = c.sandbox_exec("python3", ["-c", "print('ok')"], "", 10000, 0)
    assert r["success"] and r["output"].strip() == "ok"
    r = c.sandbox_exec("python3", ["-c", "import time; time.sleep(5)"], "", 500, 0)
    assert not r["success"]
    r = c.sandbox_exec("python3", ["-c", "x = bytearray(900*1024*1024)"], "", 10000, 64 << 20)
    assert not r["success"]


def test_run_cmd_no_shell():
    r = c.run_cmd(["echo", "a;b", "$HOME"])
    assert r["exit_code"] == 0 and r["stdout"] == b"a;b $HOME\n"
    r = c.run_cmd(["sleep", "5"], timeout_ms=200)
    assert r["timed_out"]


# ------------------------------------------------------------------------------------ memory
@pytest.fixture
def mem(tmp_path):
    return c.MemoryStore(str(tmp_path / "w.db"), str(tmp_path / "lt.db"), str(tmp_path / "kn.db"))


def test_embedding_and_relevance():
    a = c.hashed_embedding("restart the nginx service")
    b = c.hashed_embedding("restart nginx service now")
    d = c.hashed_embedding("compile the kernel module")
    assert len(a) == 64
    assert abs(sum(x * x for x in a) - 1.0) < 1e-4
    assert c.cosine(a, b) > c.cosine(a, d)
    assert c.keyword_relevance(["nginx", "restart"], "Restart NGINX please") == pytest.approx(1.0)
    assert c.estimate_tokens("x" * 400) == 100


def test_operational_ring_and_metrics(mem):
    for i in range(12):
        mem.push_event({"id": f"e{i}", "category": "cpu" if i % 2 else "disk", "source": "mon", "data_json": "{}"})
    ev = mem.recent_events(5, "cpu", "")
    assert len(ev) == 5 and all(e["category"] == "cpu" for e in ev)
    mem.update_metric("cpu.usage", 42.5, 1000)
    assert mem.get_metric("cpu.usage") == (42.5, 1000)
    assert mem.get_metric("missing") is None


def test_working_goals_patterns(mem):
    mem.store_goal({"id": "g1", "description": "check disk", "status": "in_progress", "priority": 3})
    assert [g["id"] for g in mem.active_goals()] == ["g1"]
    mem.store_task({"id": "t1", "goal_id": "g1", "description": "df", "status": "completed"})
    mem.store_tool_call({"id": "c1", "task_id": "t1", "tool_name": "monitor.disk", "success": True})
    mem.update_goal("g1", "completed", "ok")
    assert mem.active_goals() == []
    mem.store_pattern({"id": "p1", "trigger": "disk full", "action": "clean /tmp", "success_rate": 0.9, "uses": 3})
    p = mem.find_pattern("disk full", 0.5)
    assert p["id"] == "p1"
    assert mem.find_pattern("disk full", 0.95) == {} or mem.find_pattern("disk full", 0.95) is None or \
        mem.find_pattern("disk full", 0.95)["id"] == ""


def test_knowledge_search_and_context(mem):
    mem.add_knowledge({"title": "nginx restart", "content": "use systemctl restart nginx", "source": "doc",
                       "tags": ["web"]})
    mem.add_knowledge({"title": "disk cleanup", "content": "remove old logs from /var/log", "source": "doc",
                       "tags": ["disk"]})
    hits = mem.search_knowledge("how to restart nginx", 5, 0.0)
    assert hits and "nginx" in hits[0]["content"]
    assert hits[0]["relevance"] >= hits[-1]["relevance"]
    ctx = mem.assemble_context("restart nginx", 1000, ["knowledge"])
    assert ctx["chunks"] and "nginx" in ctx["chunks"][0]["content"]
    assert ctx["total_tokens"] == sum(ch["tokens"] for ch in ctx["chunks"]) <= 1000
    tiny = mem.assemble_context("restart nginx", 3, ["knowledge"])
    assert tiny["total_tokens"] <= 3


def test_longterm_semantic_search_and_migration(mem):
    mem.store_procedure({"id": "pr1", "name": "rotate logs", "description": "rotate nginx logs weekly",
                         "steps_json": "[]", "success_count": 3})
    mem.store_incident({"id": "i1", "description": "nginx crashed out of memory", "resolution": "raised limits"})
    res = mem.semantic_search("nginx logs", ["procedures", "incidents"], 5, 0.0)
    assert {r["collection"] for r in res} <= {"procedures", "incidents"} and res
    old = int(time.time()) - 7200
    mem.store_goal({"id": "g9", "description": "old goal", "status": "completed", "created_at": old - 10,
                    "completed_at": old})
    out = mem.migrate(3600, 1000, 48 * 3600)
    assert out["goals_migrated"] >= 1
    st = mem.stats()
    assert st["procedures"] >= 2


def test_search_top_n_matches_full_sort(mem):
    """The scans keep only the n best rows; that must equal scoring every row (hybrid relevance from the
    exported helpers) and stable-sorting them -- ties (the duplicated texts) keep scan order."""
    texts = [f"{w} service on node {i % 7}" for i, w in enumerate(["nginx", "disk", "backup", "nginx logs"] * 12)]
    for i, t in enumerate(texts):
        mem.add_knowledge({"id": f"k{i:03d}", "title": t, "content": "runbook entry", "tags": []})
    q = "nginx logs on node 3"
    kws = q.split()
    qe = c.hashed_embedding(q)
    scored = []
    for i, t in enumerate(texts):
        content = f"{t}: runbook entry"
        r = 0.4 * c.keyword_relevance(kws, content + " ") + 0.6 * c.cosine(qe, c.hashed_embedding(t + " runbook entry "))
        scored.append((r, f"k{i:03d}"))
    scored.sort(key=lambda x: -x[0])  # stable
    for n in (1, 5, 13):
        hits = mem.search_knowledge(q, n, 0.0)
        assert [h["id"] for h in hits] == [k for _, k in scored[:n]]
        assert all(abs(h["relevance"] - r) < 1e-6 for h, (r, _) in zip(hits, scored))
    assert len(mem.search_knowledge(q, 5, 0.99)) == 0


def test_memory_persists_across_reopen(tmp_path):
    paths = [str(tmp_path / n) for n in ("w.db", "lt.db", "kn.db")]
    m1 = c.MemoryStore(*paths)
    m1.add_knowledge({"title": "persist", "content": "knowledge survives restart"})
    del m1
    m2 = c.MemoryStore(*paths)
    assert m2.search_knowledge("knowledge survives", 5, 0.0)


# ------------------------------------------------------------------------------------ planner / llm
def test_classify_levels():
    assert c.planner.classify("check nginx status") == "reactive"
    assert c.planner.classify("check disk usage") == "operational"
    assert c.planner.classify("check cpu usage") == "tactical"  # task_planner.rs default branch
    assert c.planner.classify("design a new distributed architecture for the database cluster") == "strategic"
    assert c.planner.classify("install nginx and then configure the firewall") in ("tactical", "strategic")


def test_decompose_chains_tasks():
    tasks = c.planner.decompose("g1", "install nginx, then configure the firewall, then restart nginx", "tactical")
    assert len(tasks) >= 2
    for prev, cur in zip(tasks, tasks[1:]):
        assert cur["depends_on"] == [prev["id"]]
    assert tasks[0]["intelligence_level"] == "operational"
    assert all(t["goal_id"] == "g1" and t["status"] == "pending" for t in tasks)


def test_parse_ai_decomposition():
    text = '<think>plan</think>[{"description": "check disk", "tools": ["monitor"]}, {"description": "clean", "tools": ["fs"]}]'
    tasks = c.planner.parse_ai_decomposition(text, "g", "tactical")
    assert [t["required_tools"] for t in tasks] == [["monitor"], ["fs"]]
    assert tasks[1]["depends_on"] == [tasks[0]["id"]]
    assert c.planner.parse_ai_decomposition("no json here", "g", "tactical") == []


def test_llm_parsing():
    assert c.llm.strip_think("<think>a</think>hello") == "hello"
    assert c.llm.extract_json('blah {"a": "}{", "b": [1, 2]} tail') == {"a": "}{", "b": [1, 2]}
    calls = c.llm.parse_tool_calls('```json\n{"tool_calls": [{"tool": "fs.read", "input": {"path": "/etc/hosts"}}]}\n```')
    assert calls == [{"tool": "fs.read", "input": {"path": "/etc/hosts"}}]
    calls = c.llm.parse_tool_calls('{"steps": [{"tool": "monitor.cpu", "input": {}}]}')
    assert calls[0]["tool"] == "monitor.cpu"
    assert c.llm.is_done_signal('{"done": true}')
    assert not c.llm.is_done_signal('{"done": false}')
    q = c.llm.parse_clarification('{"needs_clarification": true, "questions": ["which host?"]}')
    assert q and "which host" in q
    call = c.llm.explicit_tool_call('run tool monitor.cpu with {}')
    assert call is None or call["tool"] == "monitor.cpu"
    h = c.llm.heuristic_calls({"description": "check cpu usage", "required_tools": ["monitor"]})
    assert any(x["tool"].startswith("monitor.") for x in h)
    s = c.llm.summarize_tool_output("monitor.cpu", {"usage_percent": 12.5, "cores": 8})
    assert "12.5" in s


# ------------------------------------------------------------------------------------ orchestrator
def test_goal_engine_lifecycle(tmp_path):
    g = c.GoalEngine(str(tmp_path / "goals.db"))
    goal = g.submit("install nginx then restart it", 3, "user", ["web"], b"")
    assert goal["status"] == "pending"
    tasks = c.planner.decompose(goal["id"], goal["description"], "tactical")
    g.add_tasks(goal["id"], tasks)
    assert g.goal(goal["id"])["status"] == "in_progress"
    ready = g.next_tasks(10)
    assert [t["id"] for t in ready] == [tasks[0]["id"]]  # dependency chain gates the rest
    g.update_task({"id": tasks[0]["id"], "status": "completed"})
    if len(tasks) > 1:
        assert [t["id"] for t in g.next_tasks(10)] == [tasks[1]["id"]]
    for t in tasks[1:]:
        g.update_task({"id": t["id"], "status": "completed"})
    assert g.progress(goal["id"]) == 100.0
    assert g.check_completion(goal["id"]) == "completed"
    g.add_message(goal["id"], "user", "hello")
    assert g.messages(goal["id"], 10)[0]["content"] == "hello"
    lst, total = g.list("", 10, 0)
    assert total == 1 and lst[0]["id"] == goal["id"]


def test_goal_engine_persistence_and_resume(tmp_path):
    path = str(tmp_path / "goals.db")
    g = c.GoalEngine(path)
    goal = g.submit("a", 5, "user", [], b"")
    g.add_tasks(goal["id"], [{"id": "t1", "description": "x", "status": "in_progress", "required_tools": [],
                              "depends_on": []}])
    g.set_goal_metadata(goal["id"], "k", {"v": 1})
    del g
    g2 = c.GoalEngine(path)
    assert g2.goal(goal["id"])["description"] == "a"
    assert json.loads(g2.goal(goal["id"])["metadata_json"]) == {"k": {"v": 1}}
    assert g2.resume_in_progress() == 1
    assert g2.task("t1")["status"] == "pending"


def test_goal_cancel_and_failure(tmp_path):
    g = c.GoalEngine(":memory:")
    a = g.submit("a", 5, "user", [], b"")
    g.add_tasks(a["id"], [{"id": "ta", "description": "x", "status": "pending"}])
    assert g.cancel(a["id"]) and g.task("ta")["status"] == "cancelled"
    assert not g.cancel(a["id"])
    b = g.submit("b", 1, "user", [], b"")
    g.add_tasks(b["id"], [{"id": "tb", "description": "y", "status": "failed"}])
    assert g.check_completion(b["id"]) == "failed"
    assert g.counts()["total_goals"] == 2


def test_agent_router():
    r = c.AgentRouter(15)
    r.register({"agent_id": "sys1", "agent_type": "system", "capabilities": ["service.restart"],
                "tool_namespaces": ["service", "process"]})
    r.register({"agent_id": "net1", "agent_type": "network", "capabilities": [], "tool_namespaces": ["net"]})
    assert r.route({"required_tools": ["service"]}) == "sys1"
    assert r.route({"required_tools": ["net"]}) == "net1"
    assert r.route({"required_tools": ["git"]}) == ""
    r.assign("sys1", "t1")
    assert r.route({"required_tools": ["service"]}) == "sys1"  # busy but only capable agent
    r.task_completed("sys1", True)
    assert r.healthy_count() == 2 and r.dead_agents() == []
    assert r.unregister("net1") and not r.unregister("net1")


def test_cluster_least_loaded_and_discovery():
    cl = c.ClusterManager(30)
    cl.register_node({"node_id": "a", "address": "10.0.0.1", "max_tasks": 10})
    cl.register_node({"node_id": "b", "address": "10.0.0.2", "max_tasks": 10})
    cl.heartbeat("a", 80.0, 50.0, 5)
    cl.heartbeat("b", 10.0, 20.0, 1)
    assert cl.route_least_loaded() == "b"
    assert len(cl.list(False)) == 2
    d = c.Discovery(30)
    assert {s["name"] for s in d.list()} >= {"orchestrator", "tools", "memory", "api-gateway", "runtime"}
    assert d.lookup("tools")["port"] == 50052
    assert d.lookup("missing") == {}


def test_decision_log_ring():
    dl = c.DecisionLog(100)
    ids = [dl.log(f"ctx{i % 2}", ["a", "b"], "a", "because", "tactical", "m") for i in range(150)]
    assert len(dl) == 100
    for i in ids[-10:]:
        dl.update_outcome(i, "success")
    assert dl.success_rate("") == 1.0
    assert len(dl.recent(5)) == 5


def test_cron_and_schedule_store(tmp_path):
    t = 1_700_000_100  # 2023-11-14 22:15:00 UTC (a Tuesday)
    assert c.cron_matches("* * * * *", t)
    assert c.cron_matches("*/5 * * * *", t)
    assert c.cron_matches("15 22 * * *", t)
    assert c.cron_matches("0,15,30 22 14 11 2", t)
    assert not c.cron_matches("16 22 * * *", t)
    assert c.cron_matches("10-20 * * * *", t)
    assert not c.cron_valid("* * *") and c.cron_valid("*/10 2 * * 1")
    s = c.ScheduleStore(str(tmp_path / "sched.db"))
    sid = s.create("*/5 * * * *", "rotate logs", 4)
    with pytest.raises(Exception):
        s.create("bad", "x", 1)
    assert [e["id"] for e in s.due(t)] == [sid]
    assert s.due(t + 10) == []  # at most once per minute
    assert s.remove(sid) and s.list() == []


def test_event_bus_and_aggregator():
    b = c.EventBus()
    sid = b.subscribe("disk.*", "warning", "Investigate {event_type} from {source}: {message}", 2)
    assert b.publish({"event_type": "disk.full", "severity": "info", "source": "mon", "message": "x"}) == []
    goals = b.publish({"event_type": "disk.full", "severity": "critical", "source": "mon", "message": "95%"})
    assert goals == [{"description": "Investigate disk.full from mon: 95%", "priority": 2, "subscription_id": sid}]
    assert b.unsubscribe(sid)
    ra = c.ResultAggregator()
    ra.record("g", {"task_id": "t1", "success": True, "tokens_used": 10, "duration_ms": 5, "model_used": "m"})
    ra.record("g", {"task_id": "t2", "success": False, "tokens_used": 3, "duration_ms": 7})
    s = ra.summary("g")
    assert (s["successful"], s["failed"], s["total_tokens"], s["total_duration_ms"]) == (1, 1, 13, 12)


def test_system_prompt_budget():
    p = c.build_system_prompt("restart nginx", "tactical", ["service.restart"],
                              [{"trigger": f"t{i}", "action": "a" * 100} for i in range(100)], 200)
    assert "restart nginx" in p and "service.restart" in p
    assert c.estimate_tokens(p) <= 260

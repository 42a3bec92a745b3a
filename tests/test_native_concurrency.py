"""Concurrency of the native control-plane core: the gRPC daemons call into aios_amd._core from many
handler threads with the GIL released (bindings_core.cpp), so the C++ stores must be race-free on
their own.  These tests hammer one instance of each shared object from 8 threads and check the
end state; scripts/sanitize.sh --thread re-runs them against a ThreadSanitizer build of the core
(SURVEY.md §5 "race detection"; the reference relies on Rust's ownership rules for the same).
"""
import json
import threading

from aios_amd.core import load

c = load()
NT = 8


def _run(worker, n=NT):
    errs = []

    def wrap(i):
        try:
            worker(i)
        except Exception as e:  # noqa: BLE001 -- surfaced below
            errs.append(repr(e))

    ts = [threading.Thread(target=wrap, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errs, errs[:3]
    assert not any(t.is_alive() for t in ts)


def test_tool_service_parallel_execute(tmp_path):
    """8 threads through the whole pipeline (capability check -> rate limit -> backup -> handler ->
    audit append) at once: every call either runs with the right result or is refused by the rate
    limiter (one shared token bucket per agent and tool), the audit hash chain stays valid under
    concurrent appends and holds exactly one entry per executed call, and a burst from one agent
    never gets more calls through than the bucket holds."""
    svc = c.ToolService(str(tmp_path / "data"), str(tmp_path))
    per = 12
    ok = [0] * NT

    def worker(i):
        for k in range(per):
            p = tmp_path / f"f{i}_{k}.txt"
            r = svc.execute("fs.write", "autonomy-loop", f"t{i}", json.dumps({"path": str(p), "content": f"{i}:{k}"}).encode(),
                            "race")
            if not r["success"]:
                assert "rate limit" in r["error"].lower(), r
                continue
            ok[i] += 1
            r = svc.execute("fs.read", "autonomy-loop", f"t{i}", json.dumps({"path": str(p)}).encode(), "race")
            if r["success"]:
                out = r["output_json"]
                out = out.decode() if isinstance(out, bytes) else out
                assert f"{i}:{k}" in out
            else:
                assert "rate limit" in r["error"].lower(), r
            svc.check("monitoring-agent", "monitor.cpu")
            if k % 4 == 0:
                svc.grant(f"agent{i}", ["fs_read"])
                svc.revoke(f"agent{i}", ["fs_read"])

    _run(worker)
    assert 0 < sum(ok) <= NT * per
    for i in range(NT):
        for k in range(per):
            p = tmp_path / f"f{i}_{k}.txt"
            assert not p.exists() or p.read_text() == f"{i}:{k}"
    assert svc.audit_verify()
    assert len(svc.audit_query(tool="fs.write", limit=10_000)) == sum(ok)

def test_memory_store_parallel(tmp_path):
    mem = c.MemoryStore(str(tmp_path / "w.db"), str(tmp_path / "lt.db"), str(tmp_path / "kn.db"))
    per = 25

    def worker(i):
        for k in range(per):
            mem.push_event({"id": f"e{i}_{k}", "category": "cpu", "source": f"w{i}", "data_json": "{}"})
            mem.update_metric(f"m{i}", float(k), 1000 + k)
            if k % 5 == 0:
                mem.add_knowledge({"title": f"doc {i} {k}", "content": f"restart service {i} step {k}", "source": "t"})
                mem.search_knowledge("restart service", 3, 0.0)
            mem.store_goal({"id": f"g{i}_{k}", "description": "x", "status": "in_progress", "priority": 1})
            mem.recent_events(5, "cpu", "")

    _run(worker)
    for i in range(NT):
        assert mem.get_metric(f"m{i}") == (float(per - 1), 1000 + per - 1)
    assert len(mem.active_goals()) == NT * per


def test_goal_engine_parallel_submit_and_complete(tmp_path):
    g = c.GoalEngine(str(tmp_path / "goals.db"))
    per = 10

    def worker(i):
        for k in range(per):
            goal = g.submit(f"goal {i}-{k}", 3, "user", [], b"")
            g.add_tasks(goal["id"], [{"id": f"t{i}_{k}", "description": "x", "status": "pending", "required_tools": [],
                                      "depends_on": []}])
            g.update_task({"id": f"t{i}_{k}", "status": "completed"})
            assert g.check_completion(goal["id"]) == "completed"
            g.next_tasks(4)
            g.counts()

    _run(worker)
    lst, total = g.list("", 1000, 0)
    assert total == NT * per
    assert all(x["status"] == "completed" for x in lst)


def test_router_bus_and_decision_log_parallel():
    r = c.AgentRouter(15)
    bus = c.EventBus()
    dl = c.DecisionLog(10_000)
    sid = bus.subscribe("disk.*", "warning", "{event_type}", 2)

    def worker(i):
        r.register({"agent_id": f"a{i}", "agent_type": "system", "capabilities": [], "tool_namespaces": ["service"]})
        for k in range(50):
            assert r.route({"required_tools": ["service"]})
            r.assign(f"a{i}", f"t{i}_{k}")
            r.task_completed(f"a{i}", True)
            out = bus.publish({"event_type": "disk.full", "severity": "critical", "source": "m", "message": ""})
            assert out and out[0]["subscription_id"] == sid
            dl.log(f"ctx{i}", ["a", "b"], "a", "r", "tactical", "m")

    _run(worker)
    assert r.healthy_count() == NT
    assert len(dl) == NT * 50

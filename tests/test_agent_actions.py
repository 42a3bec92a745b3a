"""Every agent's actions against the real control plane (CPU): tools service (capability checks
per agent principal), memory service and a scripted AIRuntime.  Reference: agent-core/python/
aios_agent/agents/*.py action sets.  Network / web actions use a local HTTP
server; nothing leaves the machine."""
import asyncio
import http.server
import json
import os
import threading

import pytest

from aios_amd.agents import AGENT_REGISTRY
from aios_amd.agents.base import AgentConfig

from test_control_plane import ScriptedRuntime, _start, _stop, run


@pytest.fixture(scope="module")
def http_url():
    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            b = b"<html><head><title>T1</title></head><body><p>hello page</p></body></html>"
            self.send_response(200)
            self.end_headers()
            self.wfile.write(b)

        def do_POST(self):
            d = self.rfile.read(int(self.headers.get("Content-Length", 0)))
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.end_headers()
            self.wfile.write(json.dumps({"echo": d.decode()}).encode())

        def log_message(self, *a):
            pass

    hs = http.server.ThreadingHTTPServer(("127.0.0.1", 0), H)
    threading.Thread(target=hs.serve_forever, daemon=True).start()
    yield f"http://127.0.0.1:{hs.server_address[1]}/page.html"
    hs.shutdown()


def _agents(tmp_path, body):
    async def go():
        st, servers, addrs, tools = await _start(tmp_path / "cp", runtime=ScriptedRuntime())
        cfg = AgentConfig(orchestrator_addr=addrs["orchestrator"], tools_addr=addrs["tools"],
                          memory_addr=addrs["memory"], runtime_addr=addrs["runtime"], grpc_timeout_s=10)
        try:
            def mk(t):
                return AGENT_REGISTRY[t](agent_id=f"{t}-agent", config=cfg)

            async def do(agent, desc, **inp):
                return await asyncio.wait_for(agent.execute_task({"id": desc[:8], "description": desc, "input": inp}),
                                              30)
            await body(mk, do)
        finally:
            await _stop(servers)
    run(go(), timeout=120)


def test_monitoring_agent(tmp_path):
    async def body(mk, do):
        a = mk("monitoring")
        m = await do(a, "collect metrics")
        assert m["success"] and 0 <= m["metrics"]["cpu.usage_percent"] <= 100 and "disk.usage_percent" in m["metrics"]
        for _ in range(3):
            await do(a, "collect metrics")
        rep = await do(a, "generate summary report")
        assert rep["report"]["memory.usage_percent"]["n"] == 4
        assert (await do(a, "check alerts"))["success"]
        assert (await do(a, "anomaly detection"))["anomalies"] == []  # < 10 samples: no z-scores yet
        fc = await do(a, "resource forecast")
        assert set(fc["forecast"]) <= {"cpu.usage_percent", "memory.usage_percent", "disk.usage_percent"}
        assert len((await do(a, "dashboard data"))["series"]["cpu.usage_percent"]) == 5
    _agents(tmp_path, body)


def test_storage_agent(tmp_path):
    src = tmp_path / "data"
    src.mkdir()
    (src / "f.txt").write_text("abc")

    async def body(mk, do):
        a = mk("storage")
        h = await do(a, "check disk health", path=str(tmp_path))
        assert h["success"] and h["status"] in ("ok", "warning", "critical")
        b = await do(a, "create backup", source=str(src), destination=str(tmp_path / "bk"))
        assert b["success"] and (tmp_path / "bk" / "f.txt").read_text() == "abc"
        mounts = (await do(a, "list mounts"))["mounts"]
        assert any(m["mountpoint"] == "/" for m in mounts)
        assert (await do(a, "capacity planning"))["success"]
    _agents(tmp_path, body)


def test_network_agent(tmp_path):
    async def body(mk, do):
        a = mk("network")
        assert "127.0.0.1" in (await do(a, "dns lookup", hostname="localhost"))["output"]["addresses"]
        assert (await do(a, "list interfaces"))["output"]["interfaces"]
        ps = await do(a, "port scan", host="127.0.0.1", ports=[1, 2])
        assert ps["success"] and ps["scanned"] == 2 and ps["open_ports"] == []
        dg = await do(a, "diagnose network")
        assert dg["success"] and "interfaces_up" in dg["findings"]
    _agents(tmp_path, body)


def test_security_agent(tmp_path):
    f = tmp_path / "f.txt"
    f.write_text("x")
    os.chmod(f, 0o600)

    async def body(mk, do):
        a = mk("security")
        sc = await do(a, "security scan")
        assert sc["success"] and isinstance(sc["findings"], list)
        pr = await do(a, "check permissions", path=str(f))
        assert pr["results"][str(f)]["mode"] == "600"
        au = await do(a, "audit logs")
        assert au["success"] and au["tool_audit"]["entries"]
        ic = await do(a, "intrusion check")
        assert ic["success"] and ic["intrusion_detected"] is False
        th = await do(a, "threat analysis")
        assert th["success"] and th["risk_score"] >= 0
    _agents(tmp_path, body)


def test_package_agent(tmp_path):
    async def body(mk, do):
        a = mk("package")
        li = await do(a, "list installed packages")
        assert li["success"], li
        se = await do(a, "search package zlib", query="zlib")
        assert se["success"] and se["output"]["packages"]
        info = await do(a, "package info apt", name="apt")
        assert info["success"] and any(p["name"] == "apt" for p in info["installed"])
    _agents(tmp_path, body)


def test_learning_agent(tmp_path):
    async def body(mk, do):
        a = mk("learning")
        assert (await do(a, "analyze patterns"))["success"]
        assert (await do(a, "tool effectiveness"))["success"]
        pa = await do(a, "performance analysis")
        assert pa["success"] and pa["system"]["memory_total_mb"] > 0
        assert (await do(a, "suggest improvements"))["success"]
    _agents(tmp_path, body)


def test_creator_agent(tmp_path):
    async def body(mk, do):
        a = mk("creator")
        sc = await do(a, "scaffold new project", name="p1", path=str(tmp_path / "proj"))
        assert sc["success"] and os.path.isdir(sc["output"]["path"])
        g = await do(a, "generate code for an add function", file_path=str(tmp_path / "gen" / "add.py"))
        assert g["success"], g
        compile((tmp_path / "gen" / "add.py").read_text(), "add.py", "exec")
        r = await do(a, "init repo", path=str(tmp_path / "repo"))
        assert r["success"] and len(r["commit"]) == 40, r
    _agents(tmp_path, body)


def test_web_agent(tmp_path, http_url):
    async def body(mk, do):
        a = mk("web")
        br = await do(a, "browse page", url=http_url)
        assert br["success"] and br["output"]["title"] == "T1"
        api = await do(a, "api call json", url=http_url, method="POST", body={"a": 1})
        assert api["success"] and json.loads(api["output"]["data"]["echo"]) == {"a": 1}
        dl = await do(a, "download file", url=http_url, path=str(tmp_path / "dl"))
        assert dl["success"] and (tmp_path / "dl" / "page.html").read_text().startswith("<html>")
        wh = await do(a, "notify webhook", url=http_url, payload={"k": 1})
        assert wh["success"] and wh["output"]["status"] == 200
        mon = await do(a, "monitor url", url=http_url)
        assert mon["up"] and mon["status"] == 200
    _agents(tmp_path, body)

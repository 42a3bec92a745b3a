"""Behaviour tests for the native tool handlers (aios_amd/native/tools_*.cpp), one per handler
family, run through the full pipeline (capability check -> rate limit -> backup -> handler ->
audit).  Reference I/O contracts: SURVEY.md §2.4 per-tool table (tools/src/<ns>/*.rs).

Network tools talk to a local HTTP server / listening socket; tools whose backend is absent in
this container (nft / iptables, podman, SMTP) must fail with a clear error, not crash.
"""
import http.server
import json
import os
import socket
import threading
import time

import pytest

from aios_amd.core import load

c = load()


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    root = tmp_path_factory.mktemp("tools")
    svc = c.ToolService(str(root / "data"), "/root/repo")
    n = [0]

    def ex(tool, **inp):
        # a fresh all-capability principal per call keeps the per-agent token bucket out of the way
        n[0] += 1
        agent = f"tester-{n[0]}"
        svc.grant(agent, c.ToolService.all_capabilities())
        r = svc.execute(tool, agent, "task-x", json.dumps(inp).encode(), "handler test")
        out = json.loads(r["output_json"]) if r["output_json"] else None
        return r, out

    class H(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            b = b"<html><head><title>T1</title></head><body><p>hello page</p></body></html>"
            self.send_response(200)
            self.send_header("Content-Type", "text/html")
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
    yield svc, ex, root, f"http://127.0.0.1:{hs.server_address[1]}/x"
    hs.shutdown()


def test_fs_family(env):
    svc, ex, root, _ = env
    w = root / "w"
    w.mkdir()
    (w / "a.txt").write_text("hello\nworld\n")
    r, out = ex("fs.list", path=str(w))
    assert r["success"] and out["entries"][0]["name"] == "a.txt" and out["entries"][0]["size"] == 12
    assert ex("fs.mkdir", path=str(w / "sub" / "deep"), recursive=True)[1] == {"created": True}
    assert ex("fs.copy", source=str(w / "a.txt"), destination=str(w / "b.txt"))[1] == {"copied": True}
    assert ex("fs.move", source=str(w / "b.txt"), destination=str(w / "sub" / "c.txt"))[1] == {"moved": True}
    assert (w / "sub" / "c.txt").read_text() == "hello\nworld\n" and not (w / "b.txt").exists()
    assert ex("fs.chmod", path=str(w / "a.txt"), mode="0640")[1] == {"changed": True}
    assert oct(os.stat(w / "a.txt").st_mode & 0o777) == "0o640"
    assert ex("fs.chown", path=str(w / "a.txt"), uid=os.getuid(), gid=os.getgid())[1] == {"changed": True}
    assert ex("fs.symlink", target=str(w / "a.txt"), link=str(w / "lnk"))[1] == {"created": True}
    assert os.readlink(w / "lnk") == str(w / "a.txt")
    m = ex("fs.search", directory=str(w), pattern="*.txt", max_depth=5)[1]["matches"]
    assert sorted(m) == sorted([str(w / "a.txt"), str(w / "sub" / "c.txt")])
    du = ex("fs.disk_usage", path=str(root))[1]
    assert du["total_bytes"] >= du["used_bytes"] > 0 and 0 <= du["usage_percent"] <= 100
    r, _ = ex("fs.read", path=str(w / "nope.txt"))
    assert not r["success"] and r["error"]


def test_process_family(env):
    _, ex, _, _ = env
    info = ex("process.info", pid=os.getpid())[1]
    assert info["pid"] == os.getpid() and info["threads"] >= 1 and "python" in info["name"]
    r, out = ex("process.spawn", command="sleep", args=["30"])
    pid = out["pid"]
    assert r["success"] and pid > 0
    assert ex("process.signal", pid=pid, signal="SIGSTOP")[1] == {"sent": True}
    assert ex("process.signal", pid=pid, signal="SIGCONT")[1] == {"sent": True}
    assert ex("process.kill", pid=pid, signal="SIGKILL")[1] == {"killed": True}
    for _ in range(50):  # reaped by the tool service's child handling, or gone
        try:
            os.kill(pid, 0)
            with open(f"/proc/{pid}/stat") as f:
                if f.read().split()[2] == "Z":
                    break
        except (ProcessLookupError, FileNotFoundError):
            break
        time.sleep(0.05)
    else:
        pytest.fail("process.kill did not end the process")
    r, _ = ex("process.cgroup", action="bogus", group_name="aios-test")
    assert not r["success"] and "unknown action" in r["error"]
    procs = ex("process.list")[1]["processes"]
    assert any(p["pid"] == os.getpid() for p in procs)


def test_network_and_web_family(env):
    _, ex, root, url = env
    assert any(i["name"] == "lo" or i["status"] in ("up", "down") for i in ex("net.interfaces")[1]["interfaces"])
    assert "127.0.0.1" in ex("net.dns", hostname="localhost")[1]["addresses"]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    s.listen()
    assert ex("net.port_scan", host="127.0.0.1", port=s.getsockname()[1])[1] == {"open": True}
    s.close()
    g = ex("net.http_get", url=url)[1]
    assert g["status"] == 200 and "hello page" in g["body"]
    hr = ex("web.http_request", url=url, method="POST", body='{"a":1}')[1]
    assert hr["status"] == 200 and json.loads(hr["body"])["echo"] == '{"a":1}' and hr["method"] == "POST"
    sc = ex("web.scrape", url=url)[1]
    assert sc["title"] == "T1" and "hello page" in sc["text"] and not sc["truncated"]
    wh = ex("web.webhook", url=url, payload={"k": "v"})[1]
    assert wh["success"] and json.loads(json.loads(wh["response_body"])["echo"]) == {"k": "v"}
    dst = root / "dl" / "page.html"
    dl = ex("web.download", url=url, destination=str(dst), create_dirs=True)[1]
    assert dl["success"] and dl["size_bytes"] == dst.stat().st_size == 73
    api = ex("web.api_call", url=url, method="POST", body={"q": 1})[1]
    assert api["success"] and json.loads(api["data"]["echo"]) == {"q": 1}


def test_security_family(env):
    _, ex, root, _ = env
    d = root / "sec"
    d.mkdir()
    (d / "f.txt").write_text("x")
    os.chmod(d / "f.txt", 0o640)
    cp = ex("sec.check_perms", path=str(d / "f.txt"))[1]
    assert cp["mode"] == "640" and not cp["writable_by_others"]
    base = ex("sec.file_integrity", mode="baseline", paths=[str(d)])[1]
    assert base["checked"] == 1 and not base["modified"]
    (d / "f.txt").write_text("changed")
    (d / "g.txt").write_text("new")
    chk = ex("sec.file_integrity", mode="check", paths=[str(d)])[1]
    assert chk["modified"] == [str(d / "f.txt")] and chk["new_files"] == [str(d / "g.txt")]
    g = ex("sec.grant", agent_id="web-agent", capabilities=["fs_write"], reason="t", duration_hours=1)[1]
    assert g["success"] and g["granted"] == ["fs_write"] and g["expires_at"]
    assert ex("sec.revoke", agent_id="web-agent", capabilities=["fs_write"])[1]["revoked_count"] == 1
    cg = ex("sec.cert_generate", service_name="svc", cert_dir=str(root / "certs"), validity_years=1)[1]
    assert cg["success"] and os.path.exists(cg["ca_cert_path"]) and os.path.exists(cg["server_key_path"])
    assert oct(os.stat(cg["server_key_path"]).st_mode & 0o777) == "0o600"
    rot = ex("sec.cert_rotate", service_name="svc", cert_dir=str(root / "certs"))[1]
    assert rot["backed_up"] and rot["regenerated"]
    assert ex("sec.scan", checks=["world_writable"])[1]["risk_level"] in ("none", "low", "medium", "high")
    assert "clean" in ex("sec.scan_rootkits")[1]
    # the audit chain saw every call above, in order, with the caller's task id
    au = ex("sec.audit", limit=200)[1]["entries"]
    names = [e["tool_name"] for e in au]
    assert "sec.file_integrity" in names and all(e["task_id"] == "task-x" for e in au)
    q = ex("sec.audit_query", tool_name="sec.check_perms", limit=5)[1]["entries"]
    assert q and all(e["tool_name"] == "sec.check_perms" for e in q)


def test_monitor_hw_pkg_family(env):
    _, ex, root, _ = env
    nw = ex("monitor.network")[1]
    assert "lo" in nw["interfaces"] and nw["interfaces"]["lo"]["rx_bytes"] >= 0
    assert "entries" in ex("monitor.logs", lines=5)[1]
    tr = ex("monitor.ebpf_trace", trace_type="syscalls", duration_secs=1)[1]
    assert tr["trace_type"] == "syscalls" and tr["events"]
    (root / "watched").mkdir()
    (root / "watched" / "x").write_text("1")
    fw = ex("monitor.fs_watch", path=str(root / "watched"), since_timestamp=0)[1]
    assert any(e["path"].endswith("/x") for e in fw["events"])
    hw = ex("hw.info")[1]
    assert hw["ram_mb"] > 0 and hw["cpu"]
    pk = ex("pkg.list_installed")[1]["packages"]
    assert any(p["name"] == "apt" for p in pk)
    assert ex("pkg.search", query="zlib")[1]["packages"]


def test_git_code_self_plugin_family(env):
    _, ex, root, _ = env
    repo = root / "repo"
    assert ex("git.init", path=str(repo))[1]["success"]
    (repo / "f.txt").write_text("1\n")
    assert ex("git.add", repo_path=str(repo), all=True)[1]["files_staged"] == ["f.txt"]
    cm = ex("git.commit", repo_path=str(repo), message="first", author="A <a@b.c>")[1]
    assert cm["success"] and len(cm["commit_hash"]) == 40
    br = ex("git.branch", repo_path=str(repo), action="create", name="dev")[1]
    assert "dev" in br["branches"]
    (repo / "f.txt").write_text("1\n2\n")
    st = ex("git.status", repo_path=str(repo))[1]
    assert not st["clean"] and "f.txt" in st["modified"]
    df = ex("git.diff", repo_path=str(repo))[1]
    assert "+2" in df["diff"] and df["files_changed"] == ["f.txt"]
    lg = ex("git.log", repo_path=str(repo), count=5)[1]["entries"]
    assert lg[0]["message"] == "first" and lg[0]["hash"] == cm["commit_hash"]
    cl = ex("git.clone", url=str(repo), destination=str(root / "clone"))[1]
    assert cl["success"] and (root / "clone" / "f.txt").read_text() == "1\n"
    assert ex("git.pull", repo_path=str(root / "clone"))[1]["success"]
    r, _ = ex("git.push", repo_path=str(root / "clone"), remote="origin", branch="nope")
    assert not r["success"] and "git push failed" in r["error"]
    sc = ex("code.scaffold", name="proj", project_type="python", path=str(root / "proj"))[1]
    assert sc["success"] and all(os.path.exists(f) for f in sc["files_created"])
    gen = ex("code.generate", file_path=str(root / "gen" / "x.py"), description="hello function", language="python",
             create_dirs=True)[1]
    assert gen["success"] and gen["lines"] > 0
    compile((root / "gen" / "x.py").read_text(), "x.py", "exec")
    ins = ex("self.inspect")[1]
    assert ins["version"] and any("aios-init" in x for x in ins["components"])
    hl = ex("self.health", check_services=False, check_disk=True)[1]
    assert hl["disk_ok"] and hl["uptime_seconds"] > 0
    pt = ex("plugin.from_template", template="file_processor", config={"name": "fp1"})[1]
    assert pt["success"] and pt["tool_name"] == "plugin.fp1"
    assert any(p["tool_name"] == "plugin.fp1" for p in ex("plugin.list")[1]["plugins"])


def test_absent_backends_fail_cleanly(env):
    _, ex, _, _ = env
    for tool, inp, needle in (("container.list", {}, "container runtime"),
                              ("email.send", {"to": "a@b.c", "subject": "s", "body": "b"}, "SMTP")):
        r, _ = ex(tool, **inp)
        assert not r["success"] and needle in r["error"]
    r, _ = ex("firewall.rules")
    assert r["success"] or "firewall backend" in r["error"]

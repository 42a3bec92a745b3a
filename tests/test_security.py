"""Security / plugin-runtime cores (native/security.cpp): TOML, secrets, firewall applicator,
JSON-schema validation of tool inputs, plugin triggers + hot reload, TLS certificates.
Reference behaviour: tools/src/{secrets,firewall_apply,schema}.rs, tools/src/plugin/{events,
triggers,mod}.rs, agent-core/src/tls.rs (their #[test]s are the model for these)."""
import json
import os
import time

import pytest

from aios_amd.core import load


@pytest.fixture(scope="module")
def C():
    return load()


# ---------------------------------------------------------------- TOML
def test_toml_tables_arrays_and_values(C):
    t = C.toml_parse("""
top = "x"  # comment
[a]
n = 1_000
f = 2.5
b = true
arr = [1, 2,
       3]
s = "hash # inside"
[a.sub]
k = 'lit'
[[items]]
name = "one"
[[items]]
name = "two"
tags = ["p", "q"]
inline = { x = 1, y = "z" }
""")
    assert t["top"] == "x"
    assert t["a"]["n"] == 1000 and t["a"]["f"] == 2.5 and t["a"]["b"] is True
    assert t["a"]["arr"] == [1, 2, 3] and t["a"]["s"] == "hash # inside"
    assert t["a"]["sub"]["k"] == "lit"
    assert [i["name"] for i in t["items"]] == ["one", "two"]
    assert t["items"][1]["tags"] == ["p", "q"] and t["items"][1]["inline"] == {"x": 1, "y": "z"}


def test_toml_reopened_table_keeps_keys(C):
    t = C.toml_parse("[a.b]\nx = 1\n[a]\ny = 2\n")
    assert t["a"]["b"]["x"] == 1 and t["a"]["y"] == 2


# ---------------------------------------------------------------- secrets
def test_secrets_load_get_wipe(C, tmp_path):
    p = tmp_path / "secrets.toml"
    p.write_text('master = "m1"\n[api_keys]\nclaude = "sk-ant"\nopenai = "sk-oai"\n')
    os.chmod(p, 0o644)
    s = C.SecretManager(str(p))
    assert s.load() == 3
    assert any("insecure permissions 644" in w for w in s.warnings())
    assert s.get("api_keys.claude") == "sk-ant" and s.get("master") == "m1"
    assert s.get("missing") is None
    keys = s.api_keys()
    assert keys["claude"] == "sk-ant" and keys["openai"] == "sk-oai"
    s.set("x", "y")
    assert len(s) == 4
    s.wipe()
    assert len(s) == 0 and s.get("master") is None
    assert s.get_or_reload("master") == "m1"  # reload on miss


def test_secrets_ttl_expiry_and_missing_file(C, tmp_path):
    p = tmp_path / "s.toml"
    p.write_text('k = "v"\n')
    os.chmod(p, 0o600)
    s = C.SecretManager(str(p), 0)  # TTL 0: every cached value is already expired
    s.load()
    assert s.warnings() == []
    assert s.get("k") is None
    m = C.SecretManager(str(tmp_path / "nope.toml"))
    assert m.load() == 0 and "not found" in m.warnings()[0]


# ---------------------------------------------------------------- firewall
RULES = """
[defaults]
input_policy = "drop"
forward_policy = "drop"
output_policy = "accept"

[[input]]
name = "est"
action = "accept"
state = ["established", "related"]
protocol = "all"

[[input]]
name = "ssh-lan"
action = "accept"
protocol = "tcp"
port = 22
source = "10.0.0.0/8"
description = "ssh from lan"

[[input]]
name = "no-spoof"
action = "drop"
source = "127.0.0.0/8"
interface = "!lo"

[[rules]]
name = "range"
action = "reject"
direction = "output"
protocol = "udp"
port_range = [6000, 6010]
"""


def test_firewall_nft_and_iptables_commands(C, tmp_path):
    p = tmp_path / "fw.toml"
    p.write_text(RULES)
    nft = C.FirewallApplicator(str(p), "nft")
    rules, pol = nft.load_config()
    assert [r["name"] for r in rules] == ["range", "est", "ssh-lan", "no-spoof"]
    assert pol == {"input": "drop", "forward": "drop", "output": "accept"}
    cmds = nft.dry_run()
    assert cmds[0] == "nft add table inet aios"
    assert "policy drop" in cmds[1] and "hook input" in cmds[1]
    assert "nft add rule inet aios output udp dport 6000-6010 reject" in cmds
    assert "nft add rule inet aios input ct state established,related accept" in cmds
    assert 'nft add rule inet aios input ip saddr 10.0.0.0/8 tcp dport 22 comment "ssh from lan" accept' in cmds
    assert 'nft add rule inet aios input iifname != "lo" ip saddr 127.0.0.0/8 drop' in cmds
    ipt = C.FirewallApplicator(str(p), "iptables")
    c2 = ipt.dry_run()
    assert "iptables -P INPUT DROP" in c2
    assert 'iptables -A INPUT -p tcp --dport 22 -s 10.0.0.0/8 -j ACCEPT -m comment --comment "ssh from lan"' in c2
    assert "iptables -A OUTPUT -p udp --dport 6000:6010 -j REJECT" in c2
    assert "iptables -A INPUT -m conntrack --ctstate ESTABLISHED,RELATED -j ACCEPT" in c2


def test_firewall_rollback_reverses_applied(C, tmp_path):
    p = tmp_path / "fw.toml"
    p.write_text(RULES)
    for backend, needle, repl in (("nft", "add rule", "delete rule"), ("iptables", "-A ", "-D ")):
        f = C.FirewallApplicator(str(p), backend)
        f.record_all_applied()
        assert f.applied_count() == 4
        rb = f.rollback_commands()
        assert len(rb) == 4 and all(repl in c and needle not in c for c in rb)
        assert "no-spoof" not in rb[0]  # newest first: the last rule comes first
        assert ("127.0.0.0/8" in rb[0])


def test_firewall_dry_apply_and_raw_rules(C, tmp_path):
    p = tmp_path / "fw.toml"
    p.write_text('default_policy = "drop"\n[[rules]]\nchain = "input"\nrule = "tcp dport 22 accept"\n')
    f = C.FirewallApplicator(str(p), "nft")
    r = f.apply(True)
    assert r["dry_run"] and r["rules"] == 1 and r["applied"] == 0
    assert "nft add rule inet aios input tcp dport 22 accept" in r["commands"]
    assert any("hook output" in c and "policy accept" in c for c in r["commands"])
    bad = tmp_path / "bad.toml"
    bad.write_text('[[rules]]\nname = "x"\naction = "explode"\n')
    with pytest.raises(RuntimeError, match="bad action"):
        C.FirewallApplicator(str(bad), "nft").dry_run()


def test_repo_firewall_config_parses(C):
    path = os.path.join(os.path.dirname(os.path.dirname(__file__)), "deploy/etc/aios/security/firewall-rules.toml")
    cmds = C.FirewallApplicator(path, "nft").dry_run()
    assert len(cmds) > 4 and all(c.startswith("nft add") for c in cmds)


# ---------------------------------------------------------------- schema
SCHEMA = {"type": "object", "required": ["path"], "additionalProperties": False,
          "properties": {"path": {"type": "string", "minLength": 1, "pattern": "^/"},
                         "recursive": {"type": "boolean"},
                         "mode": {"enum": ["0644", "0755"]},
                         "depth": {"type": "integer", "minimum": 0, "maximum": 10},
                         "tags": {"type": "array", "items": {"type": "string"}, "maxItems": 2}}}


def test_schema_validate_accepts_and_rejects(C):
    assert C.schema_validate({"path": "/etc", "recursive": True, "depth": 3, "tags": ["a"]}, SCHEMA) == []
    errs = C.schema_validate({"recursive": "yes", "depth": 2.5, "extra": 1, "tags": ["a", 1, "c"], "mode": "0777"},
                             SCHEMA)
    text = "\n".join(errs)
    assert "missing required property 'path'" in text
    assert "$.recursive: expected type boolean" in text
    assert "$.depth: expected type integer" in text
    assert "unexpected property 'extra'" in text
    assert "$.tags[1]: expected type string" in text and "more than maxItems" in text
    assert "not in enum" in text
    assert C.schema_validate({"path": "rel"}, SCHEMA) == ["$.path: does not match pattern ^/"]
    assert C.schema_validate(5, {"anyOf": [{"type": "string"}, {"type": "integer"}]}) == []
    assert C.schema_validate(5, {"oneOf": [{"type": "number"}, {"type": "integer"}]}) != []


def test_tool_pipeline_enforces_plugin_input_schema(C, tmp_path):
    svc = C.ToolService(str(tmp_path), "")
    code = "def main(input_data):\n    return {'echo': input_data.get('n')}\n"
    r = svc.execute("plugin.create", "autonomy-loop", "t", json.dumps(
        {"name": "echo_n", "description": "echo", "code": code}).encode(), "")
    assert r["success"], r["error"]
    meta_path = tmp_path / "plugins" / "echo_n.meta.json"
    meta = json.loads(meta_path.read_text())
    meta["input_schema"] = {"type": "object", "required": ["n"], "properties": {"n": {"type": "integer"}}}
    meta_path.write_text(json.dumps(meta))
    svc.deregister_tool("plugin.echo_n")
    svc.scan_plugins()
    bad = svc.execute("plugin.echo_n", "autonomy-loop", "t", b'{"n": "x"}', "")
    assert not bad["success"] and bad["error"].startswith("Input validation failed") and "$.n" in bad["error"]
    miss = svc.execute("plugin.echo_n", "autonomy-loop", "t", b"{}", "")
    assert "missing required property 'n'" in miss["error"]
    assert svc.get_tool("plugin.echo_n")["input_schema"]


# ---------------------------------------------------------------- triggers / hot reload
def test_trigger_checks(C, tmp_path):
    t0 = 1767225600  # 2026-01-01 00:00 UTC (a Thursday)
    assert C.trigger_check_cron("0 0 * * *", t0) and not C.trigger_check_cron("5 0 * * *", t0)
    assert not C.trigger_check_cron("not cron", t0)
    assert C.trigger_check_metric(91, ">", 90) and C.trigger_check_metric(90, ">=", 90)
    assert not C.trigger_check_metric(5, "<", 5) and C.trigger_check_metric(1, "!=", 2)
    assert not C.trigger_check_metric(1, "??", 0)
    assert C.trigger_check_log_pattern("ERROR disk full", r"ERROR\s+disk") and C.trigger_check_log_pattern("a(b", "a(b")
    f = tmp_path / "w"
    f.write_text("x")
    assert C.trigger_check_file_watch(str(f), 0) and not C.trigger_check_file_watch(str(f), int(time.time()) + 10)
    assert not C.trigger_check_file_watch(str(tmp_path / "none"), 0)


def test_trigger_store_persistence_and_due(C, tmp_path):
    db = str(tmp_path / "trig.db")
    s = C.TriggerStore(db)
    with pytest.raises(RuntimeError):
        s.add("p", "cron", {"expression": "bad"})
    with pytest.raises(RuntimeError):
        s.add("p", "unknown", {})
    c = s.add("plugin.a", "cron", {"expression": "*/5 * * * *"})
    m = s.add("plugin.b", "metric_threshold", {"metric": "cpu.usage", "operator": ">", "threshold": 90.0})
    lg = s.add("plugin.c", "log_pattern", {"pattern": "OOM", "log_path": "/var/log/x"})
    t = 1767225600
    fired = {x["id"] for x in s.due(t, {"cpu.usage": 95.0}, {"/var/log/x": ["ok", "kernel: OOM killer"]})}
    assert fired == {c, m, lg}
    assert {x["id"] for x in s.due(t + 30, {"cpu.usage": 10.0}, {})} == set()  # cron once per minute
    assert s.set_enabled(c, False)
    assert c not in {x["id"] for x in s.due(t + 300, {}, {})}
    del s
    s2 = C.TriggerStore(db)  # reloaded from SQLite
    got = {x["id"]: x for x in s2.list()}
    assert set(got) == {c, m, lg} and got[c]["enabled"] is False and got[m]["last_fired"] == t
    assert s2.remove(lg) and not s2.remove(lg)
    assert len(C.TriggerStore(db).list()) == 2


def test_plugin_watcher_detects_changes(C, tmp_path):
    w = C.PluginWatcher(str(tmp_path))
    (tmp_path / "a.py").write_text("x")
    first = w.poll()
    assert first["added"] == [] and first["total_files"] == 1  # first poll = baseline
    (tmp_path / "b.py").write_text("y")
    (tmp_path / "b.meta.json").write_text("{}")
    time.sleep(0.01)
    (tmp_path / "a.py").write_text("xx")
    r = w.poll()
    assert r["added"] == ["b"] and r["changed"] == ["a"] and r["removed"] == []
    (tmp_path / "a.py").unlink()
    assert w.poll()["removed"] == ["a"]


def test_plugin_runtime_hot_reload_and_trigger_dispatch(tmp_path):
    from aios_amd.tools.service import PluginRuntime

    C = load()
    svc = C.ToolService(str(tmp_path), "")
    rt = PluginRuntime(svc, str(tmp_path))
    rt.tick(0)
    code = "def main(input_data):\n    return {'got': input_data['trigger']['type']}\n"
    r = svc.execute("plugin.create", "autonomy-loop", "t", json.dumps(
        {"name": "react", "description": "d", "code": code}).encode(), "")
    assert r["success"]
    svc.deregister_tool("plugin.react")  # simulate a plugin dropped in by another process
    out = rt.tick(0)
    assert "react" in out["changes"]["added"] and svc.get_tool("plugin.react") is not None
    rt.triggers.add("react", "cron", {"expression": "* * * * *"})
    out = rt.tick(1767225600)
    assert len(out["fired"]) == 1 and rt.fired[-1]["success"], rt.fired
    os.unlink(tmp_path / "plugins" / "react.py")
    os.unlink(tmp_path / "plugins" / "react.meta.json")
    out = rt.tick(1767225600)
    assert "react" in out["changes"]["removed"] and svc.get_tool("plugin.react") is None


# ---------------------------------------------------------------- TLS
def test_tls_generate_verify_idempotent(C, tmp_path):
    d = str(tmp_path / "certs")
    m = C.TlsManager(d)
    assert not m.certs_exist()
    p = m.generate_self_signed("aios-runtime")
    assert p["generated"] and m.certs_exist()
    v = m.verify()
    assert v["ok"] and v["signed_by_ca"] and v["valid_now"] and v["key_matches"]
    assert oct(os.stat(p["server_key"]).st_mode & 0o777) == "0o600"
    before = open(p["server_cert"]).read()
    again = m.generate_self_signed("other")
    assert not again["generated"] and open(p["server_cert"]).read() == before
    # a server cert from a different CA fails verification
    other = C.TlsManager(str(tmp_path / "c2"))
    other.generate_self_signed("x")
    os.replace(other.paths()["ca_cert"], p["ca_cert"])
    assert not m.verify()["signed_by_ca"]

"""aios-init (C++): TOML config + defaults, topological start order, supervision with restart
policy and clean shutdown (reference initd/src/{main,service,config}.rs)."""
import json
import os
import signal
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def initd():
    from aios_amd import _build

    if os.environ.get("AIOS_INIT_BIN"):  # e.g. the ASan/UBSan build from scripts/sanitize.sh
        return os.environ["AIOS_INIT_BIN"]
    return str(_build.build_initd(verbose=False))


def test_default_config_and_order(initd):
    out = json.loads(subprocess.check_output([initd, "--check-config", "--config", "/nonexistent.toml"]))
    assert out["_config_file"] == "(defaults)"
    assert out["_start_order"][-1] == "aios-orchestrator" and len(out["_start_order"]) == 5
    assert out["services"]["aios-runtime"]["port"] == 50055
    assert out["models"]["strategic"]["tensor_parallel"] == 8


def test_repo_default_config_parses(initd):
    out = json.loads(subprocess.check_output([initd, "--check-config", "--config",
                                              os.path.join(ROOT, "config", "default-config.toml")]))
    assert out["_config_file"].endswith("default-config.toml")
    assert out["models"]["tactical"]["context_length"] == 4096
    assert out["api"]["claude_monthly_budget_usd"] == 100.0
    assert out["models"]["devices"] == [0]
    assert out["_unmet"] == []


def test_toml_overrides_and_unmet_deps(initd, tmp_path):
    cfg = tmp_path / "c.toml"
    cfg.write_text('''
[system]
hostname = "node-7"   # comment
[services.aios-runtime]
enabled = false
[services.extra]
command = ["sleep", "1"]
depends_on = ["missing-svc"]
[services.multi]
command = [
  "echo",
  "a, b",
]
''')
    out = json.loads(subprocess.check_output([initd, "--check-config", "--config", str(cfg)]))
    assert out["system"]["hostname"] == "node-7"
    assert "aios-runtime" not in out["_start_order"]
    assert "aios-orchestrator" in out["_unmet"] and "extra" in out["_unmet"]
    assert out["services"]["multi"]["command"] == ["echo", "a, b"]


def test_supervise_restart_and_shutdown(initd, tmp_path):
    marker = tmp_path / "starts"
    cfg = tmp_path / "c.toml"
    flaky = f"echo x >> {marker}; sleep 0.3; exit 3"
    cfg.write_text(f'''
[system]
data_dir = "{tmp_path}/data"
log_dir = "{tmp_path}/log"
[boot]
clean_shutdown_flag = "{tmp_path}/clean"
[supervisor]
check_interval_s = 1
max_restarts = 2
restart_window_s = 60
stop_timeout_s = 3
[services.aios-runtime]
enabled = false
[services.aios-memory]
enabled = false
[services.aios-tools]
enabled = false
[services.aios-api-gateway]
enabled = false
[services.aios-orchestrator]
enabled = false
[services.steady]
command = ["sleep", "100"]
[services.flaky]
command = ["sh", "-c", "{flaky}"]
''')
    p = subprocess.Popen([initd, "--config", str(cfg), "--no-mount"], stderr=subprocess.PIPE, text=True)
    time.sleep(6)
    p.send_signal(signal.SIGTERM)
    _, err = p.communicate(timeout=30)
    assert p.returncode == 0, err
    starts = marker.read_text().count("x")
    assert starts == 3, err  # initial + max_restarts
    assert "giving up" in err and "clean shutdown" in err
    assert (tmp_path / "clean").exists()
    assert json.loads((tmp_path / "data" / "hardware.json").read_text())["cpu_cores"] >= 1

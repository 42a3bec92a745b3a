"""The whole stack under aios-init (scripts/run-local.sh) on this machine: every gRPC service answers and a
submitted goal gets tasks -- tools/bench_boot.py with no model requirement (the GPU box run, with the
synthetic tiers loaded, is profiles/boot_r6.json)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ports_free():
    for p in (50051, 50052, 50053, 50054, 50055):
        with socket.socket() as s:
            if s.connect_ex(("127.0.0.1", p)) == 0:
                return False
    return True


def test_stack_boots_and_accepts_a_goal():
    if not os.path.exists(os.path.join(ROOT, "aios_amd", "bin", "aios-init")):
        pytest.skip("aios-init not built")
    if not _ports_free():
        pytest.skip("service ports in use")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_boot.py"), "--models", "0", "--timeout", "90"],
                       capture_output=True, text=True, timeout=240)
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert r.returncode == 0 and out["boot_to_autonomy_s"] is not None, out
    assert set(out["service_ready_s"]) == {"orchestrator", "tools", "memory", "api_gateway", "runtime"}
    assert out["boot_to_autonomy_s"] < 30 and out.get("tasks"), out
    assert _ports_free()  # the stack's process group was stopped


def test_memory_tier_bench_runs():
    """tools/bench_memory.py end to end at a small size: the daemon process over gRPC and the in-process
    handlers both answer every RPC of the three tiers (latencies are the GPU box's record,
    profiles/memory_tiers_r6.json; this machine's loopback is too noisy for the targets)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_memory.py"), "--calls", "5", "--entries", "20"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    for mode in ("rpc", "service"):
        assert set(out[mode]) == {"operational", "working", "long-term"}
        for tier in out[mode].values():
            assert all(c["p50_ms"] > 0 for c in tier["calls"].values())
    assert out["service"]["long-term"]["meets_target"]

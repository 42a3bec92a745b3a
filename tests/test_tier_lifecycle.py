"""Tier lifecycle of the model pool on CPU engines: on-demand load on the first request of a level,
idle unload back to the on-demand registry, replica groups with least-loaded routing, and the
node-config plan that drives them.  Reference: `load_on_demand` / `unload_after_idle_minutes`
(`/root/reference/initd/src/config.rs:108-109`), parsed but never acted on by its runtime."""
import asyncio

import pytest

from aios_amd.runtime.model_manager import ModelManager, RoutingError
from aios_amd.utils import config as node_config

SPEC = "synthetic:test-small:Q4_0#cpu"


def run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def test_on_demand_strategic_tier_loads_on_first_request():
    mgr = ModelManager(max_batch=2, max_slots=2)
    mgr.register_on_demand("llama3-70b-local", SPEC, 128)
    with pytest.raises(RoutingError) as e:
        mgr.resolve("", "strategic")  # nothing resident: the reference's error
    assert e.value.code == "FAILED_PRECONDITION"

    async def go():
        m = await mgr.resolve_async("", "strategic")
        assert m.name == "llama3-70b-local" and m.status == "ready"
        assert "llama3-70b-local" not in mgr.deferred
        # a second request routes to the resident engine without reloading
        m2 = await mgr.resolve_async("", "strategic")
        assert m2 is m and m.request_count == 2
        await mgr.unload_model(m.name)

    run(go())


def test_concurrent_first_requests_share_one_load():
    mgr = ModelManager(max_batch=2, max_slots=2)
    mgr.register_on_demand("mistral-7b-tier", SPEC, 128)
    loads = []
    orig = mgr.load_model

    async def counting(*a, **k):
        loads.append(a[0])
        return await orig(*a, **k)

    mgr.load_model = counting

    async def go():
        ms = await asyncio.gather(*[mgr.resolve_async("mistral-7b-tier", "") for _ in range(3)])
        assert all(m.status == "ready" for m in ms)
        assert loads == ["mistral-7b-tier"]
        await mgr.unload_model("mistral-7b-tier")

    run(go())


def test_idle_unload_returns_tier_to_on_demand_registry():
    mgr = ModelManager(max_batch=2, max_slots=2)
    unloaded = []

    async def hook(name):
        unloaded.append(name)

    mgr.unload_hooks.append(hook)

    async def go():
        ms = await mgr.load_replicas("tinyllama-1.1b", SPEC, 128, idle_unload_s=30.0)
        m = ms[0]
        assert m.status == "ready"
        assert await mgr.unload_idle(now=m.loaded_at + 10) == []       # still within the limit
        assert await mgr.unload_idle(now=m.loaded_at + 31) == ["tinyllama-1.1b"]
        assert unloaded == ["tinyllama-1.1b"] and "tinyllama-1.1b" in mgr.deferred
        # the next operational request reloads it with the same idle limit
        m2 = await mgr.resolve_async("", "operational")
        assert m2.name == "tinyllama-1.1b" and m2.idle_unload_s == 30.0
        await mgr.unload_model(m2.name)

    run(go())


def test_replica_group_least_loaded_routing():
    mgr = ModelManager(max_batch=2, max_slots=2)

    async def go():
        ms = await mgr.load_replicas("tinyllama-1.1b", SPEC, 128, devices=[0, 1])
        assert [m.name for m in ms] == ["tinyllama-1.1b", "tinyllama-1.1b@1"]
        assert all(m.status == "ready" and m.group == "tinyllama-1.1b" for m in ms)
        assert [m.device for m in ms] == [0, 1]
        picks = [mgr.resolve("", "operational").name for _ in range(4)]
        assert sorted(picks) == ["tinyllama-1.1b", "tinyllama-1.1b", "tinyllama-1.1b@1", "tinyllama-1.1b@1"]
        # load-aware: a replica with queued work is avoided
        busy = mgr.models["tinyllama-1.1b"]
        mgr._load_of = lambda m: 5.0 if m is busy else 0.0
        assert {mgr.resolve("tinyllama-1.1b", "").name for _ in range(3)} == {"tinyllama-1.1b@1"}
        for m in ms:
            await mgr.unload_model(m.name)

    run(go())


def test_config_tier_plan_and_tp_devices(tmp_path):
    p = tmp_path / "c.toml"
    p.write_text("""
[models]
model_dir = "/nonexistent"
[models.operational]
file = "synthetic:tinyllama-1.1b"
always_loaded = true
replicas = 2
[models.strategic]
file = "synthetic:llama3-70b"
tensor_parallel = 8
load_on_demand = true
unload_after_idle_minutes = 30
""")
    cfg = node_config.load(str(p), env={})
    plan = {t["name"]: t for t in cfg.tier_plan()}
    assert plan["operational"]["on_demand"] is False and plan["operational"]["devices"] == [0, 1]
    assert plan["strategic"]["on_demand"] is True and plan["strategic"]["spec"].endswith("#tp=8")
    assert plan["strategic"]["idle_unload_s"] == 1800.0
    # no explicit device list: TP ranks are not pinned (a default [0] put all 8 on GPU 0)
    assert cfg.tp_devices_env() == ""
    cfg2 = node_config.load(str(p), env={"AIOS_CFG__MODELS__DEVICES": "[0, 1]"})
    assert cfg2.models.devices == [0, 1] and cfg2.tp_devices_env() == ""  # 2 < tensor_parallel 8
    cfg3 = node_config.load(str(p), env={"AIOS_CFG__MODELS__DEVICES": "[0,1,2,3,4,5,6,7]"})
    assert cfg3.tp_devices_env() == "0,1,2,3,4,5,6,7"

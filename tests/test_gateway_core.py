"""Native api-gateway core (aios_amd/native/gateway.cpp): budget ledger, response cache, routing.

Reference behaviour: api-gateway/src/budget.rs (monthly budgets, 80 % warning, monthly reset),
router.rs:34-248 (TTL cache, oldest evicted, provider order, fallback chains), openai.rs:137.
"""
import calendar

import pytest

from aios_amd.core import load as load_core


@pytest.fixture(scope="module")
def gw():
    return load_core().gateway


def _t(y, m, d, hh=12):
    return calendar.timegm((y, m, d, hh, 0, 0))


def test_month_start_is_utc_first_of_month(gw):
    assert gw.BudgetLedger.month_start(_t(2026, 3, 17)) == _t(2026, 3, 1, 0)
    assert gw.BudgetLedger.month_start(_t(2026, 12, 31, 23)) == _t(2026, 12, 1, 0)


def test_budget_split_warning_exceeded_and_monthly_reset(gw):
    b = gw.BudgetLedger(10.0, 5.0)
    now = _t(2026, 3, 10)
    # no provider split -> 50/50 of tokens_used (the reference's estimate)
    assert b.record("claude", "m", 0, 0, 1001, 7.0, "agent", "task", now) == []
    u = b.usage("claude", 30, now)
    assert u["total_requests"] == 1 and u["records"][0]["input_tokens"] == 500
    assert u["records"][0]["output_tokens"] == 501 and u["records"][0]["requesting_agent"] == "agent"
    w = b.record("claude", "m", 10, 20, 30, 1.5, now=now + 1)  # 8.5 / 10 > 80 %
    assert len(w) == 1 and w[0].startswith("claude budget warning")
    assert not b.provider_exceeded("claude", now + 2)
    b.record("claude", "m", 1, 1, 2, 2.0, now=now + 3)
    assert b.provider_exceeded("claude", now + 4) and not b.exceeded(now + 4)  # openai still has budget
    assert not b.provider_exceeded("qwen3", now) and not b.provider_exceeded("local", now)
    st = b.status(now + 5)
    assert abs(st["claude_used_usd"] - 10.5) < 1e-9 and not st["budget_exceeded"]
    # next month: the counters restart, the records stay
    nxt = _t(2026, 4, 2)
    assert not b.provider_exceeded("claude", nxt) and b.used("claude", nxt) == 0
    assert b.usage("", 0, nxt)["total_requests"] == 3


def test_budget_persists_across_instances(gw, tmp_path):
    db = str(tmp_path / "gw" / "usage.db")
    b = gw.BudgetLedger(100.0, 50.0, db)
    b.record("openai", "gpt", 100, 50, 150, 0.25)
    del b
    b2 = gw.BudgetLedger(100.0, 50.0, db)
    assert abs(b2.used("openai") - 0.25) < 1e-12 and b2.usage("openai", 1)["total_tokens"] == 150


def test_cache_ttl_and_oldest_eviction(gw):
    c = gw.ResponseCache(10.0, 2)
    k = [gw.ResponseCache.key(f"p{i}", "sys") for i in range(3)]
    assert len(set(k)) == 3 and k[0] != gw.ResponseCache.key("p0", "other")
    assert k[0] == load_core().sha256_hex("p0\x00sys")
    c.put(k[0], gw.Completion("a", 1), 100.0)
    c.put(k[1], gw.Completion("b", 2), 101.0)
    c.put(k[2], gw.Completion("c", 3), 102.0)  # full: k0 (oldest) evicted
    assert len(c) == 2 and c.get(k[0], 103.0) is None and c.get(k[1], 103.0).text == "b"
    assert c.get(k[2], 111.9).tokens_used == 3
    assert c.get(k[2], 112.0) is None and len(c) == 1  # TTL expiry removes the entry


def test_routing_policy(gw):
    b = gw.BudgetLedger(1.0, 1.0)
    avail = {"claude": True, "openai": True, "qwen3": True}
    assert gw.select("", avail, b) == "claude"
    assert gw.select("local", avail, b) == "local"  # explicit provider wins
    b.record("claude", "m", 1, 1, 2, 5.0)
    assert gw.select("", avail, b) == "openai"
    assert gw.select("", {"claude": True, "openai": False, "qwen3": False}, b) == "local"
    assert gw.chain("claude", True) == ["claude", "openai", "qwen3", "local"]
    assert gw.chain("local", True) == ["local", "qwen3", "claude", "openai"]
    assert gw.chain("mystery", True) == ["mystery", "local"] and gw.chain("qwen3", False) == ["qwen3"]
    assert abs(gw.cost("claude", 1_000_000, 1_000_000) - 18.0) < 1e-9 and gw.cost("local", 10, 10) == 0
    assert gw.wants_json("Return a JSON object", "") and gw.wants_json("x", "respond with ONLY valid JSON")
    assert not gw.wants_json("plain text please", "")

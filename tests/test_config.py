"""Typed node config shared by the services (aios_amd/utils/config.py): defaults, the repo's
default-config.toml, both historical [api]/[api_gateway] schemas, env overrides, model-pool specs."""
import os

from aios_amd.utils import config as node_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_defaults_without_file():
    c = node_config.load("/nonexistent/config.toml", env={})
    assert c.source == "" and c.api.claude_monthly_budget_usd == 100.0 and c.monitoring.cpu_threshold == 90.0
    assert c.models.max_batch == 16 and c.model_specs() == []


def test_repo_default_config():
    c = node_config.load(os.path.join(ROOT, "config", "default-config.toml"), env={})
    assert c.source.endswith("default-config.toml") and not c.warnings
    assert set(c.models.tiers) == {"operational", "tactical", "strategic"}
    s = c.models.tiers["strategic"]
    assert s.tensor_parallel == 8 and s.load_on_demand and s.context_length == 8192
    assert c.agents.heartbeat_timeout_seconds == 15 and c.memory.context_max_tokens == 4000


def test_env_overrides_and_api_gateway_alias(tmp_path):
    p = tmp_path / "c.toml"
    p.write_text('[api_gateway]\nclaude_monthly_budget_usd = 7.5\n[monitoring]\ncpu_threshold = "bad"\n')
    c = node_config.load(str(p), env={"AIOS_CFG__MONITORING__DISK_THRESHOLD": "70",
                                      "AIOS_CFG__MODELS__MAX_BATCH": "32", "UNRELATED": "1"})
    assert c.api.claude_monthly_budget_usd == 7.5
    assert c.monitoring.disk_threshold == 70.0 and c.models.max_batch == 32
    assert c.monitoring.cpu_threshold == 90.0 and any("cpu_threshold" in w for w in c.warnings)


def test_model_specs_tp_cpu_and_missing_files(tmp_path):
    d = tmp_path / "models"
    d.mkdir()
    (d / "tiny.gguf").write_bytes(b"GGUF")
    p = tmp_path / "c.toml"
    p.write_text(f"""
[models]
model_dir = "{d}"
devices = [0, 1]
[models.operational]
file = "tiny.gguf"
always_loaded = true
context_length = 2048
device = "cpu"
[models.tactical]
file = "missing.gguf"
always_loaded = true
[models.strategic]
file = "synthetic:llama3-70b"
always_loaded = true
tensor_parallel = 8
[models.lazy]
file = "tiny.gguf"
load_on_demand = true
""")
    c = node_config.load(str(p), env={})
    specs = {t: (s, ctx) for t, s, ctx in c.model_specs()}
    assert specs["operational"] == (str(d / "tiny.gguf") + "#cpu", 2048)
    assert specs["strategic"][0] == "synthetic:llama3-70b#tp=8"
    assert "tactical" not in specs and "lazy" not in specs
    assert c.models.devices == [0, 1]


def test_cu_mask_words_balanced_and_disjoint():
    """co-resident tier CU masks: every aligned 32-CU group keeps CUs of both tiers (XCD-major or
    XCD-minor numbering alike), the two tiers never share a CU, sizes are exact"""
    from aios_amd.runtime.native import cu_mask_words

    a = cu_mask_words(64, 0, 256)
    b = cu_mask_words(192, 8, 256)
    bits = lambda w: {32 * i + j for i, x in enumerate(w) for j in range(32) if x >> j & 1}  # noqa: E731
    A, Bs = bits(a), bits(b)
    assert len(A) == 64 and len(Bs) == 192 and not (A & Bs) and len(A | Bs) == 256
    for xcd in range(8):
        assert any(i // 32 == xcd for i in A) and any(i % 8 == xcd for i in A)
        assert any(i // 32 == xcd for i in Bs) and any(i % 8 == xcd for i in Bs)
    import pytest

    with pytest.raises(ValueError):
        cu_mask_words(60, 0, 256)
    with pytest.raises(ValueError):
        cu_mask_words(192, 16, 256)

"""One typed node configuration for every service (SURVEY.md §5 "config / flag system": in the
reference only aios-init parses /etc/aios/config.toml, `initd/src/config.rs:445-469`, and two
schemas drift -- App. A #27: the runtime never reads the models section).

`load()` reads `$AIOS_CONFIG` (default /etc/aios/config.toml; defaults when missing), then applies
environment overrides `AIOS_CFG__<SECTION>__<KEY>=value` (double underscores, case-insensitive,
values parsed as TOML scalars).  Consumers: the runtime (model pool: tiers -> GGUF, context, TP
degree, batch/slots), the gateway (budgets, cache), the orchestrator (proactive thresholds,
heartbeat timeout), memory (database paths, context budget) and aios-init (its own C++ parser of
the same file).
"""
from __future__ import annotations

import dataclasses
import os
from typing import Any, Dict, List, Optional

try:  # Python 3.11+
    import tomllib as _toml
except ModuleNotFoundError:  # pragma: no cover - 3.10 image: the tomli wheel
    import tomli as _toml

DEFAULT_PATH = "/etc/aios/config.toml"


@dataclasses.dataclass
class SystemConfig:
    hostname: str = "aios"
    log_level: str = "info"
    log_dir: str = "/var/log/aios"
    data_dir: str = "/var/lib/aios"
    autonomy_level: str = "full"


@dataclasses.dataclass
class ModelTier:
    file: str = ""
    context_length: int = 0
    always_loaded: bool = False
    load_on_demand: bool = False
    max_tokens: int = 1024
    temperature: float = 0.3
    tensor_parallel: int = 1
    unload_after_idle_minutes: int = 0
    device: str = ""            # "" = GPU when present, "cpu" = the CPU engine
    replicas: int = 1           # engines of this tier, one per GPU (request-level data parallelism)
    devices: List[int] = dataclasses.field(default_factory=list)  # GPUs of the replicas ([] = first `replicas` of models.devices)
    kv_dtype: str = "bf16"      # KV cache: "bf16" or "fp8_e4m3" (half the cache bytes; long contexts)


@dataclasses.dataclass
class ModelsConfig:
    model_dir: str = "/var/lib/aios/models"
    # GPUs the runtime may use; [] = every GPU the node has (TP tiers then take the first
    # tensor_parallel of them).  Exported to the TP launcher only when it lists enough devices.
    devices: List[int] = dataclasses.field(default_factory=list)
    max_batch: int = 16
    max_slots: int = 16
    tiers: Dict[str, ModelTier] = dataclasses.field(default_factory=dict)


@dataclasses.dataclass
class ApiConfig:
    enabled: bool = True
    claude_monthly_budget_usd: float = 100.0
    openai_monthly_budget_usd: float = 50.0
    cache_max_entries: int = 1000
    cache_ttl_seconds: int = 3600


@dataclasses.dataclass
class MemoryConfig:
    operational_max_entries: int = 10000
    working_db: str = ""
    longterm_db: str = ""
    knowledge_db: str = ""
    context_max_tokens: int = 4000


@dataclasses.dataclass
class SecurityConfig:
    capability_mode: str = "enforce"
    audit_all_tool_calls: bool = True
    audit_db: str = ""
    sandbox_untrusted_tasks: bool = True
    secrets_file: str = "/etc/aios/secrets.toml"
    firewall_rules: str = "/etc/aios/security/firewall-rules.toml"


@dataclasses.dataclass
class AgentsConfig:
    config_dir: str = "/etc/aios/agents"
    heartbeat_timeout_seconds: int = 15
    max_restart_attempts: int = 5


@dataclasses.dataclass
class MonitoringConfig:
    cpu_threshold: float = 90.0
    memory_threshold: float = 85.0
    disk_threshold: float = 90.0


@dataclasses.dataclass
class NodeConfig:
    system: SystemConfig = dataclasses.field(default_factory=SystemConfig)
    models: ModelsConfig = dataclasses.field(default_factory=ModelsConfig)
    api: ApiConfig = dataclasses.field(default_factory=ApiConfig)
    memory: MemoryConfig = dataclasses.field(default_factory=MemoryConfig)
    security: SecurityConfig = dataclasses.field(default_factory=SecurityConfig)
    agents: AgentsConfig = dataclasses.field(default_factory=AgentsConfig)
    monitoring: MonitoringConfig = dataclasses.field(default_factory=MonitoringConfig)
    source: str = ""            # the file read ("" = defaults only)
    warnings: List[str] = dataclasses.field(default_factory=list)

    def tier_plan(self) -> List[dict]:
        """Every configured tier with a usable file: name, runtime path spec ('#tp=N' / '#cpu'),
        context length, whether to load it at start or on first request, replica devices and the
        idle-unload limit in seconds (reference `initd/src/config.rs:108-109`)."""
        out = []
        for name, t in self.models.tiers.items():
            if not t.file:
                continue
            path = t.file if (t.file.startswith("synthetic:") or os.path.isabs(t.file)) else os.path.join(
                self.models.model_dir, t.file)
            if not path.startswith("synthetic:") and not os.path.exists(path):
                continue
            frag = []
            if t.tensor_parallel > 1:
                frag.append(f"tp={t.tensor_parallel}")
            if t.device == "cpu":
                frag.append("cpu")
            if t.kv_dtype and t.kv_dtype != "bf16":
                frag.append(f"kv={t.kv_dtype}")
            devs = list(t.devices)
            if not devs and t.replicas > 1:
                devs = list(self.models.devices[:t.replicas]) or list(range(t.replicas))
            out.append(dict(name=name, spec=path + ("#" + "&".join(frag) if frag else ""),
                            ctx=t.context_length, on_demand=bool(t.load_on_demand and not t.always_loaded),
                            devices=devs if t.tensor_parallel <= 1 else [],
                            idle_unload_s=60.0 * max(0, t.unload_after_idle_minutes)))
        return out

    def tp_devices_env(self) -> str:
        """AIOS_TP_DEVICES for the runtime, or "" to let it detect every GPU: only an explicit
        models.devices list long enough for the widest TP tier is exported (a short default list
        would pin every rank of an 8-way tier to one GPU)."""
        need = max([t.tensor_parallel for t in self.models.tiers.values()] + [1])
        if self.models.devices and len(self.models.devices) >= need:
            return ",".join(str(d) for d in self.models.devices)
        return ""

    def model_specs(self) -> List[tuple]:
        """(name, runtime path spec, context_length) of the tiers to load at start: always_loaded
        tiers whose GGUF exists (absolute or under model_dir), with '#tp=N' / '#cpu' suffixes."""
        out = []
        for name, t in self.models.tiers.items():
            if not t.file or (t.load_on_demand and not t.always_loaded):
                continue
            path = t.file if (t.file.startswith("synthetic:") or os.path.isabs(t.file)) else os.path.join(
                self.models.model_dir, t.file)
            if not path.startswith("synthetic:") and not os.path.exists(path):
                continue
            frag = []
            if t.tensor_parallel > 1:
                frag.append(f"tp={t.tensor_parallel}")
            if t.device == "cpu":
                frag.append("cpu")
            if t.kv_dtype and t.kv_dtype != "bf16":
                frag.append(f"kv={t.kv_dtype}")
            out.append((name, path + ("#" + "&".join(frag) if frag else ""), t.context_length))
        return out


def _coerce(cls, raw: Dict[str, Any], warnings: List[str], where: str):
    fields = {f.name: f for f in dataclasses.fields(cls)}
    kw = {}
    for k, v in raw.items():
        f = fields.get(k)
        if f is None or k == "tiers":
            continue
        if k == "devices":
            if isinstance(v, list):
                try:
                    kw[k] = [int(x) for x in v]
                except (TypeError, ValueError):
                    warnings.append(f"{where}.{k}: cannot use {v!r}; default kept")
            continue
        want = f.type if isinstance(f.type, type) else None
        try:
            if f.type in ("int", int):
                v = int(v)
            elif f.type in ("float", float):
                v = float(v)
            elif f.type in ("bool", bool):
                v = v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes", "on")
            elif f.type in ("str", str):
                v = str(v)
        except (TypeError, ValueError):
            warnings.append(f"{where}.{k}: cannot use {v!r}; default kept")
            continue
        del want
        kw[k] = v
    return cls(**kw)


def _parse_scalar(v: str):
    try:
        return _toml.loads(f"x = {v}")["x"]
    except Exception:
        return v


def _apply_env(raw: Dict[str, Any], env) -> None:
    for k, v in env.items():
        if not k.upper().startswith("AIOS_CFG__"):
            continue
        path = [p.lower() for p in k[len("AIOS_CFG__"):].split("__") if p]
        if not path:
            continue
        node = raw
        for p in path[:-1]:
            node = node.setdefault(p, {})
            if not isinstance(node, dict):
                break
        else:
            node[path[-1]] = _parse_scalar(v)


def load(path: Optional[str] = None, env=None) -> NodeConfig:
    env = os.environ if env is None else env
    path = path or env.get("AIOS_CONFIG", DEFAULT_PATH)
    raw: Dict[str, Any] = {}
    cfg_warn: List[str] = []
    source = ""
    if path and os.path.exists(path):
        try:
            with open(path, "rb") as f:
                raw = _toml.load(f)
            source = path
        except Exception as e:  # noqa: BLE001 - defaults, like aios-init
            cfg_warn.append(f"{path}: {e}; using defaults")
    _apply_env(raw, env)
    models_raw = dict(raw.get("models", {}))
    tiers = {}
    for name, t in models_raw.items():
        if isinstance(t, dict):
            tiers[name] = _coerce(ModelTier, t, cfg_warn, f"models.{name}")
    models = _coerce(ModelsConfig, {k: v for k, v in models_raw.items() if not isinstance(v, dict)}, cfg_warn, "models")
    if isinstance(models_raw.get("devices"), list):
        models.devices = [int(x) for x in models_raw["devices"]]
    models.tiers = tiers
    api_raw = raw.get("api", raw.get("api_gateway", {}))  # both historical schemas (App. A)
    return NodeConfig(
        system=_coerce(SystemConfig, raw.get("system", {}), cfg_warn, "system"),
        models=models,
        api=_coerce(ApiConfig, api_raw, cfg_warn, "api"),
        memory=_coerce(MemoryConfig, raw.get("memory", {}), cfg_warn, "memory"),
        security=_coerce(SecurityConfig, raw.get("security", {}), cfg_warn, "security"),
        agents=_coerce(AgentsConfig, raw.get("agents", {}), cfg_warn, "agents"),
        monitoring=_coerce(MonitoringConfig, raw.get("monitoring", {}), cfg_warn, "monitoring"),
        source=source, warnings=cfg_warn)

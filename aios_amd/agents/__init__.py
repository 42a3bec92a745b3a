"""aiOS Python agents (reference `agent-core/python/aios_agent`).

`AGENT_REGISTRY` maps the agent type used in /etc/aios/agents/*.toml to its class; each module
is runnable as `python -m aios_amd.agents.<type>` (what the orchestrator's spawner launches).
Classes are imported lazily so spawning one agent does not import the other nine.
"""
from __future__ import annotations

import importlib

_TYPES = {
    "system": "SystemAgent", "task": "TaskAgent", "network": "NetworkAgent", "security": "SecurityAgent",
    "package": "PackageAgent", "storage": "StorageAgent", "monitoring": "MonitoringAgent",
    "learning": "LearningAgent", "creator": "CreatorAgent", "web": "WebAgent",
}


def agent_class(agent_type: str):
    mod = importlib.import_module(f"{__name__}.{agent_type}")
    return getattr(mod, _TYPES[agent_type])


class _Registry(dict):
    def __missing__(self, key):
        if key not in _TYPES:
            raise KeyError(key)
        cls = agent_class(key)
        self[key] = cls
        return cls

    def __iter__(self):
        return iter(_TYPES)

    def keys(self):
        return _TYPES.keys()

    def __len__(self):
        return len(_TYPES)


AGENT_REGISTRY = _Registry()


def __getattr__(name):
    for t, cls in _TYPES.items():
        if cls == name:
            return agent_class(t)
    if name in ("BaseAgent", "AgentConfig", "IntelligenceLevel"):
        return getattr(importlib.import_module(f"{__name__}.base"), name)
    if name == "OrchestratorClient":
        return importlib.import_module(f"{__name__}.orchestrator_client").OrchestratorClient
    raise AttributeError(name)

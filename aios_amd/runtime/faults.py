"""Fault injection for the runtime (SURVEY.md §5 "failure detection / fault injection": the
reference has none).  `AIOS_FAULT_INJECT` (or an explicit spec) wraps a model's engine so that
chosen calls fail or stall, which exercises the recovery paths end to end: the scheduler fails
the affected requests, the model manager marks the model `error` (reference semantics,
`runtime/src/model_manager.rs:393-447`) and -- beyond the reference -- reloads it.

Spec: comma-separated `site:mode` items, site in {load, prefill, decode}:
    decode:after=5      the 6th decode call and every later one raise
    decode:once=3       only the 4th decode call raises
    prefill:always      every prefill raises
    decode:stall=2.5    every decode call sleeps 2.5 s first (trips the stall watchdog)
    load:always         engine construction fails
`AIOS_FAULT_MODELS` (comma list) restricts injection to those model names.
"""
from __future__ import annotations

import os
import threading
import time
from typing import Dict, Optional


class InjectedFault(RuntimeError):
    pass


class FaultSpec:
    def __init__(self, spec: str = ""):
        self.rules: Dict[str, tuple] = {}
        for item in (spec or "").split(","):
            item = item.strip()
            if not item:
                continue
            site, _, mode = item.partition(":")
            kind, _, arg = mode.partition("=")
            if site not in ("load", "prefill", "decode") or kind not in ("after", "once", "always", "stall"):
                raise ValueError(f"bad fault spec item {item!r}")
            self.rules[site] = (kind, float(arg) if arg else 0.0)
        self.calls: Dict[str, int] = {}
        self.lock = threading.Lock()

    @classmethod
    def from_env(cls, model: str = "") -> Optional["FaultSpec"]:
        spec = os.environ.get("AIOS_FAULT_INJECT", "")
        only = [m for m in os.environ.get("AIOS_FAULT_MODELS", "").split(",") if m]
        if not spec or (only and model not in only):
            return None
        return cls(spec)

    def check(self, site: str):
        rule = self.rules.get(site)
        if rule is None:
            return
        with self.lock:
            n = self.calls.get(site, 0)
            self.calls[site] = n + 1
        kind, arg = rule
        if kind == "stall":
            time.sleep(arg)
        elif kind == "always" or (kind == "after" and n >= arg) or (kind == "once" and n == int(arg)):
            raise InjectedFault(f"injected {site} fault (call {n})")


class FaultyEngine:
    """Transparent proxy that consults a FaultSpec before prefill / decode."""

    def __init__(self, engine, spec: FaultSpec):
        self._engine = engine
        self._spec = spec

    def prefill(self, *a, **k):
        self._spec.check("prefill")
        return self._engine.prefill(*a, **k)

    def decode(self, *a, **k):
        self._spec.check("decode")
        return self._engine.decode(*a, **k)

    def __getattr__(self, name):
        attr = getattr(self._engine, name)
        if name == "decode_submit":  # the pipelined decode's step (present iff the engine has it)
            def submit(*a, **k):
                self._spec.check("decode")
                return attr(*a, **k)
            return submit
        return attr

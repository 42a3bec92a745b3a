"""Model pool: co-resident models in HBM, lifecycle, intelligence-level routing, health.

Mirrors `ModelManager` of the reference (`runtime/src/model_manager.rs`) without the child
processes: each model is an in-process native Engine + tokenizer + chat template + JSON grammar
+ continuous-batching Scheduler.  Differences on purpose:
  * loads run in a worker thread, so a 30-120 s load never blocks routing/inference (#14);
  * the `strategic` level first tries a local strategic model (the TP tier, e.g. llama3-70b)
    before reproducing the reference's FailedPrecondition "route via api-gateway" (§7.1);
  * `ModelStatus.port` is a real per-model OpenAI-compatible HTTP endpoint (service.py).

Model paths: a GGUF file, or `synthetic:<preset>[:<recipe>]` for a random-init model of a named
architecture (tests/benchmarks without network access).
"""
from __future__ import annotations

import asyncio
import dataclasses
import logging
import os
import threading
import time
from typing import Dict, List, Optional

log = logging.getLogger("aios.runtime.models")

BASE_PORT = 8080  # runtime/src/model_manager.rs:70

LEVEL_CANDIDATES = {
    # runtime/src/model_manager.rs:462-502 (+ the local strategic TP tier first)
    "operational": ["tinyllama-1.1b", "DeepSeek-R1-Distill-Qwen-8B", "mistral-7b"],
    "tactical": ["DeepSeek-R1-Distill-Qwen-8B", "Qwen3-14B", "mistral-7b", "tinyllama-1.1b"],
    "strategic": ["llama3-70b", "Qwen3-14B", "DeepSeek-R1-Distill-Qwen-8B", "mistral-7b"],
}


class RoutingError(Exception):
    """Carries the gRPC status name the service maps it to."""

    def __init__(self, code: str, msg: str):
        super().__init__(msg)
        self.code = code


@dataclasses.dataclass
class ManagedModel:
    name: str
    path: str
    status: str = "loading"
    port: int = 0
    context_length: int = 2048
    loaded_at: int = 0
    last_used: int = 0
    request_count: int = 0
    error: str = ""
    engine: object = None
    tokenizer: object = None
    template: object = None
    grammar: object = None
    scheduler: object = None
    config: object = None
    weight_bytes: int = 0
    kv_bytes: int = 0

    def status_string(self) -> str:
        return f"error: {self.error}" if self.status == "error" else self.status


def context_for_size(nbytes: int) -> int:
    """Reference auto-load heuristic (`runtime/src/main.rs:86-98`)."""
    gb = nbytes / 1e9
    if gb > 8:
        return 8192
    if gb > 2:
        return 4096
    return 2048


class ModelManager:
    def __init__(self, device: int = 0, max_batch: int = 8, max_slots: int = 16, base_port: int = BASE_PORT):
        self.device = device
        self.max_batch = max_batch
        self.max_slots = max_slots
        self.base_port = base_port
        self.models: Dict[str, ManagedModel] = {}
        self._lock = threading.Lock()
        self.started = time.time()

    def tp_devices(self) -> List[int]:
        env = os.environ.get("AIOS_TP_DEVICES", "")
        if env:
            return [int(x) for x in env.split(",") if x.strip()]
        try:
            import torch

            n = torch.cuda.device_count()
        except Exception:
            n = 0
        return list(range(n)) if n > 1 else [self.device]

    # ------------------------------------------------------------------ lifecycle
    def allocate_port(self, requested: int = 0) -> int:
        used = {m.port for m in self.models.values()}
        if requested and requested not in used:
            return requested
        p = self.base_port
        while p in used:
            p += 1
        return p

    async def load_model(self, name: str, path: str, context_length: int = 0, port: int = 0) -> ManagedModel:
        with self._lock:
            m = self.models.get(name)
            if m is not None and m.status in ("ready", "loading"):
                return m  # idempotent (model_manager.rs:152-157)
            m = ManagedModel(name=name, path=path, status="loading", port=self.allocate_port(port))
            self.models[name] = m
        try:
            await asyncio.to_thread(self._load_blocking, m, context_length)
            m.status = "ready"
            m.loaded_at = int(time.time())
        except Exception as e:  # noqa: BLE001
            log.exception("load of %s failed", name)
            m.status, m.error = "error", str(e)
        return m

    def _load_blocking(self, m: ManagedModel, context_length: int):
        from ..gguf.reader import GGUFReader
        from ..models.config import get_preset
        from ..models.synthetic import synthetic_vocab
        from . import chat_template, native
        from .loader import load_engine, random_engine
        from .tokenizer import SpmTokenizer, from_gguf

        E = native.require()
        from ..parallel.tp import launch_tp, parse_spec

        base, tp, act_q8 = parse_spec(m.path)
        if tp > 1:
            # strategic tier: tensor parallel over the node's GPUs (ranks 1..tp-1 are worker
            # processes; the xGMI all-reduce runs inside each rank's captured decode graph)
            ctx = context_length or 4096
            eng, cfg = launch_tp(base, tp, self.tp_devices(), ctx, self.max_slots, self.max_batch,
                                 seed=abs(hash(m.name)) % 1000, act_q8=act_q8)
            if base.startswith("synthetic:"):
                toks, scores, types = synthetic_vocab(cfg.vocab_size)
                tok = SpmTokenizer(toks, scores, types, cfg.bos_id, cfg.eos_id)
                tmpl = chat_template.for_model(cfg.chat_template if cfg.chat_template in chat_template.BUILTIN
                                               else "zephyr", tok)
            else:
                reader = GGUFReader(base)
                tok = from_gguf(reader)
                tmpl = chat_template.for_model(reader, tok)
        elif base.startswith("synthetic:"):
            parts = base.split(":")
            cfg = get_preset(parts[1])
            recipe = parts[2] if len(parts) > 2 else "Q4_K_M"
            ctx = context_length or min(cfg.max_ctx, 4096)
            eng = random_engine(cfg, recipe, seed=abs(hash(m.name)) % 1000, max_ctx=ctx, max_slots=self.max_slots,
                                max_batch=self.max_batch, device=self.device, act_q8=act_q8)
            toks, scores, types = synthetic_vocab(cfg.vocab_size)
            tok = SpmTokenizer(toks, scores, types, cfg.bos_id, cfg.eos_id)
            tmpl = chat_template.for_model(cfg.chat_template if cfg.chat_template in chat_template.BUILTIN else "zephyr",
                                           tok)
        else:
            if not os.path.exists(base):
                raise FileNotFoundError(base)
            ctx = context_length or context_for_size(os.path.getsize(base))
            eng, cfg, reader = load_engine(base, max_ctx=ctx, max_slots=self.max_slots, max_batch=self.max_batch,
                                           device=self.device, name=m.name, act_q8=act_q8)
            tok = from_gguf(reader)
            tmpl = chat_template.for_model(reader, tok)
        m.engine, m.config, m.tokenizer, m.template = eng, cfg, tok, tmpl
        m.context_length = eng.config.max_ctx
        m.grammar = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
        from .scheduler import Scheduler

        m.scheduler = Scheduler(eng, tok, self.max_batch, self.max_slots, m.context_length, m.grammar, name=m.name)
        m.weight_bytes, m.kv_bytes = eng.weight_bytes, eng.kv_bytes

    async def unload_model(self, name: str) -> bool:
        m = self.models.get(name)
        if m is None:
            return False
        m.status = "unloading"
        if m.scheduler is not None:
            await asyncio.to_thread(m.scheduler.close)
        if hasattr(m.engine, "close"):
            await asyncio.to_thread(m.engine.close)
        m.engine = None
        m.scheduler = None
        self.models.pop(name, None)
        return True

    def list_models(self) -> List[ManagedModel]:
        return list(self.models.values())

    # ------------------------------------------------------------------ routing
    def _first_ready_from(self, candidates) -> Optional[str]:
        for c in candidates:
            cl = c.lower()
            for name, m in self.models.items():
                if m.status == "ready" and cl in name.lower():
                    return name
        return None

    def first_ready(self) -> Optional[str]:
        for name, m in self.models.items():
            if m.status == "ready":
                return name
        return None

    def select_model_for_level(self, level: str) -> Optional[str]:
        if level == "reactive":
            return None
        if level in LEVEL_CANDIDATES:
            return self._first_ready_from(LEVEL_CANDIDATES[level])
        return self.first_ready()

    def resolve(self, model: str, level: str) -> ManagedModel:
        """grpc_service.rs:187-233: explicit name -> level routing -> any ready model."""
        if model:
            m = self.models.get(model)
            if m is not None and m.status == "ready":
                return self._touch(m)
        if level:
            name = self.select_model_for_level(level)
            if name is not None:
                return self._touch(self.models[name])
            if level == "reactive":
                raise RoutingError("INVALID_ARGUMENT",
                                   "Reactive level does not require LLM inference — handle with heuristics")
            if level == "strategic":
                raise RoutingError("FAILED_PRECONDITION", "Strategic level requires external API — route via api-gateway")
        name = self.first_ready()
        if name is not None:
            return self._touch(self.models[name])
        raise RoutingError("UNAVAILABLE", "No model available for inference.  Load a model first with LoadModel.")

    @staticmethod
    def _touch(m: ManagedModel) -> ManagedModel:
        m.request_count += 1
        m.last_used = int(time.time())
        return m

    # ------------------------------------------------------------------ health
    def health(self) -> Dict[str, str]:
        details = {}
        for name, m in self.models.items():
            extra = ""
            if m.scheduler is not None:
                st = m.scheduler.stats
                avg_b = st["batch_sum"] / st["steps"] if st["steps"] else 0.0
                extra = (f",queue={len(m.scheduler.queue)},active={len(m.scheduler.active)},tokens={st['tokens']}"
                         f",avg_batch={avg_b:.2f},prefix_hit_tokens={st['cached_tokens']}")
            details[f"model:{name}"] = (f"{m.status_string()},port={m.port},hbm_gb={(m.weight_bytes + m.kv_bytes) / 1e9:.2f}"
                                        + extra)
        return details

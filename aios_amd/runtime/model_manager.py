"""Model pool: co-resident models in HBM, lifecycle, intelligence-level routing, health.

Mirrors `ModelManager` of the reference (`runtime/src/model_manager.rs`) without the child
processes: each model is an in-process native Engine + tokenizer + chat template + JSON grammar
+ continuous-batching Scheduler.  Differences on purpose:
  * loads run in a worker thread, so a 30-120 s load never blocks routing/inference (#14);
  * the `strategic` level first tries a local strategic model (the TP tier, e.g. llama3-70b)
    before reproducing the reference's FailedPrecondition "route via api-gateway" (§7.1);
  * `ModelStatus.port` is a real per-model OpenAI-compatible HTTP endpoint (service.py);
  * tier lifecycle (the reference's `load_on_demand` / `unload_after_idle_minutes`,
    `initd/src/config.rs:108-109`, which its runtime never acted on): a registered on-demand
    tier is loaded by the first request its level routes to (`resolve_async`), any model with an
    idle limit is unloaded by the health pass once idle and re-registered for on-demand load;
  * replicas: one tier may run as several engines on different GPUs of the node (request-level
    data parallelism, SURVEY §2.9 DP row); routing picks the least-loaded ready replica.

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
import zlib
from typing import Dict, List, Optional

from .faults import FaultSpec, FaultyEngine


def _synth_seed(name: str) -> int:
    """Weight seed of a synthetic (random-init) model: stable across processes (str hash() is
    salted per process, which made every bench run draw different weights -- and, with JSON-mode
    plans that random weights close at arbitrary points, different plan lengths)."""
    return zlib.crc32(name.encode()) % 1000

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
    backend: str = "gpu"
    requested_ctx: int = 0
    restarts: list = dataclasses.field(default_factory=list)  # reload timestamps (restart window)
    device: int = -1                  # GPU of this engine (-1: the manager's default device)
    group: str = ""                   # replica group (tier name); "" = the model's own name
    idle_unload_s: float = 0.0        # unload after this long without a request (0 = never)

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


def estimated_q4_bytes(cfg) -> int:
    """GGUF size of a preset at ~4.5 bits per weight (Q4_K_M), for the context heuristic of
    synthetic tiers (no file to stat)"""
    d, hd = cfg.d_model, cfg.head_dim
    qd, kvd = cfg.n_heads * hd, cfg.n_kv_heads * hd
    per_layer = d * (qd + 2 * kvd) + qd * d + 3 * d * cfg.d_ff
    return int((cfg.n_layers * per_layer + 2 * cfg.vocab_size * d) * 4.5 / 8)


def tier_context(cfg, path: str = "") -> int:
    """Context for a tier without an explicit one: the reference's size heuristic (> 8 GB files:
    8192, `runtime/src/main.rs:86-98`) on the GGUF file, or on the preset's estimated size for
    synthetic tiers, capped by the model's window"""
    nbytes = os.path.getsize(path) if path and os.path.exists(path) else estimated_q4_bytes(cfg)
    return min(cfg.max_ctx, context_for_size(nbytes))


class ModelManager:
    def __init__(self, device: int = 0, max_batch: int = 16, max_slots: int = 16, base_port: int = BASE_PORT):
        self.device = device
        self.max_batch = max_batch
        self.max_slots = max_slots
        self.base_port = base_port
        self.models: Dict[str, ManagedModel] = {}
        # on-demand tiers not resident yet: name -> (path, ctx, devices, idle_unload_s)
        self.deferred: Dict[str, tuple] = {}
        self._ondemand_locks: Dict[str, asyncio.Lock] = {}
        self.unload_hooks: list = []  # async callables(name) run after a model is unloaded
        self.abandoned: list = []  # schedulers of stalled engines (their threads may still be stuck)
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

    async def load_model(self, name: str, path: str, context_length: int = 0, port: int = 0, device: int = -1,
                         group: str = "", idle_unload_s: float = 0.0) -> ManagedModel:
        with self._lock:
            m = self.models.get(name)
            if m is not None and m.status in ("ready", "loading"):
                return m  # idempotent (model_manager.rs:152-157)
            restarts = m.restarts if m is not None else []
            keep_port = m.port if m is not None and not port else port
            if m is not None:  # reload of an errored / unloading model: its port is free again
                device = m.device if device < 0 else device
                group = group or m.group
                idle_unload_s = idle_unload_s or m.idle_unload_s
                self.models.pop(name, None)
            m = ManagedModel(name=name, path=path, status="loading", port=self.allocate_port(keep_port),
                             requested_ctx=context_length, restarts=restarts, device=device, group=group,
                             idle_unload_s=idle_unload_s)
            self.models[name] = m
            self.deferred.pop(name, None)
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
        from ..parallel.tp import launch_tp, parse_spec, spec_kv_dtype

        device = self.device if m.device < 0 else m.device

        base, tp, act_q8 = parse_spec(m.path)
        kv_dtype = spec_kv_dtype(m.path)
        faults = FaultSpec.from_env(m.name)
        if faults is not None:
            faults.check("load")
        base, cpu = self._backend(base, "cpu" in m.path.partition("#")[2].split("&"))
        if cpu:
            self._load_cpu(m, base, context_length)
        elif tp > 1:
            # strategic tier: tensor parallel over the node's GPUs (ranks 1..tp-1 are worker
            # processes; the xGMI all-reduce runs inside each rank's captured decode graph)
            if not context_length:
                if base.startswith("synthetic:"):
                    context_length = tier_context(get_preset(base.split(":")[1]))
                else:
                    context_length = context_for_size(os.path.getsize(base)) if os.path.exists(base) else 8192
            ctx = context_length
            eng, cfg = launch_tp(base, tp, self.tp_devices(), ctx, self.max_slots, self.max_batch,
                                 seed=_synth_seed(m.name), act_q8=act_q8, kv_dtype=kv_dtype)
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
            ctx = context_length or tier_context(cfg)
            eng = random_engine(cfg, recipe, seed=_synth_seed(m.group or m.name), max_ctx=ctx,
                                max_slots=self.max_slots, max_batch=self.max_batch, device=device, act_q8=act_q8,
                                kv_dtype=kv_dtype)
            toks, scores, types = synthetic_vocab(cfg.vocab_size)
            tok = SpmTokenizer(toks, scores, types, cfg.bos_id, cfg.eos_id)
            tmpl = chat_template.for_model(cfg.chat_template if cfg.chat_template in chat_template.BUILTIN else "zephyr",
                                           tok)
        else:
            if not os.path.exists(base):
                raise FileNotFoundError(base)
            ctx = context_length or context_for_size(os.path.getsize(base))
            eng, cfg, reader = load_engine(base, max_ctx=ctx, max_slots=self.max_slots, max_batch=self.max_batch,
                                           device=device, name=m.name, act_q8=act_q8, kv_dtype=kv_dtype)
            tok = from_gguf(reader)
            tmpl = chat_template.for_model(reader, tok)
        if not cpu:
            m.engine, m.config, m.tokenizer, m.template = eng, cfg, tok, tmpl
        if faults is not None:
            m.engine = FaultyEngine(m.engine, faults)
        eng, tok = m.engine, m.tokenizer
        m.context_length = eng.config.max_ctx
        m.grammar = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
        from .scheduler import Scheduler

        slots = getattr(eng.config, "max_slots", self.max_slots)
        batch = getattr(eng.config, "max_batch", self.max_batch)
        m.scheduler = Scheduler(eng, tok, min(batch, self.max_batch), min(slots, self.max_slots), m.context_length,
                                m.grammar, name=m.name)
        # capture every batch size's decode-step graph now, not on the first step that reaches it
        # (a capture stalls that step by milliseconds; AIOS_GRAPH_WARMUP=0 skips)
        capture = getattr(eng, "capture_graphs", None)
        if capture is not None and os.environ.get("AIOS_GRAPH_WARMUP", "1") != "0":
            capture(m.scheduler.max_batch)
        m.weight_bytes, m.kv_bytes = eng.weight_bytes, eng.kv_bytes

    # ------------------------------------------------------------------ tier lifecycle
    def register_on_demand(self, name: str, path: str, context_length: int = 0, devices: Optional[List[int]] = None,
                           idle_unload_s: float = 0.0):
        """A tier that is not loaded at start: the first request its level (or name) routes to
        loads it (resolve_async).  `devices` > 1 entry -> one replica per device."""
        if name not in self.models:
            self.deferred[name] = (path, context_length, list(devices or []), idle_unload_s)

    async def load_replicas(self, name: str, path: str, context_length: int = 0,
                            devices: Optional[List[int]] = None, idle_unload_s: float = 0.0) -> List[ManagedModel]:
        """Load one engine per device (`name` on the first, `name@<dev>` on the others); routing
        spreads requests over the group by load.  Replicas load concurrently (one thread each)."""
        devs = list(devices or []) or [self.device]
        names = [name if i == 0 else f"{name}@{d}" for i, d in enumerate(devs)]
        res = await asyncio.gather(*[self.load_model(n, path, context_length, device=d,
                                                     group=name if len(devs) > 1 else "",
                                                     idle_unload_s=idle_unload_s)
                                     for n, d in zip(names, devs)])
        return list(res)

    def _deferred_for(self, model: str, level: str) -> Optional[str]:
        if not self.deferred:
            return None
        if model and model in self.deferred:
            return model
        for c in LEVEL_CANDIDATES.get(level, []):
            cl = c.lower()
            for name, (path, _, _, _) in self.deferred.items():
                if cl in name.lower() or cl in os.path.basename(path.partition("#")[0]).lower():
                    return name
        return None

    async def resolve_async(self, model: str, level: str) -> ManagedModel:
        """resolve() plus on-demand loading: when nothing resident serves the request but a
        registered on-demand tier does, load it (once, concurrent requests wait on the same load)
        and route to it.  Falls back to resolve()'s reference error codes when the load fails."""
        try:
            return self.resolve(model, level)
        except RoutingError as err:
            name = self._deferred_for(model, level)
            if name is None:
                raise
            lock = self._ondemand_locks.setdefault(name, asyncio.Lock())
            async with lock:
                if name in self.deferred:
                    path, ctx, devs, idle = self.deferred[name]
                    log.info("on-demand load of tier %s (%s) for level=%r model=%r", name, path, level, model)
                    ms = await self.load_replicas(name, path, ctx, devs, idle)
                    if not any(m.status == "ready" for m in ms):
                        self.deferred[name] = (path, ctx, devs, idle)  # keep it registered for a retry
                        raise RoutingError("UNAVAILABLE", f"on-demand load of {name} failed: {ms[0].error}") from err
            return self.resolve(model or name, level)

    def _busy(self, m: ManagedModel) -> bool:
        if m.scheduler is None:
            return False
        mt = m.scheduler.metrics()
        return mt.get("queued", 0) > 0 or mt.get("active", 0) > 0

    async def unload_idle(self, now: Optional[float] = None) -> List[str]:
        """Unload every ready model whose idle limit has passed (no request for idle_unload_s and
        nothing queued or decoding); each goes back to the on-demand registry so the next request
        reloads it.  A replica group unloads together."""
        now = time.time() if now is None else now
        out = []
        for m in list(self.models.values()):
            if m.status != "ready" or m.idle_unload_s <= 0:
                continue
            last = max(m.last_used, m.loaded_at)
            if now - last < m.idle_unload_s or self._busy(m):
                continue
            group = m.group or m.name
            members = [x for x in self.models.values() if (x.group or x.name) == group]
            if any(self._busy(x) or now - max(x.last_used, x.loaded_at) < x.idle_unload_s for x in members):
                continue
            devs = sorted({x.device for x in members if x.device >= 0})
            log.info("unloading idle tier %s (%d engine(s), idle %.0f s)", group, len(members), now - last)
            for x in members:
                await self.unload_model(x.name)
                out.append(x.name)
            self.deferred[group] = (m.path, m.requested_ctx, devs, m.idle_unload_s)
        return out

    # ------------------------------------------------------------------ CPU backend
    @staticmethod
    def _backend(base: str, cpu_flag: bool = False):
        """'<path>#cpu' / AIOS_RUNTIME_DEVICE=cpu / no GPU -> the CPU engine (reference default:
        llama-server with gpu_layers 0)."""
        cpu = cpu_flag or os.environ.get("AIOS_RUNTIME_DEVICE", "") == "cpu"
        if not cpu:
            from . import native

            cpu = not native.gpu_available()
        return base, cpu

    def _load_cpu(self, m: ManagedModel, base: str, context_length: int):
        from ..gguf.reader import GGUFReader
        from ..models.config import get_preset
        from ..models.synthetic import synthetic_vocab, write_synthetic_gguf
        from . import chat_template
        from .cpu_engine import CpuEngine
        from .tokenizer import SpmTokenizer, from_gguf

        slots = min(self.max_slots, 4)
        if base.startswith("synthetic:"):
            parts = base.split(":")
            cfg = get_preset(parts[1])
            recipe = parts[2] if len(parts) > 2 else "Q4_0"
            import tempfile

            path = os.path.join(tempfile.gettempdir(), f"aios-cpu-{parts[1]}-{recipe}.gguf")
            if not os.path.exists(path):
                write_synthetic_gguf(path, cfg, recipe, seed=_synth_seed(m.name))
            ctx = context_length or min(cfg.max_ctx, 2048)
            eng = CpuEngine.from_gguf(path, max_ctx=ctx, max_slots=slots, max_batch=min(self.max_batch, slots))
            toks, scores, types = synthetic_vocab(cfg.vocab_size)
            tok = SpmTokenizer(toks, scores, types, cfg.bos_id, cfg.eos_id)
            tmpl = chat_template.for_model(cfg.chat_template if cfg.chat_template in chat_template.BUILTIN
                                           else "zephyr", tok)
        else:
            if not os.path.exists(base):
                raise FileNotFoundError(base)
            ctx = context_length or context_for_size(os.path.getsize(base))
            eng = CpuEngine.from_gguf(base, max_ctx=ctx, max_slots=slots, max_batch=min(self.max_batch, slots))
            reader = GGUFReader(base)
            tok = from_gguf(reader)
            tmpl = chat_template.for_model(reader, tok)
            cfg = eng.cfg
        m.engine, m.config, m.tokenizer, m.template = eng, cfg, tok, tmpl
        m.backend = "cpu"

    # ------------------------------------------------------------------ supervision
    async def supervise(self, stall_timeout_s: float = 0.0, auto_recover: Optional[bool] = None,
                        max_restarts: int = 3, window_s: float = 300.0) -> List[str]:
        """Health pass (the reference's 10 s loop, `model_manager.rs:393-447`): a dead scheduler
        thread, an engine error or a stalled decode (no progress for stall_timeout_s with work
        pending) marks the model `error`.  Unlike the reference, an errored model is reloaded
        (AIOS_RUNTIME_AUTORECOVER, default on) at most max_restarts times per window_s; a stalled
        engine's thread is abandoned (a hung device call cannot be interrupted) and its pending
        requests are failed.  Returns the names of models reloaded in this pass."""
        if auto_recover is None:
            auto_recover = os.environ.get("AIOS_RUNTIME_AUTORECOVER", "1") != "0"
        stall_timeout_s = stall_timeout_s or float(os.environ.get("AIOS_DECODE_STALL_S", "120"))
        recovered = []
        for m in list(self.models.values()):
            if m.status == "ready" and m.scheduler is not None:
                sch = m.scheduler
                reason = ""
                if not sch.thread.is_alive():
                    reason = "scheduler thread died"
                elif sch.failed:
                    reason = f"engine failure: {sch.failed}"
                elif sch.stalled(stall_timeout_s):
                    reason = f"decode stalled for more than {stall_timeout_s:.0f} s"
                if reason:
                    self.fail_model(m, reason)
            if m.status == "error" and auto_recover:
                now = time.time()
                m.restarts[:] = [t for t in m.restarts if now - t < window_s]
                if len(m.restarts) >= max_restarts:
                    continue
                m.restarts.append(now)
                log.warning("reloading model %s (restart %d in window)", m.name, len(m.restarts))
                nm = await self.load_model(m.name, m.path, m.requested_ctx, m.port)
                if nm.status == "ready":
                    recovered.append(m.name)
        await self.unload_idle()
        return recovered

    def fail_model(self, m: ManagedModel, reason: str):
        """Take a model out of routing now (status `error`): its scheduler is abandoned, pending
        requests fail, and a multi-process engine (TP ranks) is torn down so a dead or hung rank
        cannot keep the others spinning; level routing then falls through to the next tier."""
        if m.status != "ready":
            return
        log.error("model %s -> error: %s", m.name, reason)
        m.status, m.error = "error", reason
        self._abandon(m, stalled="stalled" in reason)

    def _abandon(self, m: ManagedModel, stalled: bool):
        sch = m.scheduler
        m.scheduler = None
        eng = m.engine
        if eng is not None and hasattr(eng, "abort"):
            try:
                eng.abort()  # TP: kill the worker ranks, close the command channel
            except Exception:  # noqa: BLE001
                log.exception("engine abort of %s failed", m.name)
        if sch is None:
            m.engine = None
            return
        self.abandoned.append(sch)
        from .scheduler import GenResult

        with sch.cv:
            sch.stop_flag = True
            pending = list(sch.queue)
            sch.queue.clear()
            active = list(sch.active) if stalled else []
            sch.cv.notify()
        for r in pending:
            sch._done(r, GenResult("", [], len(r.prompt_ids), 0, "error", error=m.error))
        for seq in active:  # the stuck thread never returns to finish them
            sch._done(seq.req, GenResult("", list(seq.out), len(seq.req.prompt_ids), len(seq.out), "error",
                                         error=m.error))
        m.engine = None

    def join_abandoned(self, timeout_s: float = 10.0) -> int:
        """Wait (bounded) for abandoned scheduler threads to exit; returns how many are still stuck."""
        deadline = time.time() + timeout_s
        for sch in self.abandoned:
            sch.thread.join(max(0.0, deadline - time.time()))
        self.abandoned = [s for s in self.abandoned if s.thread.is_alive()]
        return len(self.abandoned)

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
        for hook in self.unload_hooks:
            try:
                await hook(name)
            except Exception:  # noqa: BLE001
                log.exception("unload hook failed for %s", name)
        return True

    def list_models(self) -> List[ManagedModel]:
        return list(self.models.values())

    # ------------------------------------------------------------------ routing
    def _load_of(self, m: ManagedModel) -> float:
        if m.scheduler is None:
            return 0.0
        mt = m.scheduler.metrics()
        return float(mt.get("queued", 0) + mt.get("active", 0))

    def _pick_replica(self, name: str) -> str:
        """Least-loaded ready member of `name`'s replica group (ties: fewest requests served)."""
        m = self.models[name]
        if not m.group:
            return name
        members = [x for x in self.models.values() if x.group == m.group and x.status == "ready"]
        if not members:
            return name
        best = min(members, key=lambda x: (self._load_of(x), x.request_count))
        return best.name

    def _first_ready_from(self, candidates) -> Optional[str]:
        for c in candidates:
            cl = c.lower()
            for name, m in self.models.items():
                if m.status == "ready" and cl in name.lower():
                    return self._pick_replica(name)
        return None

    def first_ready(self) -> Optional[str]:
        for name, m in self.models.items():
            if m.status == "ready":
                return self._pick_replica(name)
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
                return self._touch(self.models[self._pick_replica(model)])
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
                mt = m.scheduler.metrics()
                extra = (f",backend={m.backend},queue={mt['queued']},active={mt['active']},tokens={st['tokens']}"
                         f",avg_batch={mt['avg_batch']:.2f},prefix_hit_tokens={mt['prefix_hit_tokens']}"
                         f",tok_s={mt['tokens_per_s']:.1f},ttft_p50_ms={mt['ttft_p50_ms']:.1f}"
                         f",itl_ms={mt['itl_ms']:.2f},kv_slot_util={mt['kv_slot_util']:.2f},errors={mt['errors']}")
            if m.restarts:
                extra += f",restarts={len(m.restarts)}"
            details[f"model:{name}"] = (f"{m.status_string()},port={m.port},hbm_gb={(m.weight_bytes + m.kv_bytes) / 1e9:.2f}"
                                        + extra)
        return details

    def metrics(self) -> Dict[str, float]:
        """Aggregate runtime metrics for MemoryService.UpdateMetric (operational memory keys)."""
        out = {"runtime.models_ready": float(sum(m.status == "ready" for m in self.models.values())),
               "runtime.tokens_per_s": 0.0, "runtime.active_requests": 0.0,
               "runtime.hbm_gb": sum((m.weight_bytes + m.kv_bytes) for m in self.models.values()) / 1e9}
        for m in self.models.values():
            if m.scheduler is not None:
                mt = m.scheduler.metrics()
                out["runtime.tokens_per_s"] += mt["tokens_per_s"]
                out["runtime.active_requests"] += mt["active"]
                out[f"runtime.{m.name}.ttft_p50_ms"] = mt["ttft_p50_ms"]
                out[f"runtime.{m.name}.itl_ms"] = mt["itl_ms"]
        try:
            from ..utils import sysinfo

            out["gpu.utilization"] = sysinfo.gpu_utilization()
            gh = sysinfo.gpu_health()
            out["gpu.ecc_ue_total"] = float(gh["ecc_ue_total"])
            out["gpu.ecc_ce_total"] = float(gh["ecc_ce_total"])
            out["gpu.healthy"] = 1.0 if gh["healthy"] else 0.0
        except Exception:  # pragma: no cover
            pass
        return out

"""API gateway core: provider clients, budget manager, request router with response cache.

Reference: `api-gateway/src/{claude,openai,budget,router}.rs`.
* providers: `claude` (Anthropic /v1/messages, $3/$15 per M tokens), `openai` ($2.5/$10 per M),
  `qwen3` (OpenAI-compatible at QWEN3_BASE_URL) and `local` -- OpenAI-compatible HTTP at
  LOCAL_LLM_URL (default :8082, the strategic model's endpoint on the MI355X runtime), falling
  back to the runtime's gRPC `AIRuntime.Infer` when no HTTP server answers;
* JSON mode is switched on when the prompt asks for "valid JSON" / "JSON object" (openai.rs:137);
* budget: monthly $100 Claude / $50 OpenAI, 80 % warning, monthly reset, usage records
  persisted to SQLite (the reference kept them in memory); real prompt/completion token split
  when the provider reports it instead of the reference's 50/50 estimate;
* router: explicit provider, else claude > openai > qwen3 > local subject to budget; per-primary
  fallback chains with `local` last; response cache keyed by sha256(prompt, system), TTL 3600 s,
  1000 entries, oldest evicted (router.rs:34-248).
Streaming is real token streaming (SSE from the OpenAI-compatible / Anthropic APIs, the
runtime's StreamInfer) -- the reference sent one chunk at the end.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import logging
import os
import sqlite3
import threading
import time
from dataclasses import dataclass, field
from typing import AsyncIterator, Dict, List, Optional

log = logging.getLogger("aios.gateway")

try:  # aiohttp ships in this image; keep the module importable without it
    import aiohttp
except Exception:  # pragma: no cover
    aiohttp = None


class ProviderError(RuntimeError):
    pass


@dataclass
class Completion:
    text: str
    tokens_used: int
    latency_ms: int
    model_used: str
    input_tokens: int = 0
    output_tokens: int = 0
    provider: str = ""


def wants_json(prompt: str, system_prompt: str) -> bool:
    return ("valid JSON" in prompt or "JSON object" in prompt or "respond with ONLY valid JSON" in system_prompt)


# ------------------------------------------------------------------------------------ providers
class Provider:
    name = ""
    price_in = 0.0   # USD per 1M tokens
    price_out = 0.0

    def available(self) -> bool:
        raise NotImplementedError

    async def infer(self, prompt, system_prompt, max_tokens, temperature) -> Completion:
        raise NotImplementedError

    async def stream(self, prompt, system_prompt, max_tokens, temperature) -> AsyncIterator[str]:
        c = await self.infer(prompt, system_prompt, max_tokens, temperature)
        yield c.text

    def cost(self, tin: int, tout: int) -> float:
        return tin * self.price_in / 1e6 + tout * self.price_out / 1e6


def _defaults(max_tokens: int, temperature: float):
    return (max_tokens if max_tokens > 0 else 4096), (temperature if temperature > 0 else 0.3)


class _Http:
    _session: Optional["aiohttp.ClientSession"] = None

    @classmethod
    def session(cls) -> "aiohttp.ClientSession":
        if aiohttp is None:
            raise ProviderError("aiohttp not available")
        if cls._session is None or cls._session.closed:
            cls._session = aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=300))
        return cls._session

    @classmethod
    async def close(cls):
        if cls._session is not None and not cls._session.closed:
            await cls._session.close()


class OpenAICompatible(Provider):
    def __init__(self, name: str, api_key: str, base_url: str, model: str, price_in=0.0, price_out=0.0,
                 always_available: bool = False):
        self.name, self.api_key, self.base_url, self.model = name, api_key, base_url.rstrip("/"), model
        self.price_in, self.price_out = price_in, price_out
        self.always_available = always_available

    def available(self) -> bool:
        return self.always_available or bool(self.api_key)

    def _body(self, prompt, system_prompt, max_tokens, temperature, stream):
        mt, t = _defaults(max_tokens, temperature)
        msgs = ([{"role": "system", "content": system_prompt}] if system_prompt else []) + \
            [{"role": "user", "content": prompt}]
        body = {"model": self.model, "messages": msgs, "max_tokens": mt, "temperature": t}
        if wants_json(prompt, system_prompt):
            body["response_format"] = {"type": "json_object"}
        if stream:
            body["stream"] = True
        return body

    def _headers(self):
        h = {"Content-Type": "application/json"}
        if self.api_key:
            h["Authorization"] = f"Bearer {self.api_key}"
        return h

    async def infer(self, prompt, system_prompt, max_tokens, temperature) -> Completion:
        if not self.available():
            raise ProviderError(f"{self.name} API key not configured")
        t0 = time.time()
        try:
            async with _Http.session().post(f"{self.base_url}/v1/chat/completions", headers=self._headers(),
                                            json=self._body(prompt, system_prompt, max_tokens, temperature,
                                                            False)) as r:
                if r.status != 200:
                    raise ProviderError(f"{self.name} API error {r.status}: {(await r.text())[:500]}")
                data = await r.json(content_type=None)
        except (aiohttp.ClientError, asyncio.TimeoutError) as e:
            raise ProviderError(f"{self.name} unreachable: {e}") from e
        choice = (data.get("choices") or [{}])[0]
        text = (choice.get("message") or {}).get("content") or ""
        usage = data.get("usage") or {}
        tin, tout = int(usage.get("prompt_tokens", 0)), int(usage.get("completion_tokens", 0))
        return Completion(text=text, tokens_used=int(usage.get("total_tokens", tin + tout)),
                          latency_ms=int((time.time() - t0) * 1000), model_used=data.get("model", self.model),
                          input_tokens=tin, output_tokens=tout, provider=self.name)

    async def stream(self, prompt, system_prompt, max_tokens, temperature):
        if not self.available():
            raise ProviderError(f"{self.name} API key not configured")
        try:
            async with _Http.session().post(f"{self.base_url}/v1/chat/completions", headers=self._headers(),
                                            json=self._body(prompt, system_prompt, max_tokens, temperature,
                                                            True)) as r:
                if r.status != 200:
                    raise ProviderError(f"{self.name} API error {r.status}: {(await r.text())[:500]}")
                async for raw in r.content:
                    line = raw.decode("utf-8", "replace").strip()
                    if not line.startswith("data:"):
                        continue
                    payload = line[5:].strip()
                    if payload == "[DONE]":
                        break
                    try:
                        delta = json.loads(payload)["choices"][0].get("delta", {}).get("content")
                    except (ValueError, KeyError, IndexError):
                        continue
                    if delta:
                        yield delta
        except (aiohttp.ClientError, asyncio.TimeoutError) as e:
            raise ProviderError(f"{self.name} unreachable: {e}") from e


class Claude(Provider):
    name = "claude"
    price_in, price_out = 3.0, 15.0

    def __init__(self, api_key: str, model: str, base_url: str = "https://api.anthropic.com"):
        self.api_key, self.model, self.base_url = api_key, model, base_url

    def available(self) -> bool:
        return bool(self.api_key)

    def _req(self, prompt, system_prompt, max_tokens, temperature, stream):
        mt, t = _defaults(max_tokens, temperature)
        body = {"model": self.model, "max_tokens": mt, "temperature": t, "system": system_prompt,
                "messages": [{"role": "user", "content": prompt}]}
        if stream:
            body["stream"] = True
        hdr = {"x-api-key": self.api_key, "anthropic-version": "2023-06-01", "content-type": "application/json"}
        return body, hdr

    async def infer(self, prompt, system_prompt, max_tokens, temperature) -> Completion:
        if not self.available():
            raise ProviderError("Claude API key not configured")
        body, hdr = self._req(prompt, system_prompt, max_tokens, temperature, False)
        t0 = time.time()
        try:
            async with _Http.session().post(f"{self.base_url}/v1/messages", headers=hdr, json=body) as r:
                if r.status != 200:
                    raise ProviderError(f"Claude API error {r.status}: {(await r.text())[:500]}")
                data = await r.json(content_type=None)
        except (aiohttp.ClientError, asyncio.TimeoutError) as e:
            raise ProviderError(f"claude unreachable: {e}") from e
        text = "".join(c.get("text", "") for c in data.get("content", []) if c.get("type") == "text")
        u = data.get("usage") or {}
        tin, tout = int(u.get("input_tokens", 0)), int(u.get("output_tokens", 0))
        return Completion(text=text, tokens_used=tin + tout, latency_ms=int((time.time() - t0) * 1000),
                          model_used=data.get("model", self.model), input_tokens=tin, output_tokens=tout,
                          provider=self.name)

    async def stream(self, prompt, system_prompt, max_tokens, temperature):
        if not self.available():
            raise ProviderError("Claude API key not configured")
        body, hdr = self._req(prompt, system_prompt, max_tokens, temperature, True)
        try:
            async with _Http.session().post(f"{self.base_url}/v1/messages", headers=hdr, json=body) as r:
                if r.status != 200:
                    raise ProviderError(f"Claude API error {r.status}: {(await r.text())[:500]}")
                async for raw in r.content:
                    line = raw.decode("utf-8", "replace").strip()
                    if not line.startswith("data:"):
                        continue
                    try:
                        ev = json.loads(line[5:])
                    except ValueError:
                        continue
                    if ev.get("type") == "content_block_delta":
                        t = (ev.get("delta") or {}).get("text")
                        if t:
                            yield t
                    elif ev.get("type") == "message_stop":
                        break
        except (aiohttp.ClientError, asyncio.TimeoutError) as e:
            raise ProviderError(f"claude unreachable: {e}") from e


class LocalRuntime(OpenAICompatible):
    """`local`: the MI355X runtime.  HTTP first (LOCAL_LLM_URL), then AIRuntime gRPC."""

    def __init__(self, base_url: str, model: str, runtime_addr: str):
        super().__init__("local", "", base_url, model, always_available=True)
        self.runtime_addr = runtime_addr

    def _grpc_model(self) -> str:
        return "" if self.model == "local" else self.model

    async def infer(self, prompt, system_prompt, max_tokens, temperature) -> Completion:
        try:
            return await super().infer(prompt, system_prompt, max_tokens, temperature)
        except ProviderError as http_err:
            if "unreachable" not in str(http_err):
                raise
        from ..rpc.client import Stub, channel
        from ..rpc.schema import pb

        import grpc

        mt, t = _defaults(max_tokens, temperature)
        t0 = time.time()
        try:
            r = await Stub(channel(self.runtime_addr), "aios.runtime.AIRuntime").Infer(pb.runtime.InferRequest(
                model=self._grpc_model(), prompt=prompt, system_prompt=system_prompt, max_tokens=mt,
                temperature=t, intelligence_level="strategic", requesting_agent="api-gateway"), timeout=300)
        except grpc.aio.AioRpcError as e:
            raise ProviderError(f"local runtime unavailable: {e.details()}") from e
        return Completion(text=r.text, tokens_used=r.tokens_used, latency_ms=int((time.time() - t0) * 1000),
                          model_used=r.model_used, output_tokens=r.tokens_used, provider="local")

    async def stream(self, prompt, system_prompt, max_tokens, temperature):
        try:
            async for piece in super().stream(prompt, system_prompt, max_tokens, temperature):
                yield piece
            return
        except ProviderError as http_err:
            if "unreachable" not in str(http_err):
                raise
        from ..rpc.client import Stub, channel
        from ..rpc.schema import pb

        mt, t = _defaults(max_tokens, temperature)
        call = Stub(channel(self.runtime_addr), "aios.runtime.AIRuntime").StreamInfer(pb.runtime.InferRequest(
            model=self._grpc_model(), prompt=prompt, system_prompt=system_prompt, max_tokens=mt, temperature=t,
            intelligence_level="strategic", requesting_agent="api-gateway"))
        async for chunk in call:
            if chunk.text:
                yield chunk.text
            if chunk.done:
                break


def secret_keys(path: str = "") -> Dict[str, str]:
    """Provider keys from the secrets file (`$AIOS_SECRETS` or /etc/aios/secrets.toml, TTL cache +
    0600 check in the native SecretManager -- tools/src/secrets.rs, unwired in the reference)."""
    path = path or os.environ.get("AIOS_SECRETS", "/etc/aios/secrets.toml")
    if not os.path.exists(path):
        return {}
    try:
        from ..core import load as load_core

        sm = load_core().SecretManager(path)
        sm.load()
        for w in sm.warnings():
            log.warning("secrets: %s", w)
        return {k: v for k, v in sm.api_keys().items() if v}
    except Exception as e:  # pragma: no cover - native core missing
        log.warning("secrets file %s not read: %s", path, e)
        return {}


def providers_from_env(env=os.environ) -> Dict[str, Provider]:
    keys = secret_keys(env.get("AIOS_SECRETS", ""))
    return {
        "claude": Claude(env.get("CLAUDE_API_KEY", "") or keys.get("claude", ""),
                         env.get("CLAUDE_MODEL", "claude-sonnet-4-20250514")),
        "openai": OpenAICompatible("openai", env.get("OPENAI_API_KEY", "") or keys.get("openai", ""),
                                   env.get("OPENAI_BASE_URL", "https://api.openai.com"),
                                   env.get("OPENAI_MODEL", "gpt-5"), 2.5, 10.0),
        "qwen3": OpenAICompatible("qwen3", env.get("QWEN3_API_KEY", "") or keys.get("qwen3", ""),
                                  env.get("QWEN3_BASE_URL", "https://api.viwoapp.net"),
                                  env.get("QWEN3_MODEL", "qwen3:30b-128k")),
        "local": LocalRuntime(env.get("LOCAL_LLM_URL", "http://127.0.0.1:8082"), env.get("LOCAL_LLM_MODEL", "local"),
                              env.get("AIOS_RUNTIME_ADDR", "127.0.0.1:50055").replace("[::]", "127.0.0.1")),
    }


# ------------------------------------------------------------------------------------ budget
def _month_start(t: Optional[float] = None) -> int:
    tm = time.gmtime(t if t is not None else time.time())
    return int(time.mktime((tm.tm_year, tm.tm_mon, 1, 0, 0, 0, 0, 0, 0)) - time.timezone)


class BudgetManager:
    def __init__(self, claude_budget=100.0, openai_budget=50.0, db_path: str = ":memory:"):
        self.claude_budget, self.openai_budget = claude_budget, openai_budget
        self.lock = threading.Lock()
        if db_path != ":memory:":
            os.makedirs(os.path.dirname(db_path) or ".", exist_ok=True)
        self.db = sqlite3.connect(db_path, check_same_thread=False)
        self.db.execute("CREATE TABLE IF NOT EXISTS usage (provider TEXT, model TEXT, input_tokens INTEGER,"
                        " output_tokens INTEGER, cost_usd REAL, timestamp INTEGER, requesting_agent TEXT,"
                        " task_id TEXT)")
        self.db.commit()
        self.month_start = _month_start()

    def _used(self, provider: str) -> float:
        row = self.db.execute("SELECT COALESCE(SUM(cost_usd), 0) FROM usage WHERE provider = ? AND timestamp >= ?",
                              (provider, self.month_start)).fetchone()
        return float(row[0])

    def _maybe_reset(self):
        ms = _month_start()
        if ms > self.month_start:
            log.info("new billing month: budget counters reset")
            self.month_start = ms

    def record(self, provider: str, c: Completion, cost: float, agent: str = "", task: str = ""):
        tin, tout = c.input_tokens, c.output_tokens
        if tin == 0 and tout == 0 and c.tokens_used:
            tin, tout = c.tokens_used // 2, c.tokens_used - c.tokens_used // 2
        with self.lock:
            self._maybe_reset()
            self.db.execute("INSERT INTO usage VALUES (?,?,?,?,?,?,?,?)",
                            (provider, c.model_used, tin, tout, cost, int(time.time()), agent, task))
            self.db.commit()
            for p, b in (("claude", self.claude_budget), ("openai", self.openai_budget)):
                u = self._used(p)
                if b > 0 and u > 0.8 * b:
                    log.warning("%s budget warning: $%.2f / $%.2f (%d%%)", p, u, b, int(100 * u / b))

    def provider_exceeded(self, provider: str) -> bool:
        with self.lock:
            self._maybe_reset()
            if provider == "claude":
                return self._used("claude") >= self.claude_budget
            if provider == "openai":
                return self._used("openai") >= self.openai_budget
            return False  # qwen3 / local are not metered

    def exceeded(self) -> bool:
        return self.provider_exceeded("claude") and self.provider_exceeded("openai")

    def status(self) -> dict:
        with self.lock:
            self._maybe_reset()
            cu, ou = self._used("claude"), self._used("openai")
        day = time.gmtime().tm_mday
        return {"claude_monthly_budget_usd": self.claude_budget, "claude_used_usd": cu,
                "openai_monthly_budget_usd": self.openai_budget, "openai_used_usd": ou,
                "days_remaining": max(0, 30 - day), "daily_rate_usd": (cu + ou) / max(day, 1),
                "budget_exceeded": cu >= self.claude_budget and ou >= self.openai_budget}

    def usage(self, provider: str = "", days: int = 30) -> dict:
        cutoff = int(time.time()) - max(days, 0) * 86400 if days > 0 else 0
        q = "SELECT provider, model, input_tokens, output_tokens, cost_usd, timestamp, requesting_agent, task_id " \
            "FROM usage WHERE timestamp >= ?"
        args: list = [cutoff]
        if provider:
            q += " AND provider = ?"
            args.append(provider)
        with self.lock:
            rows = self.db.execute(q + " ORDER BY timestamp", args).fetchall()
        keys = ("provider", "model", "input_tokens", "output_tokens", "cost_usd", "timestamp", "requesting_agent",
                "task_id")
        recs = [dict(zip(keys, r)) for r in rows]
        return {"records": recs, "total_cost_usd": sum(r["cost_usd"] for r in recs), "total_requests": len(recs),
                "total_tokens": sum(r["input_tokens"] + r["output_tokens"] for r in recs)}


# ------------------------------------------------------------------------------------ router
FALLBACKS = {
    "claude": ["openai", "qwen3", "local"],
    "openai": ["claude", "qwen3", "local"],
    "qwen3": ["claude", "openai", "local"],
    "local": ["qwen3", "claude", "openai"],
}


@dataclass
class _Cached:
    resp: Completion
    at: float


class RequestRouter:
    def __init__(self, providers: Dict[str, Provider], budget: BudgetManager, ttl: float = 3600.0,
                 max_entries: int = 1000):
        self.providers, self.budget = providers, budget
        self.ttl, self.max_entries = ttl, max_entries
        self.cache: Dict[str, _Cached] = {}
        self.stats = {"requests": 0, "cache_hits": 0, "fallbacks": 0, "errors": 0}

    @staticmethod
    def key(prompt: str, system_prompt: str) -> str:
        h = hashlib.sha256()
        h.update(prompt.encode())
        h.update(b"\x00")
        h.update(system_prompt.encode())
        return h.hexdigest()

    def select(self, preferred: str) -> str:
        if preferred:
            return preferred
        for p in ("claude", "openai", "qwen3"):
            if self.providers[p].available() and not self.budget.provider_exceeded(p):
                return p
        return "local"

    def chain(self, primary: str, allow_fallback: bool) -> List[str]:
        return [primary] + (FALLBACKS.get(primary, ["local"]) if allow_fallback else [])

    def _cache_get(self, k: str) -> Optional[Completion]:
        c = self.cache.get(k)
        if c is None:
            return None
        if time.time() - c.at >= self.ttl:
            del self.cache[k]
            return None
        return c.resp

    def _cache_put(self, k: str, resp: Completion):
        if k not in self.cache and len(self.cache) >= self.max_entries:
            oldest = min(self.cache, key=lambda x: self.cache[x].at)
            del self.cache[oldest]
        self.cache[k] = _Cached(resp, time.time())

    async def _try(self, name: str, req) -> Completion:
        p = self.providers.get(name)
        if p is None:
            raise ProviderError(f"Unknown provider: {name}")
        if not p.available():
            raise ProviderError(f"{name} API key not configured")
        if self.budget.provider_exceeded(name):
            raise ProviderError(f"{name} budget exceeded")
        c = await p.infer(req.prompt, req.system_prompt, req.max_tokens, req.temperature)
        tin, tout = c.input_tokens, c.output_tokens
        if tin == 0 and tout == 0:
            tin, tout = c.tokens_used // 2, c.tokens_used - c.tokens_used // 2
        self.budget.record(name, c, p.cost(tin, tout), req.requesting_agent, req.task_id)
        return c

    async def route(self, req) -> Completion:
        self.stats["requests"] += 1
        k = self.key(req.prompt, req.system_prompt)
        hit = self._cache_get(k)
        if hit is not None:
            self.stats["cache_hits"] += 1
            return hit
        primary = self.select(req.preferred_provider)
        last: Optional[Exception] = None
        for i, name in enumerate(self.chain(primary, req.allow_fallback)):
            try:
                c = await self._try(name, req)
                if i:
                    self.stats["fallbacks"] += 1
                    log.info("fallback to %s succeeded", name)
                self._cache_put(k, c)
                return c
            except ProviderError as e:
                log.info("%s failed: %s", name, e)
                last = e
        self.stats["errors"] += 1
        raise ProviderError(str(last) if last else "no provider available")

    async def stream(self, req):
        """(provider, async-iterator of text pieces) for the first provider that starts streaming."""
        primary = self.select(req.preferred_provider)
        last: Optional[Exception] = None
        for name in self.chain(primary, req.allow_fallback):
            p = self.providers.get(name)
            if p is None or not p.available() or self.budget.provider_exceeded(name):
                continue
            it = p.stream(req.prompt, req.system_prompt, req.max_tokens, req.temperature).__aiter__()
            try:
                first = await it.__anext__()
            except StopAsyncIteration:
                first = ""
            except ProviderError as e:
                last = e
                continue
            return name, first, it
        raise ProviderError(str(last) if last else "no provider available")

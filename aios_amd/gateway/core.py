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

The ledger, the cache and the routing policy are the native C++ core (`aios_amd/native/gateway.cpp`,
`_core.gateway`); this module keeps only the provider HTTP clients (aiohttp, streaming) and the
asyncio request flow.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time
from dataclasses import dataclass
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


def _gw():
    from ..core import load as load_core

    return load_core().gateway


def wants_json(prompt: str, system_prompt: str) -> bool:
    return _gw().wants_json(prompt, system_prompt)


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
        if self.name in ("claude", "openai"):  # the native price table (gateway.cpp gw_cost)
            return _gw().cost(self.name, int(tin), int(tout))
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
class BudgetManager:
    """Monthly budget ledger over the native `_core.gateway.BudgetLedger` (SQLite, persisted)."""

    def __init__(self, claude_budget=100.0, openai_budget=50.0, db_path: str = ":memory:"):
        if db_path != ":memory:":
            os.makedirs(os.path.dirname(db_path) or ".", exist_ok=True)
        self.ledger = _gw().BudgetLedger(float(claude_budget), float(openai_budget), db_path)
        self.claude_budget, self.openai_budget = float(claude_budget), float(openai_budget)

    def record(self, provider: str, c: Completion, cost: float, agent: str = "", task: str = ""):
        for w in self.ledger.record(provider, c.model_used, int(c.input_tokens), int(c.output_tokens),
                                    int(c.tokens_used), float(cost), agent, task):
            log.warning("%s", w)

    def provider_exceeded(self, provider: str) -> bool:
        return self.ledger.provider_exceeded(provider)

    def exceeded(self) -> bool:
        return self.ledger.exceeded()

    def status(self) -> dict:
        s = self.ledger.status()
        return {k: (float(v) if k.endswith("_usd") else v) for k, v in s.items()}

    def usage(self, provider: str = "", days: int = 30) -> dict:
        u = self.ledger.usage(provider, int(days))
        u["total_cost_usd"] = float(u["total_cost_usd"])
        for r in u["records"]:
            r["cost_usd"] = float(r["cost_usd"])
        return u


# ------------------------------------------------------------------------------------ router
class RequestRouter:
    def __init__(self, providers: Dict[str, Provider], budget: BudgetManager, ttl: float = 3600.0,
                 max_entries: int = 1000):
        self.providers, self.budget = providers, budget
        self.ttl = float(ttl)
        self.max_entries = max_entries  # builds the native cache
        self.stats = {"requests": 0, "cache_hits": 0, "fallbacks": 0, "errors": 0}

    @property
    def max_entries(self) -> int:
        return self._max_entries

    @max_entries.setter
    def max_entries(self, n: int):
        """Re-sizing starts an empty cache (the native cache's capacity is fixed)."""
        self._max_entries = int(n)
        self.cache = _gw().ResponseCache(self.ttl, self._max_entries)

    @staticmethod
    def key(prompt: str, system_prompt: str) -> str:
        return _gw().ResponseCache.key(prompt, system_prompt)

    def select(self, preferred: str) -> str:
        avail = {p: bool(self.providers[p].available()) for p in ("claude", "openai", "qwen3") if p in self.providers}
        return _gw().select(preferred, avail, self.budget.ledger)

    def chain(self, primary: str, allow_fallback: bool) -> List[str]:
        return list(_gw().chain(primary, allow_fallback))

    def _cache_get(self, k: str) -> Optional[Completion]:
        c = self.cache.get(k)
        if c is None:
            return None
        return Completion(text=c.text, tokens_used=c.tokens_used, latency_ms=c.latency_ms, model_used=c.model_used,
                          input_tokens=c.input_tokens, output_tokens=c.output_tokens, provider=c.provider)

    def _cache_put(self, k: str, resp: Completion):
        self.cache.put(k, _gw().Completion(resp.text, int(resp.tokens_used), int(resp.latency_ms), resp.model_used,
                                           int(resp.input_tokens), int(resp.output_tokens), resp.provider))

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

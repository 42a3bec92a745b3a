"""AIRuntime gRPC service (:50055) + per-model OpenAI-compatible HTTP endpoints.

RPC semantics follow the reference (`runtime/src/grpc_service.rs:28-178`,
`runtime/src/inference.rs:94-186`): unary Infer always uses JSON mode, max_tokens <= 0 -> 512,
temperature == 0 -> 0.7 (API-compatible default; a *negative* temperature requests greedy
decoding, App. A #3), tokens_used = prompt + completion, latency_ms = wall time.  StreamInfer
streams real token deltas as they are generated (App. A #2).

HTTP (per loaded model on its `ModelStatus.port`, like llama-server): POST /v1/chat/completions
(+ `stream: true` SSE, `response_format: {"type":"json_object"}`) and GET /health -- so the
gateway's `local` provider (`LOCAL_LLM_URL`, default :8082) can reach the local strategic tier.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time
from typing import Dict, Optional

import grpc

from ..rpc.schema import pb
from .chat_template import build_messages
from .model_manager import ModelManager, RoutingError
from .scheduler import GenRequest, GenResult

log = logging.getLogger("aios.runtime.service")


def _gen_params(temperature: float, max_tokens: int):
    if max_tokens <= 0:
        max_tokens = 512
    if temperature < 0:
        temperature = 0.0
    elif temperature == 0:
        temperature = 0.7
    return float(temperature), int(max_tokens)


def _json_min_tokens(max_tokens: int) -> int:
    """AIOS_JSON_MIN_TOKENS (benchmarks only): JSON-mode generations run to this many tokens before
    the grammar lets the object close ("max": to max_tokens) -- a fixed plan length, since
    random-init weights close a JSON object at arbitrary points."""
    v = os.environ.get("AIOS_JSON_MIN_TOKENS", "").strip()
    if not v:
        return 0
    return max_tokens if v == "max" else min(max_tokens, int(v))


async def generate(m, messages, max_tokens: int, temperature: float, json_mode: bool, on_delta=None,
                   timeout: float = 120.0, seed: int = 0) -> GenResult:
    loop = asyncio.get_running_loop()
    fut = loop.create_future()
    prompt = m.template.render(messages, add_generation_prompt=True)
    ids = m.tokenizer.encode(prompt)

    def done(res):
        loop.call_soon_threadsafe(lambda: fut.done() or fut.set_result(res))

    delta_cb = None
    if on_delta is not None:
        def delta_cb(d):
            loop.call_soon_threadsafe(on_delta, d)
    req = GenRequest(prompt_ids=ids, max_tokens=max_tokens, temperature=temperature, json_mode=json_mode,
                     min_tokens=_json_min_tokens(max_tokens) if json_mode else 0, seed=seed, on_delta=delta_cb, on_done=done, deadline=time.time() + timeout)
    m.scheduler.submit(req)
    try:
        return await asyncio.wait_for(fut, timeout + 5)
    except asyncio.TimeoutError:
        req.cancelled = True
        raise


class AIRuntimeService:
    def __init__(self, manager: ModelManager, http: bool = True):
        self.mgr = manager
        self.http = http
        self._http_runners: Dict[str, object] = {}
        manager.unload_hooks.append(self._drop_http)

    async def _drop_http(self, name: str):
        runner = self._http_runners.pop(name, None)
        if runner is not None:
            await runner.cleanup()

    async def _route(self, request):
        """Resolve (loading an on-demand tier when needed) and expose a freshly loaded model's
        OpenAI-compatible endpoint."""
        m = await self.mgr.resolve_async(request.model, request.intelligence_level)
        if self.http and m.name not in self._http_runners:
            await self.start_http(m)
        return m

    async def _abort(self, context, e: RoutingError):
        await context.abort(getattr(grpc.StatusCode, e.code), str(e))

    @staticmethod
    def _status(m) -> object:
        return pb.runtime.ModelStatus(model_name=m.name, status=m.status_string(), port=m.port, loaded_at=m.loaded_at,
                                      last_used=m.last_used, request_count=m.request_count)

    async def LoadModel(self, request, context):
        name = request.model_name or (request.model_path.split("/")[-1].rsplit(".", 1)[0] if request.model_path else "")
        if not name or not request.model_path:
            await context.abort(grpc.StatusCode.INVALID_ARGUMENT, "model_name and model_path are required")
        m = await self.mgr.load_model(name, request.model_path, request.context_length, request.port)
        if m.status == "ready" and self.http:
            await self.start_http(m)
        return self._status(m)

    async def UnloadModel(self, request, context):
        ok = await self.mgr.unload_model(request.model_name)
        return pb.common.Status(success=ok, message="unloaded" if ok else f"model {request.model_name} not found")

    async def ListModels(self, request, context):
        return pb.runtime.ModelList(models=[self._status(m) for m in self.mgr.list_models()])

    def _engine_failed(self, m) -> bool:
        """The model's engine (not the request) failed: take it out of routing."""
        sch = m.scheduler
        if sch is not None and sch.failed:
            self.mgr.fail_model(m, f"engine failure: {sch.failed}")
            return True
        return m.status != "ready"

    async def Infer(self, request, context):
        try:
            m = await self._route(request)
        except RoutingError as e:
            await self._abort(context, e)
        temperature, max_tokens = _gen_params(request.temperature, request.max_tokens)
        t0 = time.time()
        msgs = build_messages(request.prompt, request.system_prompt)
        res = await generate(m, msgs, max_tokens, temperature, json_mode=True)
        if res.finish_reason == "error" and self._engine_failed(m):
            # e.g. a TP rank timed out: the tier is torn down and the request re-routed once to
            # the next ready model of its level (strategic -> tactical ...)
            log.warning("model %s failed (%s); re-routing the request", m.name, res.error)
            try:
                m = await self._route(request)
            except RoutingError as e:
                await self._abort(context, e)
            res = await generate(m, msgs, max_tokens, temperature, json_mode=True)
        if res.finish_reason == "error":
            await context.abort(grpc.StatusCode.INTERNAL, f"inference failed: {res.error}")
        return pb.runtime.InferResponse(text=res.text, tokens_used=res.prompt_tokens + res.completion_tokens,
                                        latency_ms=int((time.time() - t0) * 1000), model_used=m.name)

    async def StreamInfer(self, request, context):
        try:
            m = await self._route(request)
        except RoutingError as e:
            await self._abort(context, e)
            return
        temperature, max_tokens = _gen_params(request.temperature, request.max_tokens)
        q: asyncio.Queue = asyncio.Queue()
        task = asyncio.ensure_future(generate(m, build_messages(request.prompt, request.system_prompt), max_tokens,
                                              temperature, json_mode=False, on_delta=q.put_nowait))
        task.add_done_callback(lambda _t: q.put_nowait(None))
        while True:
            d = await q.get()
            if d is None:
                break
            yield pb.runtime.InferChunk(text=d, done=False)
        res = task.result()
        if res.finish_reason == "error":
            await context.abort(grpc.StatusCode.INTERNAL, res.error)
        yield pb.runtime.InferChunk(text="", done=True)

    async def HealthCheck(self, request, context):
        models = self.mgr.list_models()
        ready = sum(1 for m in models if m.status == "ready")
        h = pb.common.HealthStatus(healthy=True, service="aios-runtime",
                                   message=f"{ready}/{len(models)} models ready",
                                   uptime_seconds=int(time.time() - self.mgr.started))
        for k, v in self.mgr.health().items():
            h.details[k] = v
        try:  # amdgpu RAS / thermal verdict (uncorrectable HBM ECC or xGMI errors -> unhealthy)
            from ..utils import sysinfo

            gh = sysinfo.gpu_health()
            h.details["gpu_ecc_uncorrectable"] = str(gh["ecc_ue_total"])
            h.details["gpu_ecc_correctable"] = str(gh["ecc_ce_total"])
            if not gh["healthy"]:
                h.details["gpu_problems"] = json.dumps(gh["problems"])
                h.message += f"; GPU problems on {len(gh['problems'])} counter(s)"
        except Exception:  # pragma: no cover - no GPU sysfs
            pass
        return h

    # ------------------------------------------------------------------ HTTP (OpenAI-compatible)
    async def start_http(self, m, host: str = "127.0.0.1"):
        from aiohttp import web

        if m.name in self._http_runners:
            return
        app = web.Application()
        app["model"] = m
        app.router.add_get("/health", self._http_health)
        app.router.add_post("/v1/chat/completions", self._http_chat)
        app.router.add_get("/v1/models", self._http_models)
        runner = web.AppRunner(app, access_log=None)
        await runner.setup()
        try:
            await web.TCPSite(runner, host, m.port).start()
            self._http_runners[m.name] = runner
        except OSError as e:
            log.warning("HTTP endpoint for %s on :%d unavailable: %s", m.name, m.port, e)
            await runner.cleanup()

    async def _http_health(self, request):
        from aiohttp import web

        m = request.app["model"]
        return web.json_response({"status": "ok" if m.status == "ready" else m.status})

    async def _http_models(self, request):
        from aiohttp import web

        m = request.app["model"]
        return web.json_response({"object": "list", "data": [{"id": m.name, "object": "model"}]})

    async def _http_chat(self, request):
        from aiohttp import web

        m = request.app["model"]
        body = await request.json()
        messages = body.get("messages") or []
        max_tokens = int(body.get("max_tokens") or 512)
        temperature = float(body.get("temperature", 0.7))
        json_mode = (body.get("response_format") or {}).get("type") == "json_object"
        created = int(time.time())
        rid = f"chatcmpl-{created}{id(request) & 0xffff:04x}"
        if body.get("stream"):
            resp = web.StreamResponse(headers={"Content-Type": "text/event-stream"})
            await resp.prepare(request)
            q: asyncio.Queue = asyncio.Queue()
            task = asyncio.ensure_future(generate(m, messages, max_tokens, temperature, json_mode, on_delta=q.put_nowait))
            task.add_done_callback(lambda _t: q.put_nowait(None))
            while True:
                d = await q.get()
                if d is None:
                    break
                chunk = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": m.name,
                         "choices": [{"index": 0, "delta": {"content": d}, "finish_reason": None}]}
                await resp.write(f"data: {json.dumps(chunk)}\n\n".encode())
            res = task.result()
            end = {"id": rid, "object": "chat.completion.chunk", "created": created, "model": m.name,
                   "choices": [{"index": 0, "delta": {}, "finish_reason": "stop" if res.finish_reason != "length" else "length"}]}
            await resp.write(f"data: {json.dumps(end)}\n\ndata: [DONE]\n\n".encode())
            await resp.write_eof()
            return resp
        res = await generate(m, messages, max_tokens, temperature, json_mode)
        return web.json_response({
            "id": rid, "object": "chat.completion", "created": created, "model": m.name,
            "choices": [{"index": 0, "message": {"role": "assistant", "content": res.text},
                         "finish_reason": "length" if res.finish_reason == "length" else "stop"}],
            "usage": {"prompt_tokens": res.prompt_tokens, "completion_tokens": res.completion_tokens,
                      "total_tokens": res.prompt_tokens + res.completion_tokens},
            "timings": {"ttft_ms": res.ttft_ms, "latency_ms": res.latency_ms,
                        "cached_prompt_tokens": res.cached_prompt_tokens},
        })

    async def close(self):
        for r in self._http_runners.values():
            await r.cleanup()
        self._http_runners.clear()
        for m in list(self.mgr.list_models()):
            await self.mgr.unload_model(m.name)

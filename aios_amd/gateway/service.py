"""aios-api-gateway daemon: `aios.api_gateway.ApiGateway` on :50054.

Reference: `api-gateway/src/main.rs` (Infer `:51-92`, StreamInfer `:98-187`, GetBudget,
GetUsage).  The reference serialised every Infer behind one write lock; here requests run
concurrently (the router's cache and the SQLite-backed budget are the only shared state) and
StreamInfer forwards provider tokens as they arrive.
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import time

import grpc

from ..rpc.schema import pb
from ..rpc.server import RpcServer
from ..utils.env import data_dir, setup_logging
from .core import BudgetManager, Completion, ProviderError, RequestRouter, _Http, providers_from_env

log = logging.getLogger("aios.gateway")


class ApiGatewayService:
    def __init__(self, router: RequestRouter):
        self.router = router

    @classmethod
    def from_env(cls, db_path: str = ""):
        from ..utils import config as node_config

        cfg = node_config.load()  # [api] budgets / cache; env vars still win (reference names)
        budget = BudgetManager(float(os.environ.get("AIOS_CLAUDE_BUDGET_USD", cfg.api.claude_monthly_budget_usd)),
                               float(os.environ.get("AIOS_OPENAI_BUDGET_USD", cfg.api.openai_monthly_budget_usd)),
                               db_path or os.path.join(data_dir(), "data", "gateway_usage.db"))
        env = dict(os.environ)
        env.setdefault("AIOS_SECRETS", cfg.security.secrets_file)
        provs = providers_from_env(env)
        log.info("available providers: %s", ", ".join(n for n, p in provs.items() if p.available()))
        return cls(RequestRouter(provs, budget, ttl=float(cfg.api.cache_ttl_seconds),
                                 max_entries=int(cfg.api.cache_max_entries)))

    async def Infer(self, req, ctx):
        log.info("inference request: provider=%s agent=%s task=%s", req.preferred_provider, req.requesting_agent,
                 req.task_id)
        if self.router.budget.exceeded():
            await ctx.abort(grpc.StatusCode.RESOURCE_EXHAUSTED, "API budget exceeded")
        try:
            c = await self.router.route(req)
        except ProviderError as e:
            await ctx.abort(grpc.StatusCode.INTERNAL, f"API request failed: {e}")
        return pb.common.InferenceResponse(text=c.text, tokens_used=c.tokens_used, latency_ms=c.latency_ms,
                                           model_used=c.model_used, intelligence_level="strategic")

    async def StreamInfer(self, req, ctx):
        try:
            provider, first, it = await self.router.stream(req)
        except ProviderError as e:
            await ctx.abort(grpc.StatusCode.INTERNAL, str(e))
            return
        t0, n_chars = time.time(), 0
        if first:
            n_chars += len(first)
            yield pb.api_gateway.StreamChunk(text=first, done=False, provider=provider)
        try:
            async for piece in it:
                n_chars += len(piece)
                yield pb.api_gateway.StreamChunk(text=piece, done=False, provider=provider)
        except ProviderError as e:
            log.warning("stream from %s broke: %s", provider, e)
        yield pb.api_gateway.StreamChunk(text="", done=True, provider=provider)
        # streamed usage is estimated (4 chars/token) -- providers do not report it on SSE
        p = self.router.providers[provider]
        tin, tout = (len(req.prompt) + len(req.system_prompt)) // 4, n_chars // 4
        self.router.budget.record(provider, Completion("", tin + tout, int((time.time() - t0) * 1000), provider,
                                                       tin, tout, provider), p.cost(tin, tout),
                                  req.requesting_agent, req.task_id)

    async def GetBudget(self, req, ctx):
        return pb.api_gateway.BudgetStatus(**self.router.budget.status())

    async def GetUsage(self, req, ctx):
        u = self.router.budget.usage(req.provider, req.days or 30)
        return pb.api_gateway.UsageResponse(records=[pb.api_gateway.UsageRecord(**r) for r in u["records"]],
                                            total_cost_usd=u["total_cost_usd"], total_requests=u["total_requests"],
                                            total_tokens=u["total_tokens"])


async def amain(args):
    svc = ApiGatewayService.from_env(args.usage_db)
    server = RpcServer(args.addr, {"aios.api_gateway.ApiGateway": svc})
    await server.start()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except NotImplementedError:
            pass
    await stop.wait()
    await server.stop()
    await _Http.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description="aiOS API gateway (aios.api_gateway.ApiGateway)")
    ap.add_argument("--addr", default=os.environ.get("AIOS_API_GATEWAY_LISTEN", "0.0.0.0:50054"))
    ap.add_argument("--usage-db", default="")
    args = ap.parse_args(argv)
    setup_logging("aios-api-gateway")
    asyncio.run(amain(args))


if __name__ == "__main__":
    main()

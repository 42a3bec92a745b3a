"""aios-memory daemon: `aios.memory.MemoryService` (24 RPCs) on :50053 over the native store.

Reference: `memory/src/main.rs` (RPCs `:45-350`, AssembleContext `:353-480`, main `:487-521`).
Storage, embeddings, hybrid search and context packing run in C++ (`aios_amd/native/memory.cpp`);
this file maps protobuf records to the store and owns the background work:

* the tier-migration pipeline (`memory/src/migration.rs`) runs hourly -- the reference defined
  it but never started it;
* every 15 s a host/GPU telemetry sample (procfs + amdgpu sysfs) is written into the
  operational metrics, so GetSystemSnapshot is meaningful even without external publishers.
The knowledge base is persisted to `knowledge.db` (the reference's was in-memory only).
"""
from __future__ import annotations

import argparse
import asyncio
import concurrent.futures as cf
import logging
import os
import signal
import time

from ..core import load as load_core
from ..rpc.convert import from_dict, to_dict
from ..rpc.schema import pb
from ..rpc.server import RpcServer
from ..utils import sysinfo
from ..utils.env import data_dir, setup_logging

log = logging.getLogger("aios.memory")
MIGRATION_INTERVAL = 3600.0
TELEMETRY_INTERVAL = 15.0
M = pb.memory


def _tier(name: str) -> str:
    # the orchestrator asks for "long_term" (autonomy.rs:856); the store calls it "longterm"
    return "longterm" if name in ("long_term", "long-term") else name


class MemoryServiceImpl:
    def __init__(self, working_db: str, longterm_db: str, knowledge_db: str):
        core = load_core()
        for p in (working_db, longterm_db, knowledge_db):
            if p != ":memory:":
                os.makedirs(os.path.dirname(p) or ".", exist_ok=True)
        self.store = core.MemoryStore(working_db, longterm_db, knowledge_db)
        self.pool = cf.ThreadPoolExecutor(max_workers=4, thread_name_prefix="mem")
        self.started = time.time()

    async def _run(self, fn, *a):
        return await asyncio.get_running_loop().run_in_executor(self.pool, fn, *a)

    # ------------------------------------------------------------- operational
    async def PushEvent(self, req, ctx):
        ev = to_dict(req)
        if not ev["timestamp"]:
            ev["timestamp"] = int(time.time())
        self.store.push_event(ev)
        return M.Empty()

    async def GetRecentEvents(self, req, ctx):
        evs = self.store.recent_events(req.count or 100, req.category, req.source)
        return M.EventList(events=[from_dict(M.Event, e) for e in evs])

    async def UpdateMetric(self, req, ctx):
        self.store.update_metric(req.key, req.value, req.timestamp or int(time.time()))
        return M.Empty()

    async def GetMetric(self, req, ctx):
        v = self.store.get_metric(req.key)
        if v is None:
            return M.MetricValue(key=req.key)
        return M.MetricValue(key=req.key, value=v[0], timestamp=v[1])

    async def GetSystemSnapshot(self, req, ctx):
        return from_dict(M.SystemSnapshot, self.store.snapshot())

    # ------------------------------------------------------------- working
    async def StoreGoal(self, req, ctx):
        await self._run(self.store.store_goal, to_dict(req))
        return M.Empty()

    async def UpdateGoal(self, req, ctx):
        await self._run(self.store.update_goal, req.id, req.status, req.result)
        return M.Empty()

    async def GetActiveGoals(self, req, ctx):
        return M.GoalList(goals=[from_dict(M.GoalRecord, g) for g in await self._run(self.store.active_goals)])

    async def StoreTask(self, req, ctx):
        await self._run(self.store.store_task, to_dict(req))
        return M.Empty()

    async def GetTasksForGoal(self, req, ctx):
        ts = await self._run(self.store.tasks_for_goal, req.goal_id)
        return M.TaskList(tasks=[from_dict(M.TaskRecord, t) for t in ts])

    async def StoreToolCall(self, req, ctx):
        await self._run(self.store.store_tool_call, to_dict(req))
        return M.Empty()

    async def StoreDecision(self, req, ctx):
        await self._run(self.store.store_decision, to_dict(req))
        return M.Empty()

    async def StorePattern(self, req, ctx):
        await self._run(self.store.store_pattern, to_dict(req))
        return M.Empty()

    async def FindPattern(self, req, ctx):
        p = await self._run(self.store.find_pattern, req.trigger, req.min_success_rate)
        if not p or not p.get("id"):
            return M.PatternResult(found=False)
        return M.PatternResult(pattern=from_dict(M.Pattern, p), found=True)

    async def UpdatePatternStats(self, req, ctx):
        await self._run(self.store.update_pattern_stats, req.id, req.success)
        return M.Empty()

    async def StoreAgentState(self, req, ctx):
        await self._run(self.store.store_agent_state, req.agent_name, req.state_json.decode("utf-8", "replace"))
        return M.Empty()

    async def GetAgentState(self, req, ctx):
        return from_dict(M.AgentState, await self._run(self.store.agent_state, req.agent_name))

    # ------------------------------------------------------------- long-term + knowledge
    async def SemanticSearch(self, req, ctx):
        res = await self._run(self.store.semantic_search, req.query, [_tier(c) for c in req.collections],
                              req.n_results or 5, req.min_relevance)
        return M.SearchResults(results=[from_dict(M.SearchResult, r) for r in res])

    async def StoreProcedure(self, req, ctx):
        await self._run(self.store.store_procedure, to_dict(req))
        return M.Empty()

    async def StoreIncident(self, req, ctx):
        await self._run(self.store.store_incident, to_dict(req))
        return M.Empty()

    async def StoreConfigChange(self, req, ctx):
        await self._run(self.store.store_config_change, to_dict(req))
        return M.Empty()

    async def SearchKnowledge(self, req, ctx):
        res = await self._run(self.store.search_knowledge, req.query, req.n_results or 5, req.min_relevance)
        return M.SearchResults(results=[from_dict(M.SearchResult, r) for r in res])

    async def AddKnowledge(self, req, ctx):
        await self._run(self.store.add_knowledge, to_dict(req))
        return M.Empty()

    async def AssembleContext(self, req, ctx):
        r = await self._run(self.store.assemble_context, req.task_description, req.max_tokens,
                            [_tier(t) for t in req.memory_tiers])
        return from_dict(M.ContextResponse, r)

    # ------------------------------------------------------------- background
    def sample_telemetry(self):
        s = sysinfo.snapshot()
        ts = s["timestamp"]
        for k, v in (("cpu.usage", s["cpu_percent"]), ("memory.used_mb", s["memory_used_mb"]),
                     ("memory.total_mb", s["memory_total_mb"]), ("disk.used_gb", s["disk_used_gb"]),
                     ("disk.total_gb", s["disk_total_gb"]), ("gpu.utilization", s["gpu_utilization"])):
            self.store.update_metric(k, float(v), ts)

    async def background(self, stop: asyncio.Event):
        last_migration = time.time()
        while not stop.is_set():
            try:
                await self._run(self.sample_telemetry)
                if time.time() - last_migration >= MIGRATION_INTERVAL:
                    last_migration = time.time()
                    r = await self._run(self.store.migrate)
                    log.info("tier migration: %s", r)
            except Exception as e:  # pragma: no cover - defensive
                log.warning("memory background task failed: %s", e)
            try:
                await asyncio.wait_for(stop.wait(), TELEMETRY_INTERVAL)
            except asyncio.TimeoutError:
                pass


async def amain(args):
    svc = MemoryServiceImpl(args.working_db, args.longterm_db, args.knowledge_db)
    server = RpcServer(args.addr, {"aios.memory.MemoryService": svc})
    await server.start()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except NotImplementedError:
            pass
    await svc.background(stop)
    await server.stop()


def main(argv=None):
    mem = os.path.join(data_dir(), "memory")
    ap = argparse.ArgumentParser(description="aiOS memory service (aios.memory.MemoryService)")
    ap.add_argument("--addr", default=os.environ.get("AIOS_MEMORY_LISTEN", "0.0.0.0:50053"))
    ap.add_argument("--working-db", default=os.environ.get("AIOS_WORKING_DB", os.path.join(mem, "working.db")))
    ap.add_argument("--longterm-db", default=os.environ.get("AIOS_LONGTERM_DB", os.path.join(mem, "longterm.db")))
    ap.add_argument("--knowledge-db", default=os.environ.get("AIOS_KNOWLEDGE_DB", os.path.join(mem, "knowledge.db")))
    args = ap.parse_args(argv)
    setup_logging("aios-memory")
    asyncio.run(amain(args))


if __name__ == "__main__":
    main()

"""Orchestrator state: the native stores plus the async planner front-end.

Reference: `OrchestratorState` (`agent-core/src/main.rs:61-72`) held goal engine, planner, router,
aggregator, decision log, clients, health and cluster behind ONE `tokio::RwLock`, so a slow AI
decomposition inside SubmitGoal blocked every other RPC.  Here each native store is internally
synchronised (C++ mutexes, released GIL), so RPCs, the autonomy loop and the console run
concurrently; the only Python-side coordination is the set of tasks currently in flight.

The goal engine is the single source of truth for tasks (the reference kept a second copy in
the planner's `pending_tasks`, `task_planner.rs:105-110`, and the two could diverge).
"""
from __future__ import annotations

import logging
import os
import time
from typing import Dict, List, Optional, Set

from ..core import load as load_core
from ..utils.env import data_dir, env_flag
from .clients import ServiceClients

log = logging.getLogger("aios.orchestrator")
core = load_core()

LEVEL_ROUNDS = {"reactive": 1, "operational": 1, "tactical": 3, "strategic": 5}
LEVEL_TOKENS = {"reactive": 2048, "operational": 2048, "tactical": 8192, "strategic": 16384}
# token cap of the one decomposition call (task_planner.rs:163-218 asks for <= 1024)
PLAN_MAX_TOKENS = int(os.environ.get("AIOS_PLAN_MAX_TOKENS", "1024"))


class OrchestratorState:
    def __init__(self, data: Optional[str] = None, clients: Optional[ServiceClients] = None,
                 in_memory: bool = False):
        d = data or os.path.join(data_dir(), "data")
        if not in_memory:
            os.makedirs(d, exist_ok=True)
        self.goal_engine = core.GoalEngine(":memory:" if in_memory else os.path.join(d, "goals.db"))
        self.schedules = core.ScheduleStore(":memory:" if in_memory else os.path.join(d, "scheduler.db"))
        self.router = core.AgentRouter(15)
        self.cluster = core.ClusterManager(30)
        self.discovery = core.Discovery(30)
        self.decisions = core.DecisionLog(10000)
        self.results = core.ResultAggregator()
        self.events = core.EventBus()
        self.event_queue = None     # EventQueue (loops.py): producers publish through emit()
        self.clients = clients or ServiceClients(self.discovery)
        self.health = None          # HealthChecker (loops.py)
        self.inflight: Set[str] = set()
        self.started = time.time()
        self.node_id = os.environ.get("AIOS_NODE_ID", "local")
        self.cluster_enabled = env_flag("AIOS_CLUSTER_ENABLED")
        self.autonomy_level = os.environ.get("AIOS_AUTONOMY_LEVEL", "full")
        self.loaded_models: List[str] = []
        self.plan_latency_ms: List[float] = []   # goal -> plan latencies (for the console / bench)
        resumed = self.goal_engine.resume_in_progress()
        if resumed:
            log.info("resumed %d in-progress tasks after restart", resumed)

    # ------------------------------------------------------------------ events
    def emit(self, event_type: str, source: str, data: Optional[dict] = None, severity: str = "info") -> bool:
        """Publish a system event to the bus (event_bus.rs SystemEvent): the EventQueue matches it
        against the subscriptions and turns matches into goals.  Producers: service health
        transitions, lost agents, failed tasks, goal completion / failure, proactive triggers."""
        ev = {"id": f"ev-{time.time_ns():x}", "event_type": event_type, "source": source,
              "data": data or {}, "severity": severity, "timestamp": int(time.time())}
        if self.event_queue is None:
            self.events.publish(ev)  # recorded (recent events) even without a running queue
            return False
        return self.event_queue.publish(ev)

    def install_default_subscriptions(self):
        """Event -> goal rules on by default (AIOS_EVENT_SUBSCRIPTIONS=0 disables): a service that
        stops answering and an agent that stops heartbeating become recovery goals right away,
        instead of waiting for the proactive generator's next 60 s sweep."""
        if os.environ.get("AIOS_EVENT_SUBSCRIPTIONS", "1") in ("0", "false", "no"):
            return []
        return [
            self.events.subscribe("service_unhealthy", "critical",
                                  "Service {source} stopped responding. Diagnose the failure, restart it and "
                                  "verify it answers health checks.", 9),
            self.events.subscribe("agent_lost", "warning",
                                  "Agent {source} stopped sending heartbeats. Restart it, check its logs and "
                                  "re-queue its work.", 8),
        ]

    # ------------------------------------------------------------------ planning
    async def decompose(self, goal_id: str, description: str) -> List[dict]:
        """task_planner.rs:91-223: reactive/operational -> heuristic single task; tactical and
        strategic -> one LLM call (gateway, then runtime) asking for a 2-5 step JSON array with a
        linear depends_on chain, falling back to the keyword multi-step decomposition."""
        t0 = time.perf_counter()
        level = core.planner.classify(description)
        tasks: List[dict] = []
        if level in ("tactical", "strategic"):
            r = await self.clients.infer_any(core.planner.ai_decomposition_prompt(description),
                                             core.planner.DECOMPOSE_SYSTEM_PROMPT, PLAN_MAX_TOKENS, level="tactical",
                                             task_id=goal_id)
            if r is not None and r.success:
                tasks = core.planner.parse_ai_decomposition(r.text, goal_id, level)
                if tasks:
                    self.decisions.log("goal_decomposition", [t["description"] for t in tasks], "ai_decomposition",
                                       f"Goal {goal_id} decomposed into {len(tasks)} steps by {r.model_used}",
                                       level, r.model_used)
            if not tasks:
                log.info("AI decomposition unavailable for goal %s, falling back to heuristics", goal_id)
        if not tasks:
            tasks = core.planner.decompose(goal_id, description, level)
        self.plan_latency_ms.append((time.perf_counter() - t0) * 1000.0)
        del self.plan_latency_ms[:-1000]
        return tasks

    async def submit_goal(self, description: str, priority: int = 5, source: str = "user",
                          tags: Optional[list] = None, metadata_json: bytes = b"") -> dict:
        g = self.goal_engine.submit(description, priority or 5, source or "user", list(tags or []),
                                    metadata_json or b"")
        tasks = await self.decompose(g["id"], description)
        self.goal_engine.add_tasks(g["id"], tasks)
        log.info("goal %s decomposed into %d tasks", g["id"], len(tasks))
        return self.goal_engine.goal(g["id"])

    def preferred_provider(self, goal_id: str) -> str:
        import json

        meta = self.goal_engine.goal(goal_id).get("metadata_json", "")
        try:
            return (json.loads(meta) if meta else {}).get("preferred_provider", "")
        except ValueError:
            return ""

"""Async client for the Orchestrator service (reference `aios_agent/orchestrator_client.py`).

Same API surface (submit_goal, get_goal_status, cancel_goal, list_goals, register_agent,
heartbeat, list_agents, get_system_status, wait_for_goal) but speaking real protobuf on the
`aios.orchestrator.Orchestrator` methods -- the reference sent JSON bytes over a raw method path,
which the tonic server could not decode.
"""
from __future__ import annotations

import asyncio
import json
import os
import time
from typing import Any, Dict, List, Optional

from ..rpc.client import Stub, channel
from ..rpc.convert import to_dict
from ..rpc.schema import pb

TERMINAL = ("completed", "failed", "cancelled")


class OrchestratorClient:
    def __init__(self, address: Optional[str] = None, timeout: float = 30.0):
        self.address = (address or os.getenv("AIOS_ORCHESTRATOR_ADDR", "127.0.0.1:50051")).replace(
            "localhost", "127.0.0.1")
        self.timeout = timeout
        self._stub = None

    @property
    def stub(self) -> Stub:
        # grpc.aio channels bind to the running event loop: create lazily on first use, so a client
        # can be constructed outside a loop (agents are built before asyncio.run)
        if self._stub is None:
            self._stub = Stub(channel(self.address), "aios.orchestrator.Orchestrator", timeout=self.timeout)
        return self._stub

    async def submit_goal(self, description: str, priority: int = 5, source: str = "agent",
                          tags: Optional[List[str]] = None, metadata: Optional[Dict[str, Any]] = None) -> str:
        r = await self.stub.SubmitGoal(pb.orchestrator.SubmitGoalRequest(
            description=description, priority=priority, source=source, tags=tags or [],
            metadata_json=json.dumps(metadata).encode() if metadata else b""))
        return r.id

    async def get_goal_status(self, goal_id: str) -> Dict[str, Any]:
        r = await self.stub.GetGoalStatus(pb.common.GoalId(id=goal_id))
        return to_dict(r)

    async def cancel_goal(self, goal_id: str) -> bool:
        return (await self.stub.CancelGoal(pb.common.GoalId(id=goal_id))).success

    async def list_goals(self, status: str = "", limit: int = 50, offset: int = 0) -> Dict[str, Any]:
        r = await self.stub.ListGoals(pb.orchestrator.ListGoalsRequest(status_filter=status, limit=limit,
                                                                       offset=offset))
        return {"goals": [to_dict(g) for g in r.goals], "total": r.total}

    async def register_agent(self, agent_id: str, agent_type: str, capabilities: List[str],
                             tool_namespaces: Optional[List[str]] = None) -> bool:
        r = await self.stub.RegisterAgent(pb.common.AgentRegistration(
            agent_id=agent_id, agent_type=agent_type, capabilities=capabilities,
            tool_namespaces=tool_namespaces or sorted({c.split(".")[0] for c in capabilities if "." in c}),
            status="idle", registered_at=int(time.time())))
        return r.success

    async def heartbeat(self, agent_id: str, status: str = "idle", current_task_id: str = "") -> bool:
        return (await self.stub.Heartbeat(pb.orchestrator.HeartbeatRequest(
            agent_id=agent_id, status=status, current_task_id=current_task_id))).success

    async def list_agents(self) -> List[Dict[str, Any]]:
        return [to_dict(a) for a in (await self.stub.ListAgents(pb.common.Empty())).agents]

    async def get_system_status(self) -> Dict[str, Any]:
        return to_dict(await self.stub.GetSystemStatus(pb.common.Empty()))

    async def wait_for_goal(self, goal_id: str, timeout: float = 300.0, poll_interval: float = 1.0) -> Dict[str, Any]:
        deadline = time.time() + timeout
        while True:
            st = await self.get_goal_status(goal_id)
            if st["goal"].get("status") in TERMINAL:
                return st
            if time.time() >= deadline:
                raise asyncio.TimeoutError(f"goal {goal_id} not finished after {timeout}s")
            await asyncio.sleep(poll_interval)

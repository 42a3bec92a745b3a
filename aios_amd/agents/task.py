"""TaskAgent: plans a task as a DAG of steps, runs ready steps concurrently, delegates sub-steps
to other agents as sub-goals (reference `aios_agent/agents/task.py:24-398`: ≤20 steps, 120 s per
step, deadlock detection, memory search for past plans, delegation via submit_goal +
wait_for_goal)."""
from __future__ import annotations

import asyncio
import json
from typing import Any, Dict, List

from .base import BaseAgent, IntelligenceLevel, main_for
from .orchestrator_client import OrchestratorClient

MAX_PLAN_STEPS = 20
SUBTASK_TIMEOUT_S = 120.0


def validate_plan(steps: Any) -> List[Dict[str, Any]]:
    """Normalise an LLM plan: ids unique, deps known, ≤ MAX_PLAN_STEPS, no cycles."""
    if not isinstance(steps, list):
        return []
    out, ids = [], set()
    for i, s in enumerate(steps[:MAX_PLAN_STEPS]):
        if not isinstance(s, dict):
            continue
        sid = str(s.get("id") or f"s{i + 1}")
        if sid in ids:
            sid = f"{sid}_{i}"
        ids.add(sid)
        out.append({"id": sid, "description": str(s.get("description", "")), "agent_type": s.get("agent_type", ""),
                    "tool": s.get("tool", ""), "input": s.get("input") or {}, "depends_on": s.get("depends_on") or [],
                    "can_fail": bool(s.get("can_fail", False))})
    for s in out:
        s["depends_on"] = [d for d in map(str, s["depends_on"]) if d in ids and d != s["id"]]
    # drop edges that close a cycle (Kahn order)
    done, order = set(), []
    remaining = {s["id"]: s for s in out}
    while remaining:
        ready = [sid for sid, s in remaining.items() if all(d in done for d in s["depends_on"])]
        if not ready:  # cycle: break it by dropping the remaining deps of the first step
            sid = next(iter(remaining))
            remaining[sid]["depends_on"] = [d for d in remaining[sid]["depends_on"] if d in done]
            continue
        for sid in ready:
            done.add(sid)
            order.append(remaining.pop(sid))
    return order


class TaskAgent(BaseAgent):
    AGENT_TYPE = "task"
    CAPABILITIES = ("task.plan", "task.execute", "task.delegate", "task.pipeline", "task.decompose",
                    "task.coordinate")

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.client = OrchestratorClient(self.config.orchestrator_addr)

    async def handle_task(self, task: Dict[str, Any]) -> Dict[str, Any]:
        given = task.get("input", {}).get("plan")
        plan = validate_plan(given) if given else await self.create_plan(task)
        if not plan:
            return {"success": False, "error": "could not produce a plan"}
        return await self.execute_plan(plan)

    async def create_plan(self, task: Dict[str, Any]) -> List[Dict[str, Any]]:
        past = []
        try:
            past = await self.semantic_search(task.get("description", ""), ["procedures"], 3, 0.3)
        except Exception:
            pass
        hint = ("\nSimilar past procedures:\n" + "\n".join(p["content"] for p in past)) if past else ""
        steps = await self.think_json(
            f"Plan this task as a DAG of at most {MAX_PLAN_STEPS} steps.\nTask: {task.get('description')}{hint}\n"
            "Each step: {\"id\": \"s1\", \"description\": \"...\", \"agent_type\": \"system|network|security|"
            "package|storage|monitoring|web|creator|\", \"tool\": \"namespace.action or empty\", \"input\": {}, "
            "\"depends_on\": [], \"can_fail\": false}. JSON: {\"steps\": [...]}", IntelligenceLevel.TACTICAL)
        if isinstance(steps, dict):
            steps = steps.get("steps")
        return validate_plan(steps)

    async def execute_plan(self, plan: List[Dict[str, Any]]) -> Dict[str, Any]:
        results: Dict[str, Dict[str, Any]] = {}
        pending = {s["id"]: s for s in plan}
        failed_hard = False
        while pending and not failed_hard:
            ready = [s for s in pending.values() if all(d in results for d in s["depends_on"])]
            if not ready:
                return {"success": False, "error": "deadlock: unsatisfiable dependencies",
                        "pending": list(pending), "results": results}
            outs = await asyncio.gather(*(self.run_step(s) for s in ready))
            for s, r in zip(ready, outs):
                results[s["id"]] = r
                pending.pop(s["id"])
                if not r.get("success") and not s["can_fail"]:
                    failed_hard = True
        ok = not failed_hard and all(r.get("success") or s["can_fail"] for s in plan for r in [results.get(s["id"], {})])
        try:
            await self.push_event("task.plan_executed", {"steps": len(plan), "success": ok})
        except Exception:
            pass
        return {"success": ok, "steps": len(plan), "results": results,
                **({} if ok else {"error": "a required step failed"})}

    async def run_step(self, step: Dict[str, Any]) -> Dict[str, Any]:
        try:
            if step["tool"]:
                return await asyncio.wait_for(self.call_tool(step["tool"], step["input"]), SUBTASK_TIMEOUT_S)
            if step["agent_type"] and step["agent_type"] != self.AGENT_TYPE:
                return await self.delegate(step)
            return {"success": True, "note": "no-op step", "description": step["description"]}
        except asyncio.TimeoutError:
            return {"success": False, "error": f"step {step['id']} timed out after {SUBTASK_TIMEOUT_S}s"}

    async def delegate(self, step: Dict[str, Any]) -> Dict[str, Any]:
        gid = await self.client.submit_goal(step["description"], priority=4, source=f"task-agent:{self.agent_id}",
                                            metadata={"delegated_from": self.current_task_id or ""})
        try:
            st = await self.client.wait_for_goal(gid, SUBTASK_TIMEOUT_S)
        except asyncio.TimeoutError:
            return {"success": False, "error": f"sub-goal {gid} timed out", "goal_id": gid}
        status = st["goal"]["status"]
        return {"success": status == "completed", "goal_id": gid, "status": status}


if __name__ == "__main__":
    main_for(TaskAgent)

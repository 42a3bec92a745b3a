"""The autonomy loop: goals -> tasks -> (agent | cluster node | heuristic | AI reasoning) -> results.

Reference: `agent-core/src/autonomy.rs` -- 500 ms tick (`:22-64`), per-tick decomposition of
pending goals, up to 3 unblocked tasks (`:376`), routing order agent -> cluster node ->
heuristic tool calls -> AI work (`:396-560`), multi-round observe->think->act reasoning with
round / token limits by tier (`:100-224`, `:597-606`), JSON self-correction (`:290-328`),
`{"done": true}` completion, result recording with the awaiting_input / 3-strike rule
(`:2380-2583`) and housekeeping (dead-agent requeue, goal completion; `:695-733`).

Differences, on purpose:
* reasoning loops are launched as background tasks (≤3 concurrent) instead of being awaited
  inside the tick, so a 30 s strategic task never stalls goal pickup for everything else;
* every ready task is routed (the reference routed only the first and sent the rest to the AI
  path unconditionally).
All text parsing (think-tag stripping, JSON extraction, tool-call fallbacks, heuristics,
summaries) runs in the native core (`aios_amd/native/llm_parse.cpp`).
"""
from __future__ import annotations

import asyncio
import json
import logging
import time
from dataclasses import dataclass, field
from typing import List, Optional

from ..rpc.schema import pb
from .clients import InferResult
from .remote import RemoteExecutor, find_node, tools_address_of
from .state import LEVEL_ROUNDS, LEVEL_TOKENS, OrchestratorState, core

log = logging.getLogger("aios.autonomy")

TICK_S = 0.5
MAX_PARALLEL_AI = 3
SYSTEM_JSON_RULE = ("\n\nYou MUST always respond with ONLY a valid JSON object. Never output natural language, "
                    "markdown, or explanations outside of JSON. Your response must contain a \"tool_calls\" array "
                    "with at least one tool to execute.")
FORMAT_RULES = (
    "IMPORTANT — Self-Evolution:\nIf the task requires a tool you do NOT have, create one using plugin.create.\n"
    "The code must define: def main(input_data: dict) -> dict\n\n"
    "You MUST respond with ONLY a valid JSON object. No prose, no markdown, no explanation outside JSON.\n\n"
    "FORMAT — Execute tools:\n"
    "{\"reasoning\": \"brief explanation\", \"tool_calls\": [{\"tool\": \"monitor.cpu\", \"input\": {}}], "
    "\"result\": \"summary of what will be done\"}\n\n"
    "FORMAT — Need user input:\n{\"needs_clarification\": true, \"questions\": [\"What specific thing?\"]}\n\n"
    "FORMAT — Create new tool then use it:\n"
    "{\"reasoning\": \"Need custom tool\", \"tool_calls\": [{\"tool\": \"plugin.create\", \"input\": {\"name\": "
    "\"my_tool\", \"description\": \"Does X\", \"code\": \"def main(input_data):\\n    return {'result': 'done'}\", "
    "\"capabilities\": [], \"dependencies\": []}}, {\"tool\": \"plugin.my_tool\", \"input\": {}}], "
    "\"result\": \"Created and executed tool\"}\n\n"
    "RULES:\n1. ALWAYS include tool_calls array with at least one tool call — never just describe a plan\n"
    "2. Output ONLY valid JSON — no text before or after\n"
    "3. Tool names use namespace.action format (e.g. monitor.cpu, fs.read, net.ping)\n"
    "4. If unsure which tool, use the closest match from the catalog above")


@dataclass
class AiResult:
    success: bool
    text: str
    tool_calls: List[dict] = field(default_factory=list)
    model_used: str = "none"
    tokens_used: int = 0


class AutonomyLoop:
    def __init__(self, state: OrchestratorState, tick_s: float = TICK_S):
        self.st = state
        self.tick_s = tick_s
        self.sem = asyncio.Semaphore(MAX_PARALLEL_AI)
        self.remote = RemoteExecutor()
        self._lost: set = set()  # agents already reported lost (agent_lost events fire once)
        self.bg: set = set()
        self.ticks = 0

    # ------------------------------------------------------------------ loop
    async def run(self, stop: asyncio.Event):
        log.info("autonomy loop started (tick=%d ms)", int(self.tick_s * 1000))
        while not stop.is_set():
            try:
                await self.tick()
            except Exception:
                log.exception("autonomy tick error")
            try:
                await asyncio.wait_for(stop.wait(), self.tick_s)
            except asyncio.TimeoutError:
                pass
        for t in list(self.bg):
            t.cancel()
        log.info("autonomy loop stopped")

    async def tick(self):
        self.ticks += 1
        ge = self.st.goal_engine
        if ge.counts()["active_goals"] == 0:
            return
        # 1. decompose pending goals without tasks; advance the rest
        pending, _ = ge.list("pending", 10, 0)
        for g in pending:
            if not ge.tasks_for_goal(g["id"]):
                tasks = await self.st.decompose(g["id"], g["description"])
                ge.add_tasks(g["id"], tasks)
            ge.set_goal_status(g["id"], "in_progress")
        # 2. route ready tasks
        free = MAX_PARALLEL_AI - len(self.bg)
        ready = [t for t in ge.next_tasks(MAX_PARALLEL_AI + len(self.st.inflight)) if t["id"] not in self.st.inflight]
        for task in ready[:max(free, 0) or 1]:
            await self.dispatch(task)
        # 3. housekeeping
        self.housekeeping()

    def _mark(self, task: dict, status: str, **extra):
        upd = {"id": task["id"], "status": status}
        upd.update(extra)
        self.st.goal_engine.update_task(upd)

    async def dispatch(self, task: dict):
        st, tid, gid = self.st, task["id"], task["goal_id"]
        level = task.get("intelligence_level") or "operational"
        # agent route
        agent = st.router.route(task)
        if agent:
            st.router.assign(agent, tid)
            self._mark(task, "assigned", assigned_agent=agent, started_at=int(time.time()))
            st.decisions.log("task_routing", [agent], "agent_dispatch",
                             f"Task {tid} dispatched to agent {agent} (level: {level})", level, "heuristic")
            return
        # cluster route
        if st.cluster_enabled:
            node = st.cluster.route_least_loaded()
            if node and node != st.node_id and await self._remote(task, node):
                return
        self._mark(task, "in_progress", started_at=int(time.time()))
        st.inflight.add(tid)
        # heuristic execution (reactive tier, no LLM)
        calls = core.llm.heuristic_calls(task)
        if calls:
            st.decisions.log("task_routing", [tid], "heuristic_execution",
                             f"Task '{task['description']}' executed via heuristic (no AI inference needed)",
                             level, "heuristic")
            self._spawn(self._heuristic(task, calls))
            return
        self._spawn(self._reason(task))

    def _spawn(self, coro):
        t = asyncio.ensure_future(coro)
        self.bg.add(t)
        t.add_done_callback(self.bg.discard)

    async def _remote(self, task: dict, node_id: str) -> bool:
        n = find_node(self.st.cluster, node_id)
        if not n:
            return False
        try:
            rid = await self.remote.submit_remote_goal(n["address"], task["description"], 5, f"cluster:{task['id']}")
        except Exception as e:
            log.warning("remote dispatch of %s to %s failed: %s", task["id"], node_id, e)
            return False
        self._mark(task, "completed", completed_at=int(time.time()),
                   output_json=json.dumps({"remote_node": node_id, "remote_goal_id": rid}))
        self.st.decisions.log("task_routing", [node_id], "cluster_dispatch",
                              f"Task {task['id']} routed to remote cluster node", task.get("intelligence_level", ""),
                              "cluster")
        return True

    # ------------------------------------------------------------------ execution paths
    async def _heuristic(self, task: dict, calls: List[dict]):
        try:
            res = AiResult(True, json.dumps({"reasoning": "Heuristic execution", "tool_calls": calls,
                                             "result": "Executing directly"}), calls, "heuristic", 0)
            results, ok = await self.run_tools(task["id"], calls)
            self.record(task, res, results, ok)
        finally:
            self.st.inflight.discard(task["id"])
            self.housekeeping()

    async def _reason(self, task: dict):
        try:
            async with self.sem:
                res, results, ok = await self.reasoning_loop(task)
            self.record(task, res, results, ok)
        except Exception as e:
            log.exception("reasoning for task %s crashed", task["id"])
            self.record(task, AiResult(False, f"internal error: {e}"), [], False)
        finally:
            self.st.inflight.discard(task["id"])
            self.housekeeping()

    async def run_tools(self, task_id: str, calls: List[dict]):
        results, ok = [], True
        for c in calls:
            node = c.get("node") or ""
            if node and node != self.st.node_id:
                r = await self.run_remote_tool(task_id, c, node)
            else:
                r = await self.st.clients.execute_tool(c["tool"], c.get("input", {}), task_id)
            ok = ok and r["success"]
            results.append(r)
        return results, ok

    async def run_remote_tool(self, task_id: str, call: dict, node_id: str) -> dict:
        """A tool call addressed to another cluster node runs on that node's tool service."""
        tool = call["tool"]
        n = find_node(self.st.cluster, node_id)
        if n is None:
            return {"tool": tool, "success": False, "node": node_id,
                    "error": f"Remote node '{node_id}' is not registered or not healthy"}
        data = json.dumps(call.get("input") or {}).encode()
        try:
            ok, out, err = await self.remote.execute_remote_tool(tools_address_of(n), tool, "autonomy-loop",
                                                                 task_id, data)
        except Exception as e:  # noqa: BLE001 - unreachable node: a failed tool call, not a crash
            return {"tool": tool, "success": False, "node": node_id, "error": f"Remote tool execution failed: {e}"}
        self.st.decisions.log("tool_routing", [node_id], "remote_tool", f"Tool {tool} for task {task_id} executed on "
                              f"cluster node {node_id}", "", "cluster")
        if not ok:
            return {"tool": tool, "success": False, "node": node_id, "error": f"Tool '{tool}' failed on {node_id}: {err}"}
        try:
            parsed = json.loads(out) if out else {}
        except ValueError:
            parsed = out.decode("utf-8", "replace")
        return {"tool": tool, "success": True, "node": node_id, "output": parsed}

    async def ai_call(self, task: dict, prompt_body: str, provider: str) -> AiResult:
        """execute_ai_task (autonomy.rs:823-983): system prompt + memory context + conversation +
        live tool catalog + format rules; gateway with the goal's preferred provider, runtime
        as a fallback."""
        st = self.st
        level = task.get("intelligence_level") or "operational"
        system = core.build_system_prompt(task["description"], level, [], [], 4096) + SYSTEM_JSON_RULE
        chunks = await st.clients.memory_context(task["description"], 2048)
        if chunks:
            system += "\n\nRelevant memory context:\n" + "".join(f"- [{c['source']}] {c['content']}\n" for c in chunks)
        prompt = f"Task: {prompt_body}\n\n"
        msgs = [m for m in st.goal_engine.messages(task["goal_id"], 50) if m["sender"] in ("user", "ai")]
        if msgs:
            prompt += "Previous conversation:\n" + "".join(
                f"{'[User]' if m['sender'] == 'user' else '[AI]'}: {m['content']}\n" for m in msgs)
            prompt += "\nExecute the task using the provided context.\n\n"
        prompt += await st.clients.tool_catalog()
        prompt += FORMAT_RULES
        r: Optional[InferResult] = await st.clients.infer_any(prompt, system, 4096 if provider else 2048, level,
                                                              provider=provider, task_id=task["id"])
        if r is None:
            return AiResult(False, "All AI backends are currently unavailable. The task could not be executed.")
        return AiResult(True, r.text, core.llm.parse_tool_calls(r.text), r.model_used, r.tokens_used)

    @staticmethod
    def round_prompt(task: dict, rnd: int, turns: List[List[dict]]) -> str:
        if rnd == 0 or not turns:
            return task["description"]
        p = f"Task: {task['description']}\n\nPrevious tool results:\n"
        for tr_list in turns:
            for tr in tr_list:
                if tr.get("success"):
                    s = json.dumps(tr.get("output"))
                    p += f"- {tr['tool']}: {s[:1000] + '...(truncated)' if len(s) > 1000 else s}\n"
                else:
                    p += f"- {tr['tool']}: FAILED — {tr.get('error', 'unknown error')}\n"
        return p + ("\nBased on the results above, decide what to do next:\n"
                    "- If more information is needed, call additional tools.\n"
                    "- If the task is complete, respond with: {\"done\": true, \"summary\": \"brief summary of what "
                    "was accomplished\"}\n- Respond with ONLY valid JSON.\n")

    async def reasoning_loop(self, task: dict):
        level = task.get("intelligence_level") or "operational"
        max_rounds, max_tokens = LEVEL_ROUNDS.get(level, 1), LEVEL_TOKENS.get(level, 2048)
        provider = self.st.preferred_provider(task["goal_id"]) or ""
        turns: List[List[dict]] = []
        all_results: List[dict] = []
        all_ok, used = True, 0
        executed: List[dict] = []
        final: Optional[AiResult] = None
        for rnd in range(max_rounds):
            res = await self.ai_call(task, self.round_prompt(task, rnd, turns), provider)
            used += res.tokens_used
            if used > max_tokens or core.llm.is_done_signal(res.text):
                # the work was done by the tool calls of earlier rounds; a bare {"done": true}
                # must not push the task to awaiting_input (reference defect, autonomy.rs:2433)
                if not res.tool_calls and executed:
                    res.tool_calls = executed
                final = res
                break
            if not res.tool_calls and res.text.strip() and res.success:
                corr = await self.ai_call(task, (
                    "Your previous response was not valid JSON for tool execution. Your response was: "
                    f"{res.text[:300]}\n\nYou MUST respond with ONLY a valid JSON object in this exact format:\n"
                    "{\"tool_calls\": [{\"tool\": \"namespace.action\", \"input\": {}}]}\n\nOr if the task is "
                    "complete:\n{\"done\": true, \"summary\": \"what was accomplished\"}\n\n"
                    f"Original task: {task['description']}"), provider)
                if corr.tool_calls or core.llm.is_done_signal(corr.text):
                    used += corr.tokens_used
                    res = corr
            if not res.tool_calls:
                final = res
                break
            results, ok = await self.run_tools(task["id"], res.tool_calls)
            executed += res.tool_calls
            all_ok = all_ok and ok
            all_results += results
            turns.append(results)
            final = res
            if max_rounds == 1 or not all_ok:
                break
        if final is None:
            final = AiResult(False, "Reasoning loop completed without producing a result", tokens_used=used)
        final.tokens_used = used
        return final, all_results, all_ok

    # ------------------------------------------------------------------ recording
    def record(self, task: dict, res: AiResult, results: List[dict], all_ok: bool):
        """record_ai_result (autonomy.rs:2380-2583)."""
        st, tid, gid = self.st, task["id"], task["goal_id"]
        ge = st.goal_engine
        level = task.get("intelligence_level") or "operational"
        now = int(time.time())

        def fail(msg: str, output=""):
            ge.update_task({"id": tid, "status": "failed", "error": msg, "completed_at": now, "output_json": output})
            ge.add_message(gid, "system", f"Task failed: {msg}")
            st.results.record(gid, {"task_id": tid, "success": False, "error": msg, "tokens_used": res.tokens_used,
                                    "model_used": res.model_used})

        if not res.success and not res.tool_calls:
            fail(res.text or "AI inference failed — all backends unavailable")
            return
        if not res.tool_calls:
            ai_msgs = sum(1 for m in ge.messages(gid, 1000) if m["sender"] == "ai")
            if ai_msgs >= 3:
                fail("AI was unable to produce executable tool calls after multiple attempts. "
                     "The model may not support the required JSON output format.")
                return
            q = core.llm.parse_clarification(res.text)
            parsed = core.llm.extract_json(res.text)
            display = q or (core.llm.json_to_readable(parsed) if parsed is not None else res.text.strip())
            ge.add_message(gid, "ai", display or "I received this task but wasn't able to determine what actions "
                                                "to take. Please provide more specific instructions.")
            ge.update_task({"id": tid, "status": "awaiting_input"})
            return
        if not all_ok:
            err = "; ".join(r.get("error", "") for r in results if not r.get("success"))
            fail(err, json.dumps(results))
            st.decisions.log("ai_execution", [tid], "failed",
                             f"Task '{task['description']}' failed during tool execution", level, "ai")
            return
        output = json.dumps({"ai_response": res.text, "tool_results": results, "model_used": res.model_used})
        summary = self.completion_summary(res.text, results)
        if summary:
            ge.add_message(gid, "ai", summary)
        ge.add_message(gid, "system", f"Task completed: {task['description']}")
        ge.update_task({"id": tid, "status": "completed", "completed_at": now, "output_json": output})
        st.results.record(gid, {"task_id": tid, "success": True, "tokens_used": res.tokens_used,
                                "model_used": res.model_used, "output_json": output})
        st.decisions.log("ai_execution", [tid], "executed",
                         f"Executed {level} task '{task['description']}' via "
                         f"{'heuristic' if res.model_used == 'heuristic' else 'AI inference'}", level,
                         "heuristic" if res.model_used == "heuristic" else "ai")

    @staticmethod
    def completion_summary(text: str, results: List[dict]) -> str:
        parts = []
        parsed = core.llm.extract_json(text)
        if isinstance(parsed, dict):
            for k in ("reasoning", "result"):
                if isinstance(parsed.get(k), str) and parsed[k] and parsed[k] != "Heuristic execution":
                    parts.append(parsed[k])
        for tr in results:
            if tr.get("success"):
                parts.append(f"**{tr['tool']}**: {core.llm.summarize_tool_output(tr['tool'], tr.get('output'))}")
            else:
                parts.append(f"**{tr['tool']}** failed: {tr.get('error', 'unknown error')}")
        return "\n\n".join(parts)

    # ------------------------------------------------------------------ housekeeping
    def housekeeping(self):
        st = self.st
        ge = st.goal_engine
        dead_now = set()
        for dead in st.router.dead_agents():
            dead_now.add(dead["agent_id"])
            if dead["agent_id"] not in self._lost:
                st.emit("agent_lost", dead["agent_id"], {"task_id": dead["task_id"]}, "warning")
            if dead["task_id"]:
                log.warning("agent %s is dead with task %s assigned — re-queuing", dead["agent_id"], dead["task_id"])
                st.router.task_completed(dead["agent_id"], False)
                ge.update_task({"id": dead["task_id"], "status": "pending", "assigned_agent": ""})
        self._lost = dead_now
        goals, _ = ge.list("in_progress", 100, 0)
        for g in goals:
            ns = ge.check_completion(g["id"])
            if ns:
                st.emit(f"goal_{ns}", g["id"], {"goal_id": g["id"], "description": g["description"]},
                        "warning" if ns == "failed" else "info")
            if ns == "completed":
                log.info("goal %s completed", g["id"])
                st.decisions.log("goal_completion", [g["id"]], "completed",
                                 f"All tasks for goal '{g['description']}' completed successfully", "reactive",
                                 "heuristic")
            elif ns == "failed":
                log.info("goal %s failed", g["id"])

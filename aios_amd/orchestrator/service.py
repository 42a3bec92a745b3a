"""`aios.orchestrator.Orchestrator` -- the 19 RPCs (reference `agent-core/src/main.rs:142-586`).

Changes from the reference, on purpose:
* RequestCapability goes through policy + the tool service's `sec.grant` (the reference
  auto-granted everything without recording it, `main.rs:385-411`); critical capabilities need
  AIOS_ALLOW_CRITICAL_GRANTS=true;
* Create/List/DeleteSchedule are wired to the persisted cron store (stubs in the reference,
  `main.rs:426-468`);
* GetGoalStatus reports the real phase instead of the constant "executing".
"""
from __future__ import annotations

import json
import logging
import time

import grpc

from ..rpc.convert import from_dict, to_dict
from ..rpc.schema import pb
from ..utils import sysinfo
from ..utils.env import env_flag
from .state import OrchestratorState

log = logging.getLogger("aios.orchestrator")
C, O = pb.common, pb.orchestrator
CRITICAL_CAPS = {"self_update", "sec_manage", "firewall_manage", "pkg_manage", "process_manage", "fs_delete"}


def goal_pb(g: dict):
    return from_dict(C.Goal, g)


def task_pb(t: dict):
    return from_dict(C.Task, t)


class OrchestratorService:
    def __init__(self, state: OrchestratorState):
        self.st = state

    # ------------------------------------------------------------------ goals
    async def SubmitGoal(self, req, ctx):
        log.info("received goal: %s", req.description)
        if not req.description.strip():
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, "empty goal description")
        g = await self.st.submit_goal(req.description, req.priority, req.source, list(req.tags), req.metadata_json)
        return C.GoalId(id=g["id"])

    async def GetGoalStatus(self, req, ctx):
        ge = self.st.goal_engine
        g = ge.goal(req.id)
        if not g:
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"Goal not found: {req.id}")
        return O.GoalStatusResponse(goal=goal_pb(g), tasks=[task_pb(t) for t in ge.tasks_for_goal(req.id)],
                                    current_phase=ge.phase(req.id), progress_percent=ge.progress(req.id))

    async def CancelGoal(self, req, ctx):
        if not self.st.goal_engine.goal(req.id):
            await ctx.abort(grpc.StatusCode.NOT_FOUND, f"Goal not found: {req.id}")
        ok = self.st.goal_engine.cancel(req.id)
        return C.Status(success=ok, message=f"Goal {req.id} " + ("cancelled" if ok else "already finished"))

    async def ListGoals(self, req, ctx):
        goals, total = self.st.goal_engine.list(req.status_filter, req.limit or 50, req.offset)
        return O.GoalListResponse(goals=[goal_pb(g) for g in goals], total=total)

    # ------------------------------------------------------------------ agents
    async def RegisterAgent(self, req, ctx):
        log.info("agent registering: %s (type: %s)", req.agent_id, req.agent_type)
        self.st.router.register(to_dict(req))
        return C.Status(success=True, message="Agent registered")

    async def UnregisterAgent(self, req, ctx):
        ok = self.st.router.unregister(req.id)
        return C.Status(success=ok, message=f"Agent {req.id} " + ("unregistered" if ok else "not registered"))

    async def Heartbeat(self, req, ctx):
        ok = self.st.router.heartbeat(req.agent_id, req.status, "")
        return C.Status(success=ok, message="OK" if ok else "unknown agent; re-register")

    async def ListAgents(self, req, ctx):
        return O.AgentListResponse(agents=[from_dict(C.AgentRegistration, a) for a in self.st.router.list()])

    async def GetAssignedTask(self, req, ctx):
        """main.rs:299-317; an empty Task means "nothing yet, keep polling".  Handing the task
        out moves it assigned -> in_progress."""
        ge = self.st.goal_engine
        goals, _ = ge.list("in_progress", 1000, 0)
        for g in goals:
            for t in ge.tasks_for_goal(g["id"]):
                if t["assigned_agent"] == req.id and t["status"] in ("assigned", "in_progress"):
                    if t["status"] == "assigned":
                        ge.update_task({"id": t["id"], "status": "in_progress"})
                        t["status"] = "in_progress"
                    return task_pb(t)
        return C.Task()

    async def ReportTaskResult(self, req, ctx):
        st = self.st
        t = st.goal_engine.task(req.task_id)
        if not t:
            log.warning("agent reported result for unknown task %s", req.task_id)
            return C.Status(success=False, message=f"Task {req.task_id} not found")
        gid = t["goal_id"]
        if t.get("assigned_agent"):
            st.router.task_completed(t["assigned_agent"], req.success)
        now = int(time.time())
        if req.success:
            st.goal_engine.update_task({"id": req.task_id, "status": "completed", "completed_at": now,
                                        "output_json": req.output_json.decode("utf-8", "replace")})
            st.goal_engine.add_message(gid, "system", f"Task {req.task_id} completed by agent")
        else:
            st.goal_engine.update_task({"id": req.task_id, "status": "failed", "completed_at": now,
                                        "error": req.error})
            st.goal_engine.add_message(gid, "system", f"Task {req.task_id} failed: {req.error}")
            st.emit("task_failed", t.get("assigned_agent") or "agent",
                    {"task_id": req.task_id, "goal_id": gid, "error": req.error}, "warning")
        st.results.record(gid, to_dict(req))
        ns = st.goal_engine.check_completion(gid)
        if ns:
            st.emit(f"goal_{ns}", gid, {"goal_id": gid}, "warning" if ns == "failed" else "info")
        return C.Status(success=True, message=f"Result recorded for task {req.task_id}")

    # ------------------------------------------------------------------ capabilities
    async def RequestCapability(self, req, ctx):
        caps = [c.replace(".", "_") for c in req.capabilities]
        crit = sorted(set(caps) & CRITICAL_CAPS)
        hours = req.duration_hours if req.duration_hours > 0 else 24
        if crit and not env_flag("AIOS_ALLOW_CRITICAL_GRANTS"):
            self.st.decisions.log("capability_request", list(req.capabilities), "denied",
                                  f"{req.agent_id} asked for critical {crit}: {req.reason}", "reactive", "policy")
            return O.CapabilityResponse(granted=False, denial_reason=f"critical capabilities need operator "
                                        f"approval: {', '.join(crit)}")
        r = await self.st.clients.execute_tool("sec.grant", {"agent_id": req.agent_id, "capabilities": caps,
                                                             "reason": req.reason, "duration_hours": hours},
                                               task_id="", agent="autonomy-loop")
        if not r["success"]:
            return O.CapabilityResponse(granted=False, denial_reason=r.get("error", "grant failed"))
        exp = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime(time.time() + hours * 3600))
        self.st.decisions.log("capability_request", list(req.capabilities), "granted",
                              f"{req.agent_id}: {req.reason}", "reactive", "policy")
        return O.CapabilityResponse(granted=True, capabilities=list(req.capabilities), expires_at=exp)

    async def RevokeCapability(self, req, ctx):
        r = await self.st.clients.execute_tool("sec.revoke", {
            "agent_id": req.agent_id, "capabilities": [c.replace(".", "_") for c in req.capabilities],
            "revoke_all": req.revoke_all}, task_id="", agent="autonomy-loop")
        return C.Status(success=r["success"], message=r.get("error", "") or f"Capabilities revoked from {req.agent_id}")

    # ------------------------------------------------------------------ schedules
    async def CreateSchedule(self, req, ctx):
        try:
            sid = self.st.schedules.create(req.cron_expr, req.goal_template, req.priority or 5)
        except Exception as e:
            await ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        return O.ScheduleResponse(schedule_id=sid, success=True)

    async def ListSchedules(self, req, ctx):
        return O.ScheduleListResponse(schedules=[from_dict(O.ScheduleEntry, e) for e in self.st.schedules.list()])

    async def DeleteSchedule(self, req, ctx):
        ok = self.st.schedules.remove(req.schedule_id)
        return C.Status(success=ok, message=f"Schedule {req.schedule_id} " + ("deleted" if ok else "not found"))

    # ------------------------------------------------------------------ cluster
    async def RegisterNode(self, req, ctx):
        self.st.cluster.register_node(to_dict(req))
        return C.Status(success=True, message=f"Node {req.node_id} registered")

    async def NodeHeartbeat(self, req, ctx):
        ok = self.st.cluster.heartbeat(req.node_id, req.cpu_usage, req.memory_usage, req.active_tasks)
        return C.Status(success=ok, message="OK" if ok else "unknown node; re-register")

    async def ListNodes(self, req, ctx):
        return O.NodeListResponse(nodes=[from_dict(O.NodeInfo, n) for n in self.st.cluster.list(req.include_dead)])

    # ------------------------------------------------------------------ status
    async def GetSystemStatus(self, req, ctx):
        c = self.st.goal_engine.counts()
        used, total = sysinfo.memory_mb()
        models = list(self.st.loaded_models)
        try:
            ml = await self.st.clients.runtime.ListModels(C.Empty(), timeout=2)
            models = [m.model_name for m in ml.models if m.status == "ready"]
            self.st.loaded_models = models
        except grpc.aio.AioRpcError:
            pass
        return O.SystemStatusResponse(active_goals=c["active_goals"], pending_tasks=c["pending_tasks"],
                                      active_agents=self.st.router.healthy_count(), loaded_models=models,
                                      cpu_percent=sysinfo.cpu_percent(), memory_used_mb=used, memory_total_mb=total,
                                      autonomy_level=self.st.autonomy_level,
                                      uptime_seconds=int(time.time() - self.st.started))

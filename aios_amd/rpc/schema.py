"""The aiOS gRPC contract: 7 packages, 6 services, 63 RPCs.

Wire compatibility with the reference (`agent-core/proto/*.proto`) is the point, so package
names, service/method names, field names, numbers and types are identical; the schema is kept
here as a compact spec instead of .proto files because the image has no `protoc` and no
grpcio-tools.  `build_pool()` compiles the spec into FileDescriptorProtos at
import time (descriptor_pb2 -> descriptor_pool -> message_factory), and `emit_proto()` renders
standard .proto text for external tooling (grpcurl etc.).

Spec grammar (one declaration per line):
    package <name> [import <file> ...]
    msg <Name> <field>:<type>=<num> ...        types: scalar | Msg | pkg.Msg | []type | map<k,v>
    enum <Name> <VALUE>=<num> ...
    svc <Name> <Method>(<Req>)-><Resp> ...     "~Resp" = server-streaming response
"""
from __future__ import annotations

import functools
from typing import Dict, List, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

SPEC: Dict[str, str] = {}

SPEC["common.proto"] = """
package aios.common
msg Empty
msg Status success:bool=1 message:string=2
msg AgentId id:string=1
msg GoalId id:string=1
msg Goal id:string=1 description:string=2 priority:int32=3 source:string=4 status:string=5 created_at:int64=6 updated_at:int64=7 tags:[]string=8 metadata_json:bytes=9
enum GoalStatus GOAL_PENDING=0 GOAL_PLANNING=1 GOAL_IN_PROGRESS=2 GOAL_COMPLETED=3 GOAL_FAILED=4 GOAL_CANCELLED=5
msg Task id:string=1 goal_id:string=2 description:string=3 assigned_agent:string=4 status:string=5 intelligence_level:string=6 required_tools:[]string=7 depends_on:[]string=8 input_json:bytes=9 output_json:bytes=10 created_at:int64=11 started_at:int64=12 completed_at:int64=13 error:string=14
enum TaskStatus TASK_PENDING=0 TASK_ASSIGNED=1 TASK_IN_PROGRESS=2 TASK_COMPLETED=3 TASK_FAILED=4 TASK_CANCELLED=5
msg TaskResult task_id:string=1 success:bool=2 output_json:bytes=3 error:string=4 duration_ms:int64=5 tokens_used:int32=6 model_used:string=7
msg AgentRegistration agent_id:string=1 agent_type:string=2 capabilities:[]string=3 tool_namespaces:[]string=4 status:string=5 registered_at:int64=6
msg InferenceRequest prompt:string=1 system_prompt:string=2 max_tokens:int32=3 temperature:float=4 intelligence_level:string=5 model:string=6 requesting_agent:string=7 task_id:string=8
msg InferenceResponse text:string=1 tokens_used:int32=2 latency_ms:int64=3 model_used:string=4 intelligence_level:string=5
msg ServiceRegistration name:string=1 address:string=2 port:int32=3 protocol:string=4 status:string=5 registered_at:int64=6
msg HealthStatus healthy:bool=1 service:string=2 message:string=3 uptime_seconds:int64=4 details:map<string,string>=5
"""

SPEC["runtime.proto"] = """
package aios.runtime import common.proto
msg LoadModelRequest model_name:string=1 model_path:string=2 context_length:int32=3 gpu_layers:int32=4 threads:int32=5 port:int32=6
msg UnloadModelRequest model_name:string=1
msg ModelStatus model_name:string=1 status:string=2 port:int32=3 loaded_at:int64=4 last_used:int64=5 request_count:int64=6
msg ModelList models:[]ModelStatus=1
msg InferRequest model:string=1 prompt:string=2 system_prompt:string=3 max_tokens:int32=4 temperature:float=5 intelligence_level:string=6 requesting_agent:string=7 task_id:string=8
msg InferResponse text:string=1 tokens_used:int32=2 latency_ms:int64=3 model_used:string=4
msg InferChunk text:string=1 done:bool=2
svc AIRuntime LoadModel(LoadModelRequest)->ModelStatus UnloadModel(UnloadModelRequest)->aios.common.Status ListModels(aios.common.Empty)->ModelList Infer(InferRequest)->InferResponse StreamInfer(InferRequest)->~InferChunk HealthCheck(aios.common.Empty)->aios.common.HealthStatus
"""

SPEC["orchestrator.proto"] = """
package aios.orchestrator import common.proto
msg SubmitGoalRequest description:string=1 priority:int32=2 source:string=3 tags:[]string=4 metadata_json:bytes=5
msg GoalStatusResponse goal:aios.common.Goal=1 tasks:[]aios.common.Task=2 current_phase:string=3 progress_percent:double=4
msg ListGoalsRequest status_filter:string=1 limit:int32=2 offset:int32=3
msg GoalListResponse goals:[]aios.common.Goal=1 total:int32=2
msg HeartbeatRequest agent_id:string=1 status:string=2 current_task_id:string=3 cpu_usage:double=4 memory_usage_mb:double=5
msg AgentListResponse agents:[]aios.common.AgentRegistration=1
msg SystemStatusResponse active_goals:int32=1 pending_tasks:int32=2 active_agents:int32=3 loaded_models:[]string=4 cpu_percent:double=5 memory_used_mb:double=6 memory_total_mb:double=7 autonomy_level:string=8 uptime_seconds:int64=9
msg CapabilityRequest agent_id:string=1 capabilities:[]string=2 reason:string=3 duration_hours:int64=4
msg CapabilityResponse granted:bool=1 capabilities:[]string=2 expires_at:string=3 denial_reason:string=4
msg CapabilityRevocation agent_id:string=1 capabilities:[]string=2 revoke_all:bool=3
msg CreateScheduleRequest cron_expr:string=1 goal_template:string=2 priority:int32=3
msg ScheduleResponse schedule_id:string=1 success:bool=2
msg ScheduleEntry id:string=1 cron_expr:string=2 goal_template:string=3 priority:int32=4 enabled:bool=5 last_run:int64=6
msg ScheduleListResponse schedules:[]ScheduleEntry=1
msg DeleteScheduleRequest schedule_id:string=1
msg NodeRegistration node_id:string=1 hostname:string=2 address:string=3 agents:[]string=4 metadata:map<string,string>=5 max_tasks:uint32=6
msg NodeStatus node_id:string=1 cpu_usage:double=2 memory_usage:double=3 active_tasks:uint32=4
msg ListNodesRequest include_dead:bool=1
msg NodeInfo node_id:string=1 hostname:string=2 address:string=3 agents:[]string=4 cpu_usage:double=5 memory_usage:double=6 active_tasks:uint32=7 healthy:bool=8
msg NodeListResponse nodes:[]NodeInfo=1
svc Orchestrator SubmitGoal(SubmitGoalRequest)->aios.common.GoalId GetGoalStatus(aios.common.GoalId)->GoalStatusResponse CancelGoal(aios.common.GoalId)->aios.common.Status ListGoals(ListGoalsRequest)->GoalListResponse RegisterAgent(aios.common.AgentRegistration)->aios.common.Status UnregisterAgent(aios.common.AgentId)->aios.common.Status Heartbeat(HeartbeatRequest)->aios.common.Status ListAgents(aios.common.Empty)->AgentListResponse GetSystemStatus(aios.common.Empty)->SystemStatusResponse GetAssignedTask(aios.common.AgentId)->aios.common.Task ReportTaskResult(aios.common.TaskResult)->aios.common.Status RequestCapability(CapabilityRequest)->CapabilityResponse RevokeCapability(CapabilityRevocation)->aios.common.Status CreateSchedule(CreateScheduleRequest)->ScheduleResponse ListSchedules(aios.common.Empty)->ScheduleListResponse DeleteSchedule(DeleteScheduleRequest)->aios.common.Status RegisterNode(NodeRegistration)->aios.common.Status NodeHeartbeat(NodeStatus)->aios.common.Status ListNodes(ListNodesRequest)->NodeListResponse
"""

SPEC["agent.proto"] = """
package aios.agent import common.proto
msg CancelTaskRequest task_id:string=1 reason:string=2
msg AgentStatusResponse agent_id:string=1 agent_type:string=2 status:string=3 current_task_id:string=4 tasks_completed:int32=5 tasks_failed:int32=6 uptime_seconds:int64=7 cpu_usage:double=8 memory_usage_mb:double=9
svc Agent ExecuteTask(aios.common.Task)->aios.common.TaskResult CancelTask(CancelTaskRequest)->aios.common.Status GetStatus(aios.common.Empty)->AgentStatusResponse Shutdown(aios.common.Empty)->aios.common.Status
"""

SPEC["tools.proto"] = """
package aios.tools
msg ListToolsRequest namespace:string=1
msg ToolDefinition name:string=1 namespace:string=2 version:string=3 description:string=4 input_schema:bytes=5 output_schema:bytes=6 required_capabilities:[]string=7 risk_level:string=8 requires_confirmation:bool=9 idempotent:bool=10 reversible:bool=11 timeout_ms:int32=12 rollback_tool:string=13
msg ListToolsResponse tools:[]ToolDefinition=1
msg GetToolRequest name:string=1
msg ExecuteRequest tool_name:string=1 agent_id:string=2 task_id:string=3 input_json:bytes=4 reason:string=5
msg ExecuteResponse success:bool=1 output_json:bytes=2 error:string=3 execution_id:string=4 duration_ms:int64=5 backup_id:string=6
msg RollbackRequest execution_id:string=1 reason:string=2
msg RollbackResponse success:bool=1 error:string=2
msg RegisterToolRequest tool:ToolDefinition=1 handler_address:string=2
msg RegisterToolResponse accepted:bool=1 error:string=2
msg DeregisterToolRequest tool_name:string=1
msg Status success:bool=1 message:string=2
svc ToolRegistry ListTools(ListToolsRequest)->ListToolsResponse GetTool(GetToolRequest)->ToolDefinition Execute(ExecuteRequest)->ExecuteResponse Rollback(RollbackRequest)->RollbackResponse Register(RegisterToolRequest)->RegisterToolResponse Deregister(DeregisterToolRequest)->Status
"""

SPEC["api_gateway.proto"] = """
package aios.api_gateway import common.proto
msg ApiInferRequest prompt:string=1 system_prompt:string=2 max_tokens:int32=3 temperature:float=4 preferred_provider:string=5 requesting_agent:string=6 task_id:string=7 allow_fallback:bool=8
msg StreamChunk text:string=1 done:bool=2 provider:string=3
msg BudgetStatus claude_monthly_budget_usd:double=1 claude_used_usd:double=2 openai_monthly_budget_usd:double=3 openai_used_usd:double=4 days_remaining:int32=5 daily_rate_usd:double=6 budget_exceeded:bool=7
msg UsageRequest provider:string=1 days:int32=2
msg UsageRecord provider:string=1 model:string=2 input_tokens:int32=3 output_tokens:int32=4 cost_usd:double=5 timestamp:int64=6 requesting_agent:string=7 task_id:string=8
msg UsageResponse records:[]UsageRecord=1 total_cost_usd:double=2 total_requests:int32=3 total_tokens:int32=4
svc ApiGateway Infer(ApiInferRequest)->aios.common.InferenceResponse StreamInfer(ApiInferRequest)->~StreamChunk GetBudget(aios.common.Empty)->BudgetStatus GetUsage(UsageRequest)->UsageResponse
"""

SPEC["memory.proto"] = """
package aios.memory
msg Empty
msg Event id:string=1 timestamp:int64=2 category:string=3 source:string=4 data_json:bytes=5 critical:bool=6
msg RecentEventsRequest count:int32=1 category:string=2 source:string=3
msg EventList events:[]Event=1
msg MetricUpdate key:string=1 value:double=2 timestamp:int64=3
msg MetricRequest key:string=1
msg MetricValue key:string=1 value:double=2 timestamp:int64=3
msg SystemSnapshot cpu_percent:double=1 memory_used_mb:double=2 memory_total_mb:double=3 disk_used_gb:double=4 disk_total_gb:double=5 gpu_utilization:double=6 active_tasks:int32=7 active_agents:int32=8 loaded_models:[]string=9
msg GoalRecord id:string=1 description:string=2 status:string=3 priority:int32=4 created_at:int64=5 completed_at:int64=6 result:string=7 metadata_json:bytes=8
msg GoalUpdate id:string=1 status:string=2 result:string=3
msg GoalIdRequest goal_id:string=1
msg GoalList goals:[]GoalRecord=1
msg TaskRecord id:string=1 goal_id:string=2 description:string=3 agent:string=4 status:string=5 input_json:bytes=6 output_json:bytes=7 started_at:int64=8 completed_at:int64=9 duration_ms:int64=10 error:string=11
msg TaskList tasks:[]TaskRecord=1
msg ToolCallRecord id:string=1 task_id:string=2 tool_name:string=3 agent:string=4 input_json:bytes=5 output_json:bytes=6 success:bool=7 duration_ms:int64=8 reason:string=9 timestamp:int64=10
msg Decision id:string=1 context:string=2 options_json:bytes=3 chosen:string=4 reasoning:string=5 intelligence_level:string=6 model_used:string=7 outcome:string=8 timestamp:int64=9
msg Pattern id:string=1 trigger:string=2 action:string=3 success_rate:double=4 uses:int32=5 last_used:int64=6 created_from:string=7
msg PatternQuery trigger:string=1 min_success_rate:double=2
msg PatternResult pattern:Pattern=1 found:bool=2
msg PatternStatsUpdate id:string=1 success:bool=2
msg AgentState agent_name:string=1 state_json:bytes=2 updated_at:int64=3
msg AgentStateRequest agent_name:string=1
msg SemanticSearchRequest query:string=1 collections:[]string=2 n_results:int32=3 min_relevance:double=4
msg SearchResult content:string=1 metadata_json:bytes=2 relevance:double=3 collection:string=4 id:string=5
msg SearchResults results:[]SearchResult=1
msg Procedure id:string=1 name:string=2 description:string=3 steps_json:bytes=4 success_count:int32=5 fail_count:int32=6 avg_duration_ms:int64=7 tags:[]string=8 created_at:int64=9 last_used:int64=10
msg Incident id:string=1 description:string=2 symptoms_json:bytes=3 root_cause:string=4 resolution:string=5 resolved_by:string=6 prevention:string=7 timestamp:int64=8
msg ConfigChange id:string=1 file_path:string=2 content:string=3 changed_by:string=4 reason:string=5 timestamp:int64=6
msg KnowledgeEntry title:string=1 content:string=2 source:string=3 tags:[]string=4
msg ContextRequest task_description:string=1 max_tokens:int32=2 memory_tiers:[]string=3
msg ContextChunk source:string=1 content:string=2 relevance:double=3 tokens:int32=4
msg ContextResponse chunks:[]ContextChunk=1 total_tokens:int32=2
svc MemoryService PushEvent(Event)->Empty GetRecentEvents(RecentEventsRequest)->EventList UpdateMetric(MetricUpdate)->Empty GetMetric(MetricRequest)->MetricValue GetSystemSnapshot(Empty)->SystemSnapshot StoreGoal(GoalRecord)->Empty UpdateGoal(GoalUpdate)->Empty GetActiveGoals(Empty)->GoalList StoreTask(TaskRecord)->Empty GetTasksForGoal(GoalIdRequest)->TaskList StoreToolCall(ToolCallRecord)->Empty StoreDecision(Decision)->Empty StorePattern(Pattern)->Empty FindPattern(PatternQuery)->PatternResult UpdatePatternStats(PatternStatsUpdate)->Empty StoreAgentState(AgentState)->Empty GetAgentState(AgentStateRequest)->AgentState SemanticSearch(SemanticSearchRequest)->SearchResults StoreProcedure(Procedure)->Empty StoreIncident(Incident)->Empty StoreConfigChange(ConfigChange)->Empty SearchKnowledge(SemanticSearchRequest)->SearchResults AddKnowledge(KnowledgeEntry)->Empty AssembleContext(ContextRequest)->ContextResponse
"""

_SCALARS = {
    "double": descriptor_pb2.FieldDescriptorProto.TYPE_DOUBLE,
    "float": descriptor_pb2.FieldDescriptorProto.TYPE_FLOAT,
    "int64": descriptor_pb2.FieldDescriptorProto.TYPE_INT64,
    "uint64": descriptor_pb2.FieldDescriptorProto.TYPE_UINT64,
    "int32": descriptor_pb2.FieldDescriptorProto.TYPE_INT32,
    "uint32": descriptor_pb2.FieldDescriptorProto.TYPE_UINT32,
    "bool": descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
    "string": descriptor_pb2.FieldDescriptorProto.TYPE_STRING,
    "bytes": descriptor_pb2.FieldDescriptorProto.TYPE_BYTES,
}
F = descriptor_pb2.FieldDescriptorProto


def _qualify(t: str, pkg: str) -> str:
    return "." + t if "." in t else f".{pkg}.{t}"


def _camel(s: str) -> str:
    return "".join(p.capitalize() for p in s.split("_"))


def _parse(fname: str, text: str) -> Tuple[descriptor_pb2.FileDescriptorProto, list]:
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = fname
    fdp.syntax = "proto3"
    services = []
    pkg = ""
    for line in text.strip().splitlines():
        toks = line.split()
        kind = toks[0]
        if kind == "package":
            pkg = toks[1]
            fdp.package = pkg
            if len(toks) > 2 and toks[2] == "import":
                fdp.dependency.extend(toks[3:])
        elif kind == "msg":
            m = fdp.message_type.add()
            m.name = toks[1]
            for f in toks[2:]:
                name, rest = f.split(":", 1)
                ftype, num = rest.rsplit("=", 1)
                fd = m.field.add()
                fd.name = name
                fd.number = int(num)
                fd.json_name = name[0] + _camel(name)[1:] if "_" in name else name
                if ftype.startswith("map<"):
                    kt, vt = ftype[4:-1].split(",")
                    entry = m.nested_type.add()
                    entry.name = _camel(name) + "Entry"
                    entry.options.map_entry = True
                    for i, (n, t) in enumerate((("key", kt), ("value", vt)), 1):
                        ef = entry.field.add()
                        ef.name, ef.number, ef.label = n, i, F.LABEL_OPTIONAL
                        ef.json_name = n
                        ef.type = _SCALARS[t]
                    fd.label = F.LABEL_REPEATED
                    fd.type = F.TYPE_MESSAGE
                    fd.type_name = f".{pkg}.{m.name}.{entry.name}"
                    continue
                fd.label = F.LABEL_OPTIONAL
                if ftype.startswith("[]"):
                    fd.label = F.LABEL_REPEATED
                    ftype = ftype[2:]
                if ftype in _SCALARS:
                    fd.type = _SCALARS[ftype]
                else:
                    fd.type = F.TYPE_MESSAGE
                    fd.type_name = _qualify(ftype, pkg)
        elif kind == "enum":
            e = fdp.enum_type.add()
            e.name = toks[1]
            for v in toks[2:]:
                n, num = v.split("=")
                ev = e.value.add()
                ev.name, ev.number = n, int(num)
        elif kind == "svc":
            s = fdp.service.add()
            s.name = toks[1]
            for mdef in toks[2:]:
                mname, rest = mdef.split("(", 1)
                req, resp = rest.split(")->")
                md = s.method.add()
                md.name = mname
                md.input_type = _qualify(req, pkg)
                if resp.startswith("~"):
                    md.server_streaming = True
                    resp = resp[1:]
                md.output_type = _qualify(resp, pkg)
            services.append(s.name)
        else:
            raise ValueError(f"{fname}: bad spec line {line!r}")
    return fdp, services


ORDER = ["common.proto", "runtime.proto", "orchestrator.proto", "agent.proto", "tools.proto",
         "api_gateway.proto", "memory.proto"]


@functools.lru_cache(maxsize=1)
def build_pool() -> descriptor_pool.DescriptorPool:
    pool = descriptor_pool.DescriptorPool()
    for fname in ORDER:
        fdp, _ = _parse(fname, SPEC[fname])
        pool.Add(fdp)
    return pool


@functools.lru_cache(maxsize=None)
def message(full_name: str):
    """Message class by full name, e.g. message('aios.runtime.InferRequest')."""
    return message_factory.GetMessageClass(build_pool().FindMessageTypeByName(full_name))


@functools.lru_cache(maxsize=None)
def service(full_name: str):
    return build_pool().FindServiceByName(full_name)


SERVICES = {
    "aios.runtime.AIRuntime": 50055,
    "aios.orchestrator.Orchestrator": 50051,
    "aios.tools.ToolRegistry": 50052,
    "aios.memory.MemoryService": 50053,
    "aios.api_gateway.ApiGateway": 50054,
    "aios.agent.Agent": 0,
}


class _Namespace:
    """Attribute access to a package's messages: pb.runtime.InferRequest(...)."""

    def __init__(self, pkg: str):
        self._pkg = pkg

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        try:
            return message(f"{self._pkg}.{name}")
        except KeyError as e:
            raise AttributeError(name) from e


class pb:  # noqa: N801 - namespace object
    common = _Namespace("aios.common")
    runtime = _Namespace("aios.runtime")
    orchestrator = _Namespace("aios.orchestrator")
    agent = _Namespace("aios.agent")
    tools = _Namespace("aios.tools")
    api_gateway = _Namespace("aios.api_gateway")
    memory = _Namespace("aios.memory")


def emit_proto(fname: str) -> str:
    """Render one spec file as standard proto3 text."""
    fdp, _ = _parse(fname, SPEC[fname])
    inv = {v: k for k, v in _SCALARS.items()}
    out = ['syntax = "proto3";', f"package {fdp.package};", ""]
    for dep in fdp.dependency:
        out.append(f'import "{dep}";')

    def tname(fd):
        if fd.type == F.TYPE_MESSAGE:
            t = fd.type_name[1:]
            return t[len(fdp.package) + 1:] if t.startswith(fdp.package + ".") else t
        return inv[fd.type]

    for s in fdp.service:
        out.append(f"\nservice {s.name} {{")
        for md in s.method:
            req = md.input_type[1:].replace(fdp.package + ".", "")
            resp = md.output_type[1:].replace(fdp.package + ".", "")
            out.append(f"  rpc {md.name}({req}) returns ({'stream ' if md.server_streaming else ''}{resp});")
        out.append("}")
    for e in fdp.enum_type:
        out.append(f"\nenum {e.name} {{")
        out += [f"  {v.name} = {v.number};" for v in e.value]
        out.append("}")
    for m in fdp.message_type:
        maps = {n.name: n for n in m.nested_type if n.options.map_entry}
        out.append(f"\nmessage {m.name} {{")
        for fd in m.field:
            if fd.type == F.TYPE_MESSAGE and fd.type_name.split(".")[-1] in maps:
                ent = maps[fd.type_name.split(".")[-1]]
                out.append(f"  map<{inv[ent.field[0].type]}, {inv[ent.field[1].type]}> {fd.name} = {fd.number};")
                continue
            rep = "repeated " if fd.label == F.LABEL_REPEATED else ""
            out.append(f"  {rep}{tname(fd)} {fd.name} = {fd.number};")
        out.append("}")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    import os
    import sys

    dst = sys.argv[1] if len(sys.argv) > 1 else "proto"
    os.makedirs(dst, exist_ok=True)
    for f in ORDER:
        with open(os.path.join(dst, f), "w") as fh:
            fh.write(emit_proto(f))
    print(f"wrote {len(ORDER)} .proto files to {dst}")

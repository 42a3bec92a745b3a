"""Memory tier access latency (aios.memory.MemoryService over the native memory core) against the
reference's targets: operational < 1 ms, working < 5 ms, long-term < 50 ms
(docs/architecture/MEMORY-SYSTEM.md:17,23,30).

Two measurements of the same RPC mix, each over fresh databases:
  * rpc      -- the aios-memory daemon as its own process (as under aios-init) on a loopback port; the
                round trip a client sees (client stub, gRPC, server, native store).  `grpc_floor_ms` is an
                empty RPC against a bare gRPC server on the same machine: the transport's share.
  * service  -- the same handlers called in-process: the tier access itself (native store + record
                conversion), without the transport.
The long-term / knowledge tiers are filled first (--entries each) so the searches run over a populated
store; the working tier holds --goals active goals (upserted in rotation, as the orchestrator updates
its goals) with their tasks.  p50 / p99 over --calls calls per RPC.

  python tools/bench_memory.py [--calls 300] [--entries 2000] [--goals 20] [--json out.json]
"""
import argparse
import asyncio
import json
import os
import shutil
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import grpc  # noqa: E402

from aios_amd.memory.service import MemoryServiceImpl  # noqa: E402
from aios_amd.rpc import client  # noqa: E402
from aios_amd.rpc.schema import message  # noqa: E402

TARGET_MS = {"operational": 1.0, "working": 5.0, "long-term": 50.0}
TOPICS = ["disk", "gpu temperature", "nginx", "firewall", "backup", "kernel update", "memory leak", "network"]
M = lambda _msg, **kw: message("aios.memory." + _msg)(**kw)  # noqa: E731


def stats(lat):
    lat = sorted(lat)
    return {"p50_ms": round(statistics.median(lat), 3), "p99_ms": round(lat[min(len(lat) - 1, int(0.99 * len(lat)))], 3)}


def rpc_mix(goals):
    """tier -> {rpc name: i -> request}"""
    return {
        "operational": {
            "PushEvent": lambda i: M("Event", id=f"e{i}", timestamp=i + 1, category="bench", source="b", data_json=b"{}"),
            "GetRecentEvents": lambda i: M("RecentEventsRequest", count=50),
            "UpdateMetric": lambda i: M("MetricUpdate", key="gpu.temp", value=float(i), timestamp=i + 1),
            "GetMetric": lambda i: M("MetricRequest", key="gpu.temp"),
        },
        "working": {
            "StoreGoal": lambda i: M("GoalRecord", id=f"g{i % goals}", description=f"goal {i}", status="pending",
                                     priority=5, created_at=i + 1),
            "GetActiveGoals": lambda i: M("Empty"),
            "StoreTask": lambda i: M("TaskRecord", id=f"t{i}", goal_id=f"g{i % goals}", description="task",
                                     status="pending"),
            "GetTasksForGoal": lambda i: M("GoalIdRequest", goal_id=f"g{i % goals}"),
            "StoreAgentState": lambda i: M("AgentState", agent_name="system", state_json=b"{}", updated_at=i + 1),
            "GetAgentState": lambda i: M("AgentStateRequest", agent_name="system"),
        },
        "long-term": {
            "SemanticSearch": lambda i: M("SemanticSearchRequest", query=f"{TOPICS[i % 8]} problem", n_results=5),
            "SearchKnowledge": lambda i: M("SemanticSearchRequest", query=f"{TOPICS[i % 8]} issue", n_results=5),
            "AssembleContext": lambda i: M("ContextRequest", task_description=f"fix the {TOPICS[i % 8]}", max_tokens=1024),
        },
    }


async def exercise(call, args):
    """Populate through `call(rpc, request)`, then time the RPC mix."""
    for i in range(args.entries):
        t = TOPICS[i % len(TOPICS)]
        await call("AddKnowledge", M("KnowledgeEntry", title=f"{t} note {i}", content=f"how to handle {t} issue "
                                     f"number {i} on an MI355X node: check the logs, then the service state",
                                     source="bench", tags=[t]))
        await call("StoreProcedure", M("Procedure", name=f"fix {t} {i}", description=f"procedure for {t} case {i}",
                                       steps_json=json.dumps([{"step": "inspect"}, {"step": "repair"}]).encode()))
    out = {}
    for tier, rpcs in rpc_mix(args.goals).items():
        res = {}
        for name, req in rpcs.items():
            lat = []
            for i in range(args.calls):
                r = req(i)
                t0 = time.perf_counter()
                await call(name, r)
                lat.append((time.perf_counter() - t0) * 1e3)
            res[name] = stats(lat)
        worst = max(r["p50_ms"] for r in res.values())
        out[tier] = {"calls": res, "worst_p50_ms": worst, "meets_target": worst < TARGET_MS[tier]}
    return out


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


async def grpc_floor(calls):
    """Empty unary RPC round trip against a bare in-process gRPC server (no service code at all)."""
    E = message("aios.memory.Empty")

    async def echo(req, ctx):
        return E()

    server = grpc.aio.server()
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("bench.Floor", {
        "Echo": grpc.unary_unary_rpc_method_handler(echo, request_deserializer=E.FromString,
                                                    response_serializer=E.SerializeToString)}),))
    port = server.add_insecure_port("127.0.0.1:0")
    await server.start()
    try:
        async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch:
            f = ch.unary_unary("/bench.Floor/Echo", request_serializer=E.SerializeToString,
                               response_deserializer=E.FromString)
            lat = []
            for _ in range(calls):
                t0 = time.perf_counter()
                await f(E())
                lat.append((time.perf_counter() - t0) * 1e3)
    finally:
        await server.stop(0)
    return stats(lat)


async def over_rpc(args):
    d = tempfile.mkdtemp(prefix="aios-mem-")
    port = free_port()
    proc = subprocess.Popen([sys.executable, "-m", "aios_amd.memory.service", "--addr", f"127.0.0.1:{port}",
                             "--working-db", os.path.join(d, "working.db"), "--longterm-db",
                             os.path.join(d, "longterm.db"), "--knowledge-db", os.path.join(d, "knowledge.db")],
                            cwd=ROOT, stdout=open(os.path.join(d, "memory.log"), "w"), stderr=subprocess.STDOUT,
                            env=dict(os.environ, AIOS_DATA_DIR=d))
    try:
        st = client.Stub(client.channel(f"127.0.0.1:{port}", fresh=True), "aios.memory.MemoryService", timeout=30)
        t0 = time.perf_counter()
        while True:
            try:
                await st.GetSystemSnapshot(M("Empty"))
                break
            except grpc.aio.AioRpcError:
                if proc.poll() is not None or time.perf_counter() - t0 > 60:
                    raise RuntimeError("aios-memory did not come up")
                await asyncio.sleep(0.1)
        return await exercise(lambda name, req: getattr(st, name)(req), args)
    finally:
        proc.terminate()
        try:
            proc.wait(timeout=20)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
        await client.close_all()
        shutil.rmtree(d, ignore_errors=True)


async def in_process(args):
    d = tempfile.mkdtemp(prefix="aios-mem-")
    svc = MemoryServiceImpl(os.path.join(d, "working.db"), os.path.join(d, "longterm.db"), os.path.join(d, "knowledge.db"))
    try:
        return await exercise(lambda name, req: getattr(svc, name)(req, None), args)
    finally:
        svc.pool.shutdown()
        del svc
        shutil.rmtree(d, ignore_errors=True)


async def run(args):
    return {"bench": "memory tier access latency", "calls": args.calls, "entries_per_long_term_store": args.entries,
            "active_goals": args.goals, "target_ms": TARGET_MS, "grpc_floor_ms": await grpc_floor(args.calls),
            "rpc": await over_rpc(args), "service": await in_process(args)}


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--entries", type=int, default=2000)
    ap.add_argument("--goals", type=int, default=20, help="active goals in the working tier")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    out = asyncio.run(run(args))
    print(json.dumps(out), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())

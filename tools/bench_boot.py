"""Boot to autonomy on one node: the whole stack under aios-init (scripts/run-local.sh: runtime with the
synthetic TinyLlama + Mistral tiers, tools, memory, api-gateway, orchestrator with its agents), timed from
the init process's start until every service answers and the runtime reports its models loaded -- the
reference's "boot to autonomy loop < 30 s" target (docs/architecture/SYSTEM.md:366) -- then
one tactical goal submitted over gRPC and timed until the orchestrator holds its planned tasks.

  python tools/bench_boot.py [--timeout 240] [--json out.json]

The stack runs as the caller (no root, private data dir, no mounts); the process group it starts is
terminated at the end.  This process never touches the GPU (the runtime daemon does).
"""
import argparse
import asyncio
import json
import os
import signal
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from aios_amd.rpc import client  # noqa: E402
from aios_amd.rpc.schema import message  # noqa: E402

PORTS = {"orchestrator": 50051, "tools": 50052, "memory": 50053, "api_gateway": 50054, "runtime": 50055}


async def probe(name: str, want_models: int):
    """True when the service answers (the runtime: with >= want_models models loaded)."""
    ch = client.channel(f"127.0.0.1:{PORTS[name]}", fresh=True)
    try:
        empty = message("aios.common.Empty")()
        if name == "runtime":
            st = client.Stub(ch, "aios.runtime.AIRuntime", timeout=2)
            ml = await st.ListModels(empty)
            return sum(1 for m in ml.models if m.status in ("loaded", "ready")) >= want_models
        if name == "orchestrator":
            st = client.Stub(ch, "aios.orchestrator.Orchestrator", timeout=2)
            await st.ListGoals(message("aios.orchestrator.ListGoalsRequest")())
            return True
        if name == "tools":
            st = client.Stub(ch, "aios.tools.ToolRegistry", timeout=2)
            r = await st.ListTools(message("aios.tools.ListToolsRequest")())
            return len(r.tools) > 0
        if name == "memory":
            st = client.Stub(ch, "aios.memory.MemoryService", timeout=2)
            await st.GetSystemSnapshot(message("aios.memory.Empty")())
            return True
        if name == "api_gateway":
            st = client.Stub(ch, "aios.api_gateway.ApiGateway", timeout=2)
            await st.GetBudget(empty)
            return True
    except Exception:
        return False
    finally:
        await ch.close()
    return False


async def run(args):
    data = tempfile.mkdtemp(prefix="aios-boot-")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    t0 = time.perf_counter()
    proc = subprocess.Popen(["bash", os.path.join(ROOT, "scripts", "run-local.sh"), "--data", data, "--seconds",
                             str(int(args.timeout) + 30)], stdout=open(os.path.join(data, "init.log"), "w"),
                            stderr=subprocess.STDOUT, env=env, start_new_session=True)
    ready = {}
    out = {"bench": "boot to autonomy (aios-init -> every service answering, runtime models loaded)",
           "target_s": 30, "data": "synthetic models (random-init TinyLlama-1.1B + Mistral-7B Q4_K_M)"}
    try:
        while len(ready) < len(PORTS) and time.perf_counter() - t0 < args.timeout:
            if proc.poll() is not None:
                raise RuntimeError(f"aios-init exited with {proc.returncode}")
            for name in PORTS:
                if name not in ready and await probe(name, args.models):
                    ready[name] = round(time.perf_counter() - t0, 2)
            await asyncio.sleep(0.1)
        out["service_ready_s"] = ready
        out["boot_to_autonomy_s"] = max(ready.values()) if len(ready) == len(PORTS) else None
        if out["boot_to_autonomy_s"] is not None:
            # one tactical goal through the running stack: submit -> planned tasks in the orchestrator
            st = client.Stub(client.channel("127.0.0.1:50051", fresh=True), "aios.orchestrator.Orchestrator", timeout=10)
            g0 = time.perf_counter()
            gid = await st.SubmitGoal(message("aios.orchestrator.SubmitGoalRequest")(
                description="analyze why the disk filled up last night and clean it",  # a tactical goal: LLM decomposition
                priority=5, source="bench_boot"))
            while time.perf_counter() - g0 < 120:
                s = await st.GetGoalStatus(gid)
                if len(s.tasks) > 0:
                    out["goal_to_first_task_s"] = round(time.perf_counter() - g0, 3)
                    out["tasks"] = [t.description[:80] for t in s.tasks][:6]
                    out["goal_phase"] = s.current_phase
                    break
                await asyncio.sleep(0.05)
    finally:
        try:
            os.killpg(proc.pid, signal.SIGTERM)
            proc.wait(timeout=30)
        except (ProcessLookupError, subprocess.TimeoutExpired):
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
        await client.close_all()
    if args.log:
        import shutil

        shutil.copy(os.path.join(data, "init.log"), args.log)
    if out.get("boot_to_autonomy_s") is None:
        with open(os.path.join(data, "init.log")) as f:
            out["init_log_tail"] = f.read()[-3000:]
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--timeout", type=float, default=240)
    ap.add_argument("--models", type=int, default=2, help="models the runtime must report loaded")
    ap.add_argument("--json", default="")
    ap.add_argument("--log", default="", help="copy the stack's log here")
    args = ap.parse_args()
    out = asyncio.run(run(args))
    print(json.dumps(out), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0 if out.get("boot_to_autonomy_s") is not None else 1


if __name__ == "__main__":
    sys.exit(main())

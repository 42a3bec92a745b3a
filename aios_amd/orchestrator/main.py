"""aios-orchestrator daemon (reference `agent-core/src/main.rs:589-801`).

Starts: the Orchestrator gRPC service on :50051, the autonomy loop (500 ms), the health checker
(10 s after a 60 s grace), the proactive goal generator (60 s), the cron scheduler (60 s), the
event bus consumer, cluster/discovery maintenance (15 s), the management console (:9090) and,
unless --no-agents, the Python agent spawner.
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal

from ..rpc.server import RpcServer
from ..utils.env import setup_logging
from .autonomy import AutonomyLoop
from .loops import (AgentSpawner, EventQueue, HealthChecker, ProactiveConfig, load_agent_configs, maintenance_loop,
                    proactive_loop, scheduler_loop)
from .management import ManagementConsole
from .service import OrchestratorService
from .state import OrchestratorState

log = logging.getLogger("aios.orchestrator")


async def amain(args):
    st = OrchestratorState(args.data_dir or None)
    st.health = HealthChecker(grace=args.health_grace, on_change=lambda name, up, s: st.emit(
        "service_recovered" if up else "service_unhealthy", name,
        {"address": s.address, "consecutive_failures": s.consecutive_failures}, "info" if up else "critical"))
    st.install_default_subscriptions()
    svc = OrchestratorService(st)
    server = RpcServer(args.addr, {"aios.orchestrator.Orchestrator": svc})
    await server.start()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except NotImplementedError:
            pass
    st.event_queue = EventQueue(st)
    tasks = [AutonomyLoop(st, args.tick_ms / 1000.0).run(stop), st.health.run(stop),
             scheduler_loop(st, stop), st.event_queue.run(stop), maintenance_loop(st, stop)]
    if not args.no_proactive:
        from ..utils import config as node_config

        mon = node_config.load().monitoring  # [monitoring] thresholds of the node config
        tasks.append(proactive_loop(st, stop, ProactiveConfig(cpu_threshold=mon.cpu_threshold,
                                                              memory_threshold=mon.memory_threshold,
                                                              disk_threshold=mon.disk_threshold)))
    console = None
    if args.console_port > 0:
        console = ManagementConsole(st, port=args.console_port)
        await console.start()
    if not args.no_agents:
        port = server.port
        tasks.append(AgentSpawner(load_agent_configs(args.agents_dir), f"127.0.0.1:{port}").run(stop))
    log.info("orchestrator up (node %s)", st.node_id)
    await asyncio.gather(*tasks)
    if console:
        await console.stop()
    await server.stop()


def main(argv=None):
    ap = argparse.ArgumentParser(description="aiOS orchestrator (aios.orchestrator.Orchestrator)")
    ap.add_argument("--addr", default=os.environ.get("AIOS_ORCHESTRATOR_LISTEN", "0.0.0.0:50051"))
    ap.add_argument("--data-dir", default="")
    ap.add_argument("--tick-ms", type=int, default=500)
    ap.add_argument("--console-port", type=int, default=int(os.environ.get("AIOS_CONSOLE_PORT", "9090")))
    ap.add_argument("--agents-dir", default=os.environ.get("AIOS_AGENTS_DIR", "/etc/aios/agents"))
    ap.add_argument("--health-grace", type=float, default=60.0)
    ap.add_argument("--no-agents", action="store_true")
    ap.add_argument("--no-proactive", action="store_true")
    args = ap.parse_args(argv)
    setup_logging("aios-orchestrator")
    asyncio.run(amain(args))


if __name__ == "__main__":
    main()

"""aios-runtime daemon (`runtime/src/main.rs` equivalent).

* builds the ModelManager on the local MI355X,
* auto-loads every `*.gguf` in $AIOS_MODEL_DIR (default /var/lib/aios/models/) with the
  reference's size-based context heuristic, plus `AIOS_SYNTHETIC_MODELS` entries
  (`name=synthetic:preset[:recipe]`, comma separated),
* serves aios.runtime.AIRuntime on [::]:50055 (AIOS_RUNTIME_ADDR), with a 10 s health loop
  that marks models whose engine died as errored.
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
from pathlib import Path

from ..rpc.client import Stub, channel
from ..rpc.schema import pb
from ..rpc.server import RpcServer
from .model_manager import ModelManager
from .service import AIRuntimeService

log = logging.getLogger("aios.runtime")
HEALTH_CHECK_INTERVAL = 10.0


async def auto_load(svc: AIRuntimeService, model_dir: str, cfg=None):
    """Start-up model pool: the node config's always-loaded tiers first (context length, TP degree
    and device from [models.<tier>] -- the reference runtime ignored that section, App. A #27),
    then every other *.gguf in the model directory (reference auto-load, runtime/src/main.rs:65-132),
    then AIOS_SYNTHETIC_MODELS specs."""
    loaded = set()
    for t in (cfg.tier_plan() if cfg is not None else []):
        spec, ctx = t["spec"], t["ctx"]
        base = spec.partition("#")[0]
        name = t["name"] if base.startswith("synthetic:") else Path(base).stem
        loaded.add(base)
        if t["on_demand"]:
            log.info("tier %s (%s) registered for on-demand load", t["name"], spec)
            svc.mgr.register_on_demand(name, spec, ctx, t["devices"], t["idle_unload_s"])
            continue
        log.info("loading %s tier %s from %s (ctx %s, devices %s)", t["name"], name, spec, ctx or "auto",
                 t["devices"] or "default")
        for m in await svc.mgr.load_replicas(name, spec, ctx, t["devices"], t["idle_unload_s"]):
            if m.status == "ready" and svc.http:
                await svc.start_http(m)
    d = Path(model_dir)
    if d.is_dir():
        for f in sorted(d.glob("*.gguf")):
            if str(f) in loaded:
                continue
            req_name = f.stem
            log.info("auto-loading %s", f)
            m = await svc.mgr.load_model(req_name, str(f))
            if m.status == "ready" and svc.http:
                await svc.start_http(m)
    for spec in filter(None, os.environ.get("AIOS_SYNTHETIC_MODELS", "").split(",")):
        name, _, path = spec.partition("=")
        m = await svc.mgr.load_model(name.strip(), path.strip())
        if m.status == "ready" and svc.http:
            await svc.start_http(m)


async def publish_metrics(mgr: ModelManager, addr: str):
    """Best effort: runtime metrics -> MemoryService.UpdateMetric (the reference's operational
    store has a `gpu.utilization` key that no producer ever writes)."""
    try:
        stub = Stub(channel(addr), "aios.memory.MemoryService", timeout=2.0)
        for k, v in mgr.metrics().items():
            await stub.UpdateMetric(pb.memory.MetricUpdate(key=k, value=float(v)))
    except Exception as e:  # noqa: BLE001 - memory service not up
        log.debug("metric publish skipped: %s", e)


async def health_loop(mgr: ModelManager, stop: asyncio.Event, memory_addr: str = ""):
    """10 s health pass (runtime/src/main.rs:55-63): supervision (dead scheduler / engine error /
    decode stall -> error -> bounded auto-reload) and metric publication."""
    memory_addr = memory_addr or os.environ.get("AIOS_MEMORY_ADDR", "127.0.0.1:50053")
    while not stop.is_set():
        try:
            await mgr.supervise()
        except Exception:  # noqa: BLE001
            log.exception("supervision pass failed")
        await publish_metrics(mgr, memory_addr)
        try:
            await asyncio.wait_for(stop.wait(), HEALTH_CHECK_INTERVAL)
        except asyncio.TimeoutError:
            pass


async def amain(args):
    from ..utils import config as node_config

    cfg = node_config.load()
    for w in cfg.warnings:
        log.warning("config: %s", w)
    max_batch = args.max_batch or cfg.models.max_batch
    max_slots = args.max_slots or cfg.models.max_slots
    tp_env = cfg.tp_devices_env()
    if tp_env and "AIOS_TP_DEVICES" not in os.environ:
        os.environ["AIOS_TP_DEVICES"] = tp_env
    mgr = ModelManager(device=args.device, max_batch=max_batch, max_slots=max_slots,
                       base_port=int(os.environ.get("AIOS_RUNTIME_BASE_PORT", "8080")))
    svc = AIRuntimeService(mgr, http=not args.no_http)
    server = RpcServer(args.addr, {"aios.runtime.AIRuntime": svc})
    await server.start()
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except NotImplementedError:
            pass
    asyncio.ensure_future(auto_load(svc, args.model_dir, cfg))
    await health_loop(mgr, stop)
    await server.stop()
    await svc.close()
    stuck = mgr.join_abandoned(5.0)
    if stuck:
        log.warning("%d stalled engine thread(s) still blocked at shutdown", stuck)


def main(argv=None):
    ap = argparse.ArgumentParser(description="aiOS MI355X AI runtime")
    ap.add_argument("--addr", default=os.environ.get("AIOS_RUNTIME_ADDR", "[::]:50055"))
    ap.add_argument("--model-dir", default=os.environ.get("AIOS_MODEL_DIR", "/var/lib/aios/models/"))
    ap.add_argument("--device", type=int, default=int(os.environ.get("AIOS_DEVICE", "0")))
    ap.add_argument("--max-batch", type=int, default=0, help="0 = [models] max_batch of the node config")
    ap.add_argument("--max-slots", type=int, default=0, help="0 = [models] max_slots of the node config")
    ap.add_argument("--no-http", action="store_true")
    args = ap.parse_args(argv)
    logging.basicConfig(level=os.environ.get("AIOS_LOG", "INFO"), format="%(asctime)s %(levelname)s %(name)s %(message)s")
    asyncio.run(amain(args))


if __name__ == "__main__":
    main()

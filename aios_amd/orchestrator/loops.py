"""Orchestrator background loops: health checker, proactive goal generator, cron scheduler,
event bus, cluster / discovery maintenance and the Python agent spawner.

Reference map:
  HealthChecker       agent-core/src/health.rs:34-127   (TCP probe every 10 s after a 60 s grace)
  proactive           agent-core/src/proactive.rs:22-370 (60 s; cpu>90, mem>85, disk>90, failed
                      agents, services with >=6 consecutive failures, cert age >30 d, backup age
                      >24 h, DNS/ping, >50 ERROR lines, world-writable /etc files; keyword dedup)
  cron scheduler      agent-core/src/scheduler.rs:104-183 (60 s tick, at most once per minute)
  event bus           agent-core/src/event_bus.rs:116-210 (subscriptions -> goals)
  cluster / discovery cluster.rs:136-158, discovery.rs:148-164 (15 s prune)
  agent spawner       agent-core/src/agent_spawner.rs:64-315 (agents/*.toml, 5 s monitor,
                      <=5 restarts, 5 s delay)
Probes use the native no-shell runner (`_core.run_cmd`) for nslookup/ping/find.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import subprocess
import sys
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..utils import sysinfo
from ..utils.env import addr, data_dir
from .state import OrchestratorState, core

log = logging.getLogger("aios.orchestrator.loops")


async def _sleep(stop: asyncio.Event, s: float) -> bool:
    """Sleep s seconds; True if stop was requested."""
    try:
        await asyncio.wait_for(stop.wait(), s)
        return True
    except asyncio.TimeoutError:
        return False


# ---------------------------------------------------------------------------------- health
@dataclass
class ServiceHealth:
    name: str
    address: str
    healthy: bool = False
    last_check_ms: float = 0.0
    last_checked_at: int = 0
    consecutive_failures: int = 0


class HealthChecker:
    def __init__(self, services: Optional[Dict[str, str]] = None, interval: float = 10.0, timeout: float = 2.0,
                 grace: float = 60.0, on_change=None):
        names = services or {n: addr(n) for n in ("runtime", "tools", "memory", "api-gateway")}
        self.services = {n: ServiceHealth(n, a) for n, a in names.items()}
        self.interval, self.timeout, self.grace = interval, timeout, grace
        self.on_change = on_change  # (service, healthy_now, ServiceHealth) on every transition
        self._seen: Dict[str, bool] = {}

    async def _probe(self, s: ServiceHealth):
        host, _, port = s.address.rpartition(":")
        t0 = time.perf_counter()
        try:
            _, w = await asyncio.wait_for(asyncio.open_connection(host.strip("[]") or "127.0.0.1", int(port)),
                                          self.timeout)
            w.close()
            ok = True
        except (OSError, asyncio.TimeoutError, ValueError):
            ok = False
        s.last_check_ms = (time.perf_counter() - t0) * 1000
        s.last_checked_at = int(time.time())
        if ok:
            s.healthy, s.consecutive_failures = True, 0
        else:
            s.healthy = False
            s.consecutive_failures += 1
            if s.consecutive_failures <= 3:
                log.warning("service %s health check failed (attempt %d)", s.name, s.consecutive_failures)
        # transitions, debounced: down after 3 consecutive failed probes (also a service that never
        # came up), up again on the first good probe after a reported down
        was = self._seen.get(s.name)
        now = True if s.healthy else (False if s.consecutive_failures >= 3 else was)
        if now is not None and now != was:
            self._seen[s.name] = now
            if self.on_change is not None and (not now or was is False):
                try:
                    self.on_change(s.name, now, s)
                except Exception:  # noqa: BLE001
                    log.exception("health transition hook failed")

    async def check_all(self):
        await asyncio.gather(*(self._probe(s) for s in self.services.values()))

    def status(self) -> List[dict]:
        return [s.__dict__.copy() for s in self.services.values()]

    def all_healthy(self) -> bool:
        return all(s.healthy for s in self.services.values())

    async def run(self, stop: asyncio.Event):
        if await _sleep(stop, self.grace):
            return
        while True:
            await self.check_all()
            if await _sleep(stop, self.interval):
                return


# ---------------------------------------------------------------------------------- proactive
@dataclass
class ProactiveConfig:
    interval: float = 60.0
    cpu_threshold: float = 90.0
    memory_threshold: float = 85.0
    disk_threshold: float = 90.0
    cert_path: str = field(default_factory=lambda: os.path.join(data_dir(), "certs", "server.crt"))
    backup_status_path: str = field(default_factory=lambda: os.path.join(data_dir(), "backup_status.json"))
    log_path: str = "/var/log/aios/orchestrator.log"
    network_probe: bool = True
    etc_probe: bool = True
    sysfs_root: str = "/"


def has_similar_active_goal(st: OrchestratorState, description: str) -> bool:
    goals, _ = st.goal_engine.list("", 100, 0)
    kws = [w for w in description.split() if len(w) > 4][:5]
    need = max(len(kws), 1) // 2 + 1
    for g in goals:
        if g["status"] in ("completed", "cancelled"):
            continue
        d = g["description"].lower()
        if sum(1 for k in kws if k.lower() in d) >= need:
            return True
    return False


def proactive_candidates(st: OrchestratorState, cfg: ProactiveConfig) -> List[tuple]:
    out = []
    cpu = sysinfo.cpu_percent()
    if cpu > cfg.cpu_threshold:
        out.append((f"Investigate high CPU usage ({cpu:.1f}% > {cfg.cpu_threshold:.0f}% threshold). "
                    "Identify top processes and take corrective action.", 7))
    used, total = sysinfo.memory_mb()
    if total > 0 and 100 * used / total > cfg.memory_threshold:
        out.append((f"Investigate high memory usage ({100 * used / total:.1f}% > {cfg.memory_threshold:.0f}% "
                    "threshold). Identify memory-heavy processes and free memory.", 7))
    dp = sysinfo.disk_percent("/")
    if dp > cfg.disk_threshold:
        out.append((f"Disk usage critically high ({dp:.1f}% > {cfg.disk_threshold:.0f}% threshold). "
                    "Clean up temporary files, old logs, and unnecessary data.", 8))
    failed = [a["agent_id"] for a in st.router.list() if a.get("status") in ("failed", "unresponsive")]
    if failed:
        out.append((f"Restart failed agents: {', '.join(failed)}. Investigate root cause.", 8))
    if st.health is not None:
        bad = [s["name"] for s in st.health.status() if not s["healthy"] and s["consecutive_failures"] >= 6]
        if bad:
            out.append((f"Services unhealthy: {', '.join(bad)}. Restart and investigate root cause.", 9))
    try:
        age_d = (time.time() - os.stat(cfg.cert_path).st_mtime) / 86400
        if age_d > 30:
            out.append((f"TLS certificate is {int(age_d)} days old. Rotate certificates using sec.cert_rotate "
                        "before expiry.", 7))
    except OSError:
        pass
    try:
        with open(cfg.backup_status_path) as f:
            last = int(json.load(f).get("last_backup_timestamp", 0))
        hours = (int(time.time()) - last) // 3600
        if last and hours > 24:
            out.append((f"No backup in {hours} hours. Run system backup to protect data and configurations.", 6))
    except (OSError, ValueError, AttributeError):
        pass
    if cfg.network_probe:
        dns = core.run_cmd(["nslookup", "1.1.1.1"], 5000)
        if dns["exit_code"] != 0:
            ping = core.run_cmd(["ping", "-c", "1", "-W", "2", "1.1.1.1"], 5000)
            if ping["exit_code"] != 0:
                out.append(("Network connectivity issue: DNS and ping to 1.1.1.1 failed. Diagnose network "
                            "configuration and restore connectivity.", 9))
    try:
        with open(cfg.log_path, errors="replace") as f:
            lines = f.readlines()[-500:]
        errs = sum(1 for ln in lines if "ERROR" in ln or "CRITICAL" in ln)
        if errs > 50:
            out.append((f"Log anomaly: {errs} ERROR/CRITICAL entries in recent logs. Investigate root cause and "
                        "resolve recurring errors.", 7))
    except OSError:
        pass
    try:  # MI355X RAS: uncorrectable HBM ECC / xGMI link errors, overtemperature (amdgpu sysfs)
        gh = sysinfo.gpu_health(cfg.sysfs_root)
        for p in gh["problems"]:
            if p["kind"] == "uncorrectable_ecc":
                out.append((f"GPU {p['card']} reports {p['count']} uncorrectable ECC errors "
                            f"({', '.join(p['blocks'])}). Drain its model tiers, move them to healthy GPUs and "
                            "schedule a GPU reset.", 9))
            elif p["kind"] == "xgmi_link_errors":
                out.append((f"GPU {p['card']} reports {p['count']} uncorrectable xGMI link errors. Move "
                            "tensor-parallel tiers off this GPU and check the node's xGMI links.", 9))
            else:
                out.append((f"GPU {p['card']} is overheating ({p['temp_c']:.0f} C). Reduce its load and check "
                            "cooling.", 8))
    except Exception:  # pragma: no cover - no GPU sysfs
        pass
    if cfg.etc_probe:
        r = core.run_cmd(["find", "/etc", "-maxdepth", "2", "-perm", "-o+w", "-type", "f"], 10000)
        n = len([ln for ln in r["stdout"].decode(errors="replace").splitlines() if ln.strip()])
        if n > 0:
            out.append((f"Security: {n} world-writable files found in /etc. Fix file permissions to prevent "
                        "unauthorized modification.", 8))
    return out


async def proactive_loop(st: OrchestratorState, stop: asyncio.Event, cfg: Optional[ProactiveConfig] = None):
    cfg = cfg or ProactiveConfig()
    log.info("proactive goal generator started (interval=%ds)", cfg.interval)
    while not await _sleep(stop, cfg.interval):
        try:
            cands = await asyncio.get_running_loop().run_in_executor(None, proactive_candidates, st, cfg)
            for desc, prio in cands:
                st.emit("proactive_trigger", "proactive", {"description": desc, "priority": prio},
                        "critical" if prio >= 9 else "warning")
                if has_similar_active_goal(st, desc):
                    continue
                g = await st.submit_goal(desc, prio, "proactive")
                log.info("proactive goal %s: %s", g["id"], desc[:80])
        except Exception:
            log.exception("proactive check failed")


# ---------------------------------------------------------------------------------- cron / events
async def scheduler_loop(st: OrchestratorState, stop: asyncio.Event, interval: float = 60.0):
    while True:
        try:
            for e in st.schedules.due(int(time.time())):
                g = await st.submit_goal(e["goal_template"], int(e["priority"]), "scheduler")
                log.info("scheduled goal %s fired from %s (%s)", g["id"], e["id"], e["cron_expr"])
        except Exception:
            log.exception("scheduler tick failed")
        if await _sleep(stop, interval):
            return


class EventQueue:
    """Bounded async queue in front of the native EventBus (event_bus.rs: mpsc(1000))."""

    def __init__(self, st: OrchestratorState, maxsize: int = 1000):
        self.st = st
        self.q: asyncio.Queue = asyncio.Queue(maxsize)

    def publish(self, event: dict) -> bool:
        try:
            self.q.put_nowait(event)
            return True
        except asyncio.QueueFull:
            log.warning("event queue full; dropping %s", event.get("event_type"))
            return False

    async def run(self, stop: asyncio.Event):
        while not stop.is_set():
            try:
                ev = await asyncio.wait_for(self.q.get(), 1.0)
            except asyncio.TimeoutError:
                continue
            for goal in self.st.events.publish(ev):
                if has_similar_active_goal(self.st, goal["description"]):
                    continue  # the same incident already has an open goal
                g = await self.st.submit_goal(goal["description"], int(goal["priority"]),
                                              f"event_bus:{ev.get('event_type', '')}")
                log.info("event %s -> goal %s", ev.get("event_type"), g["id"])


async def maintenance_loop(st: OrchestratorState, stop: asyncio.Event, interval: float = 15.0):
    while not await _sleep(stop, interval):
        n = st.cluster.prune() if st.cluster_enabled else 0
        m = st.discovery.prune()
        if n or m:
            log.info("pruned %d dead nodes, %d stale services", n, m)


# ---------------------------------------------------------------------------------- agent spawner
@dataclass
class AgentSpec:
    name: str
    agent_type: str
    module: str
    namespaces: List[str]
    enabled: bool = True


def load_agent_configs(config_dir: str = "/etc/aios/agents") -> List[AgentSpec]:
    """agent_spawner.rs:64-176: one TOML per agent; namespaces are the deduplicated prefixes of
    [capabilities].tools; defaults system / network / security when the directory is empty."""
    specs: List[AgentSpec] = []
    try:
        import tomli
    except ImportError:  # pragma: no cover
        tomli = None
    if tomli is not None and os.path.isdir(config_dir):
        for fn in sorted(os.listdir(config_dir)):
            if not fn.endswith(".toml"):
                continue
            try:
                with open(os.path.join(config_dir, fn), "rb") as f:
                    cfg = tomli.load(f)
            except Exception as e:
                log.warning("bad agent config %s: %s", fn, e)
                continue
            a = cfg.get("agent", cfg)
            atype = a.get("type", a.get("agent_type", fn[:-5]))
            tools = cfg.get("capabilities", {}).get("tools", [])
            ns = list(dict.fromkeys(t.split(".")[0] for t in tools))
            specs.append(AgentSpec(a.get("name", f"{atype}-agent"), atype, f"aios_amd.agents.{atype}", ns,
                                   bool(a.get("enabled", True))))
    if not specs:
        specs = [AgentSpec("system-agent", "system", "aios_amd.agents.system", ["monitor", "service", "process"]),
                 AgentSpec("network-agent", "network", "aios_amd.agents.network", ["net", "firewall"]),
                 AgentSpec("security-agent", "security", "aios_amd.agents.security", ["sec", "monitor"])]
    return [s for s in specs if s.enabled]


class AgentSpawner:
    MAX_RESTARTS = 5
    RESTART_DELAY = 5.0
    MONITOR_INTERVAL = 5.0

    def __init__(self, specs: List[AgentSpec], orchestrator_addr: str, python: str = ""):
        self.specs = specs
        self.addr = orchestrator_addr
        self.python = python or os.environ.get("AIOS_PYTHON", sys.executable)
        self.procs: Dict[str, subprocess.Popen] = {}
        self.restarts: Dict[str, int] = {}

    def spawn(self, s: AgentSpec):
        env = dict(os.environ, AIOS_AGENT_NAME=s.name, AIOS_AGENT_TYPE=s.agent_type,
                   AIOS_ORCHESTRATOR_ADDR=self.addr)
        self.procs[s.name] = subprocess.Popen([self.python, "-m", s.module], env=env)
        log.info("spawned agent %s (pid %d)", s.name, self.procs[s.name].pid)

    async def run(self, stop: asyncio.Event):
        for s in self.specs:
            self.spawn(s)
        while not await _sleep(stop, self.MONITOR_INTERVAL):
            for s in self.specs:
                p = self.procs.get(s.name)
                if p is None or p.poll() is None:
                    continue
                n = self.restarts.get(s.name, 0)
                if n >= self.MAX_RESTARTS:
                    continue
                log.warning("agent %s exited with %s; restarting (%d/%d)", s.name, p.returncode, n + 1,
                            self.MAX_RESTARTS)
                self.restarts[s.name] = n + 1
                if await _sleep(stop, self.RESTART_DELAY):
                    break
                self.spawn(s)
        self.stop_all()

    def stop_all(self):
        for p in self.procs.values():
            if p.poll() is None:
                p.terminate()
        for p in self.procs.values():
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                p.kill()

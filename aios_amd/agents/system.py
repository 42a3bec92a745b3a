"""SystemAgent: host health, services, processes (reference `aios_agent/agents/system.py:33-433`).

Health check = monitor.cpu / memory / disk in parallel with warn/crit thresholds (85/95 CPU,
80/95 memory, 85/95 disk), metrics pushed to memory, a 30 s background health loop that raises an
event when something is critical.  On MI355X hosts the check also reports per-GPU busy % and
VRAM from amdgpu sysfs (via hw.info).
"""
from __future__ import annotations

import re
from typing import Any, Dict

from .base import BaseAgent, IntelligenceLevel, main_for

CPU_WARN, CPU_CRIT = 85.0, 95.0
MEM_WARN, MEM_CRIT = 80.0, 95.0
DISK_WARN, DISK_CRIT = 85.0, 95.0
HEALTH_CHECK_INTERVAL_S = 30.0


def _level(v: float, warn: float, crit: float) -> str:
    return "critical" if v >= crit else "warning" if v >= warn else "ok"


def service_name(text: str) -> str:
    """'restart service nginx' / 'restart nginx' / 'status of sshd' -> the unit name"""
    m = re.search(r"(?:restart|start|stop|status of|service)\s+(?:the\s+)?(?:service\s+)?([a-zA-Z0-9_.@-]+)", text)
    return m.group(1) if m else ""


class SystemAgent(BaseAgent):
    AGENT_TYPE = "system"
    CAPABILITIES = ("system.health_check", "monitor.cpu", "monitor.memory", "monitor.disk", "system.restart_service",
                    "service.status", "service.list", "process.list", "system.uptime", "hw.info")
    ACTIONS = ((("health", "check system", "diagnos"), "check_health"),
               (("restart",), "restart_service"),
               (("service status", "status of", "is running"), "service_status"),
               (("services",), "list_services"),
               (("process", "top "), "list_processes"),
               (("uptime",), "uptime"),
               (("metric", "cpu", "memory", "ram", "disk"), "metrics"))

    async def check_health(self, task: Dict[str, Any]) -> Dict[str, Any]:
        cpu, mem, disk = await self.call_tools([("monitor.cpu", {}), ("monitor.memory", {}),
                                                ("monitor.disk", {"path": "/"})])
        c = float(cpu.get("output", {}).get("percent", 0.0)) if cpu["success"] else 0.0
        m = float(mem.get("output", {}).get("percent", 0.0)) if mem["success"] else 0.0
        dout = disk.get("output", {}) if disk["success"] else {}
        parts = dout.get("disks") or dout.get("partitions") or [dout]
        d = max((float(p.get("percent", p.get("usage_percent", 0.0)) or 0.0) for p in parts), default=0.0)
        status = {"cpu": _level(c, CPU_WARN, CPU_CRIT), "memory": _level(m, MEM_WARN, MEM_CRIT),
                  "disk": _level(d, DISK_WARN, DISK_CRIT)}
        overall = "critical" if "critical" in status.values() else "warning" if "warning" in status.values() else "ok"
        hw = await self.call_tool("hw.info", {})
        gpus = hw.get("output", {}).get("amd_gpu_agents", []) if hw["success"] else []
        for k, v in (("system.cpu_percent", c), ("system.memory_percent", m), ("system.disk_percent", d)):
            try:
                await self.update_metric(k, v)
            except Exception:
                pass
        recommended: list = []
        if overall == "critical":
            try:
                await self.push_event("system.health_critical", {"status": status, "cpu": c, "memory": m, "disk": d},
                                      critical=True)
            except Exception:
                pass
            # the model proposes the immediate remediation (reference system.py:174, tactical)
            failed = [k for k, v in status.items() if v != "ok"]
            recommended = self.advice_lines(await self.analyze(
                f"System health is CRITICAL. Issues: {failed}. Current metrics: CPU={c:.1f}%, MEM={m:.1f}%, "
                f"DISK={d:.1f}%. What immediate actions should I take? List up to 3 actions, one per line.",
                IntelligenceLevel.TACTICAL), 3)
        return {"success": True, "overall": overall, "status": status, "cpu_percent": c, "memory_percent": m,
                "disk_percent": d, "gpus": gpus, "recommended_actions": recommended}

    async def restart_service(self, task: Dict[str, Any]) -> Dict[str, Any]:
        name = task.get("input", {}).get("service") or service_name(task.get("description", ""))
        if not name:
            return {"success": False, "error": "no service name in task"}
        pre = await self.call_tool("service.status", {"name": name}, reason=f"pre-restart status of {name}")
        previous = str(pre.get("output", {}).get("status", "unknown")) if pre.get("success") else "unknown"
        if previous in ("running", "active"):
            # a running service is restarted only if the model judges it safe (reference system.py:238)
            verdict = await self.safety_check(
                f"Service '{name}' is currently running (status: {previous}). Should I restart it? Consider: is it "
                "a critical service? What are the risks? Answer YES or NO with a brief reason.",
                IntelligenceLevel.OPERATIONAL)
            if verdict is None:
                return self.safety_unavailable(f"restarting the running service {name}", service=name,
                                               previous_status=previous)
            if verdict.lower().lstrip(" *\"'").startswith("no"):
                return {"success": False, "service": name, "action": "restart_skipped", "reason": verdict,
                        "previous_status": previous}
        r = await self.call_tool("service.restart", {"name": name}, reason=f"restart {name} (was: {previous})")
        if not r["success"]:
            return r
        st = await self.call_tool("service.status", {"name": name})
        return {"success": True, "service": name, "status": st.get("output", {})}

    async def service_status(self, task: Dict[str, Any]) -> Dict[str, Any]:
        name = task.get("input", {}).get("service") or service_name(task.get("description", ""))
        return await self.call_tool("service.status", {"name": name})

    async def list_services(self, task: Dict[str, Any]) -> Dict[str, Any]:
        return await self.call_tool("service.list", {})

    async def list_processes(self, task: Dict[str, Any]) -> Dict[str, Any]:
        r = await self.call_tool("process.list", {})
        if r["success"]:
            procs = sorted(r["output"].get("processes", []), key=lambda p: -float(p.get("cpu", 0)))
            r["output"]["top"] = procs[:10]
        return r

    async def uptime(self, task: Dict[str, Any]) -> Dict[str, Any]:
        try:
            with open("/proc/uptime") as f:
                up = float(f.read().split()[0])
        except OSError:
            up = 0.0
        return {"success": True, "uptime_seconds": int(up), "agent_uptime_seconds": self.uptime_seconds()}

    async def metrics(self, task: Dict[str, Any]) -> Dict[str, Any]:
        return await self.check_health(task)

    async def fallback(self, task: Dict[str, Any]) -> Dict[str, Any]:
        r = await super().fallback(task)
        if r.get("success", True):
            return r
        analysis = await self.think_json(f"As the system agent, analyse: {task.get('description')}. JSON: "
                                         "{\"analysis\": \"...\", \"recommended_tools\": []}",
                                         IntelligenceLevel.TACTICAL)
        return {"success": analysis is not None, "analysis": analysis} if analysis else r

    async def background(self):
        return [self.periodic(HEALTH_CHECK_INTERVAL_S, lambda: self.check_health({}))]


if __name__ == "__main__":
    main_for(SystemAgent)

"""MonitoringAgent: metric collection, reports, threshold alerts, anomaly detection (rolling
z-score), resource forecast, dashboard data (reference `aios_agent/agents/monitoring.py:30-582`;
30 s collection loop, 60 s alert / anomaly loop, 100-sample baseline).  GPU busy % and VRAM are
collected alongside CPU / memory / disk / network."""
from __future__ import annotations

import math
import time
from collections import defaultdict, deque
from typing import Any, Deque, Dict, List

from .base import BaseAgent, main_for

METRIC_COLLECTION_INTERVAL_S = 30.0
ANOMALY_CHECK_INTERVAL_S = 60.0
BASELINE_WINDOW_SIZE = 100
ALERT_RULES = (
    ("cpu.usage_percent", 90, "critical", "cpu_critical"), ("cpu.usage_percent", 80, "warning", "cpu_warning"),
    ("memory.usage_percent", 95, "critical", "memory_critical"),
    ("memory.usage_percent", 85, "warning", "memory_warning"),
    ("disk.usage_percent", 95, "critical", "disk_critical"), ("disk.usage_percent", 85, "warning", "disk_warning"),
    ("gpu.busy_percent", 99, "warning", "gpu_saturated"),
)


class MonitoringAgent(BaseAgent):
    AGENT_TYPE = "monitoring"
    CAPABILITIES = ("monitoring.collect_metrics", "monitoring.generate_report", "monitoring.check_alerts",
                    "monitoring.anomaly_detection", "monitoring.resource_forecast", "monitoring.dashboard_data",
                    "monitor.cpu", "monitor.memory", "monitor.disk", "monitor.network", "hw.info")
    ACTIONS = ((("report", "summary"), "generate_report"),
               (("alert",), "check_alerts"),
               (("anomal", "unusual"), "anomaly_detection"),
               (("forecast", "predict", "trend"), "resource_forecast"),
               (("dashboard",), "dashboard_data"),
               (("metric", "collect", "monitor"), "collect_metrics"))

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.history: Dict[str, Deque] = defaultdict(lambda: deque(maxlen=BASELINE_WINDOW_SIZE))
        self.active_alerts: Dict[str, Dict[str, Any]] = {}

    async def collect_metrics(self, task: Dict[str, Any]) -> Dict[str, Any]:
        cpu, mem, disk, net, hw = await self.call_tools([("monitor.cpu", {}), ("monitor.memory", {}),
                                                         ("monitor.disk", {"path": "/"}), ("monitor.network", {}),
                                                         ("hw.info", {})])
        now = time.time()
        m = {"cpu.usage_percent": cpu.get("output", {}).get("percent"),
             "memory.usage_percent": mem.get("output", {}).get("percent"),
             "disk.usage_percent": disk.get("output", {}).get("percent"),
             "network.rx_bytes": net.get("output", {}).get("rx_bytes"),
             "network.tx_bytes": net.get("output", {}).get("tx_bytes")}
        gpus = hw.get("output", {}).get("amd_gpu_agents", []) if hw["success"] else []
        busy = [float(g.get("busy_percent", 0)) for g in gpus if isinstance(g, dict) and "busy_percent" in g]
        if busy:
            m["gpu.busy_percent"] = sum(busy) / len(busy)
        m = {k: float(v) for k, v in m.items() if v is not None}
        for k, v in m.items():
            self.history[k].append((now, v))
            try:
                await self.update_metric(k, v)
            except Exception:
                pass
        return {"success": True, "metrics": m, "timestamp": int(now)}

    def _stats(self, key: str):
        xs = [v for _, v in self.history[key]]
        if not xs:
            return None
        mu = sum(xs) / len(xs)
        sd = math.sqrt(sum((x - mu) ** 2 for x in xs) / len(xs))
        return {"mean": mu, "std": sd, "min": min(xs), "max": max(xs), "last": xs[-1], "n": len(xs)}

    async def generate_report(self, task: Dict[str, Any]) -> Dict[str, Any]:
        if not self.history:
            await self.collect_metrics(task)
        return {"success": True, "report": {k: self._stats(k) for k in list(self.history)},
                "active_alerts": list(self.active_alerts.values())}

    async def check_alerts(self, task: Dict[str, Any]) -> Dict[str, Any]:
        cur = (await self.collect_metrics(task))["metrics"]
        fired: Dict[str, Dict[str, Any]] = {}
        for metric, thr, sev, name in ALERT_RULES:
            v = cur.get(metric)
            if v is not None and v > thr and not any(a["metric"] == metric and a["severity"] == "critical"
                                                     for a in fired.values()):
                fired[name] = {"name": name, "metric": metric, "value": v, "threshold": thr, "severity": sev}
        new = [a for n, a in fired.items() if n not in self.active_alerts]
        resolved = [a for n, a in self.active_alerts.items() if n not in fired]
        self.active_alerts = fired
        try:
            if new:
                await self.push_event("monitoring.alerts_triggered", {"alerts": new},
                                      critical=any(a["severity"] == "critical" for a in new))
            if resolved:
                await self.push_event("monitoring.alerts_resolved", {"alerts": resolved})
        except Exception:
            pass
        return {"success": True, "active": list(fired.values()), "new": new, "resolved": resolved}

    async def anomaly_detection(self, task: Dict[str, Any]) -> Dict[str, Any]:
        anomalies: List[Dict[str, Any]] = []
        for k in list(self.history):
            s = self._stats(k)
            if s and s["n"] >= 10 and s["std"] > 0:
                z = (s["last"] - s["mean"]) / s["std"]
                if abs(z) >= 3.0:
                    anomalies.append({"metric": k, "value": s["last"], "mean": s["mean"], "z": z})
        if anomalies:
            try:
                await self.push_event("monitoring.anomalies_detected", {"anomalies": anomalies})
            except Exception:
                pass
        return {"success": True, "anomalies": anomalies}

    async def resource_forecast(self, task: Dict[str, Any]) -> Dict[str, Any]:
        out = {}
        for k in ("cpu.usage_percent", "memory.usage_percent", "disk.usage_percent"):
            pts = list(self.history[k])
            if len(pts) < 3:
                continue
            t0 = pts[0][0]
            xs, ys = [p[0] - t0 for p in pts], [p[1] for p in pts]
            mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
            den = sum((x - mx) ** 2 for x in xs) or 1.0
            slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / den  # %/s
            out[k] = {"slope_per_hour": slope * 3600, "forecast_1h": ys[-1] + slope * 3600,
                      "hours_to_100": (100 - ys[-1]) / (slope * 3600) if slope > 0 else None}
        return {"success": True, "forecast": out}

    async def dashboard_data(self, task: Dict[str, Any]) -> Dict[str, Any]:
        return {"success": True, "series": {k: list(v)[-30:] for k, v in self.history.items()},
                "alerts": list(self.active_alerts.values())}

    async def background(self):
        async def alerts_and_anomalies():
            await self.check_alerts({})
            await self.anomaly_detection({})
        return [self.periodic(METRIC_COLLECTION_INTERVAL_S, lambda: self.collect_metrics({})),
                self.periodic(ANOMALY_CHECK_INTERVAL_S, alerts_and_anomalies)]


if __name__ == "__main__":
    main_for(MonitoringAgent)

"""MonitoringAgent: metric collection, reports, threshold alerts, anomaly detection (rolling
z-score), resource forecast, dashboard data (reference `aios_agent/agents/monitoring.py:30-582`;
30 s collection loop, 60 s alert / anomaly loop, 100-sample baseline).  GPU busy % and VRAM are
collected alongside CPU / memory / disk / network."""
from __future__ import annotations

import math
import time
from collections import defaultdict, deque
from typing import Any, Deque, Dict, List

from .base import BaseAgent, IntelligenceLevel, main_for

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
        report = {k: self._stats(k) for k in list(self.history)}
        kind = (task.get("input") or {}).get("report_type", "daily")
        # executive summary of health and trends (reference monitoring.py:229)
        summary = await self.analyze(
            f"Generate a {kind} report summary.\n\nCurrent metrics (mean -> last over the window):\n" +
            "\n".join(f"  {k}: {v['mean']:.1f} -> {v['last']:.1f} (min {v['min']:.1f}, max {v['max']:.1f})"
                      for k, v in sorted(report.items()) if v) +
            f"\n\nActive alerts: {len(self.active_alerts)}\n\nProvide a 3-5 sentence executive summary covering "
            "system health, notable trends and recommended actions.", IntelligenceLevel.OPERATIONAL)
        return {"success": True, "report": report, "summary": summary,
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
        analysis = ""
        if anomalies:
            # are they concerning, likely causes, actions (reference monitoring.py:377)
            analysis = await self.analyze(
                f"Anomaly detection found {len(anomalies)} anomalies:\n" +
                "\n".join(f"- {a['metric']}: {a['value']:.2f} ({'above' if a['z'] > 0 else 'below'} baseline "
                          f"{a['mean']:.2f}, z={a['z']:.1f})" for a in anomalies) +
                "\n\nAre these anomalies concerning? What might cause them? Provide brief analysis and "
                "recommended actions.", IntelligenceLevel.TACTICAL)
            try:
                await self.push_event("monitoring.anomalies_detected", {"anomalies": anomalies},
                                      critical=any(abs(a["z"]) > 4 for a in anomalies))
            except Exception:
                pass
        return {"success": True, "anomalies": anomalies, "analysis": analysis}

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
        summary = ""
        if out:
            # forecast summary + capacity planning advice (reference monitoring.py:468)
            summary = await self.analyze(
                "Resource forecast for the next hours:\n" +
                "\n".join(f"- {k}: projected in 1h={v['forecast_1h']:.1f}, trend={v['slope_per_hour']:.2f}/hr"
                          + (f" WARNING: capacity in {v['hours_to_100']:.1f}h"
                             if v["hours_to_100"] is not None and v["hours_to_100"] < 24 else "")
                          for k, v in out.items()) +
                "\n\nProvide a brief forecast summary with any capacity planning recommendations.",
                IntelligenceLevel.OPERATIONAL)
        return {"success": True, "forecast": out, "summary": summary}

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

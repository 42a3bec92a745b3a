"""LearningAgent: learns from the system's own history -- pattern analysis over recent events and
decisions, parameter optimisation from metric history, improvement suggestions, pattern store
updates, performance analysis, tool effectiveness (reference `aios_agent/agents/learning.py:
29-751`; 5 min learning cycle, ≥10 data points, 0.7 confidence to act; the cycle may propose goals).
"""
from __future__ import annotations

from collections import Counter, defaultdict
from typing import Any, Dict, List

from .base import BaseAgent, IntelligenceLevel, main_for
from .orchestrator_client import OrchestratorClient

LEARNING_CYCLE_INTERVAL_S = 300.0
MIN_DATA_POINTS = 10
IMPROVEMENT_CONFIDENCE_THRESHOLD = 0.7


class LearningAgent(BaseAgent):
    AGENT_TYPE = "learning"
    CAPABILITIES = ("learning.analyze_patterns", "learning.optimize_parameters", "learning.suggest_improvements",
                    "learning.update_patterns", "learning.performance_analysis", "learning.tool_effectiveness")
    ACTIONS = ((("tool effect", "tool usage"), "tool_effectiveness"),
               (("optimi", "tune", "parameter"), "optimize_parameters"),
               (("suggest", "improve"), "suggest_improvements"),
               (("update pattern", "learn"), "update_patterns"),
               (("performance",), "performance_analysis"),
               (("pattern", "analy"), "analyze_patterns"))

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.client = OrchestratorClient(self.config.orchestrator_addr)
        self.proposed: set = set()

    async def analyze_patterns(self, task: Dict[str, Any]) -> Dict[str, Any]:
        events = await self.get_recent_events(500)
        if len(events) < MIN_DATA_POINTS:
            return {"success": True, "patterns": [], "note": f"only {len(events)} events (need {MIN_DATA_POINTS})"}
        by_cat = Counter(e["category"] for e in events)
        crit = Counter(e["category"] for e in events if e["critical"])
        total = len(events)
        patterns = []
        for cat, n in by_cat.most_common(20):
            conf = min(1.0, n / total * 4) if total else 0.0
            patterns.append({"trigger": cat, "occurrences": n, "critical": crit.get(cat, 0), "confidence": conf})
        # which patterns are worth promoting to rules, which are anti-patterns (reference learning.py:181)
        analysis = await self.analyze(
            f"Pattern analysis over {total} recent events discovered {len(patterns)} patterns:\n" +
            "\n".join(f"- '{p['trigger']}' (n={p['occurrences']}, critical={p['critical']}, "
                      f"conf={p['confidence']:.2f})" for p in patterns[:15]) +
            "\n\nWhich patterns are most valuable for the system? Any patterns that should be promoted to "
            "automatic rules? Any concerning anti-patterns?", IntelligenceLevel.STRATEGIC) if patterns else ""
        return {"success": True, "patterns": patterns, "events_analyzed": total, "analysis": analysis}

    async def update_patterns(self, task: Dict[str, Any]) -> Dict[str, Any]:
        ana = await self.analyze_patterns(task)
        stored = 0
        for p in ana.get("patterns", []):
            if p["confidence"] >= IMPROVEMENT_CONFIDENCE_THRESHOLD and p["critical"]:
                await self.store_pattern(p["trigger"], f"investigate recurring {p['trigger']}", p["confidence"])
                stored += 1
        return {"success": True, "patterns_stored": stored}

    async def _metric_history(self) -> Dict[str, List[float]]:
        hist: Dict[str, List[float]] = defaultdict(list)
        for k in ("cpu.usage", "memory.used_mb", "disk.used_gb", "gpu.utilization", "system.cpu_percent",
                  "system.memory_percent", "system.disk_percent"):
            v = await self.get_metric(k)
            if v is not None:
                hist[k].append(v)
        past = (await self.recall_memory("metric_history")) or {}
        for k, vs in past.items():
            hist[k] = (list(vs) + hist.get(k, []))[-200:]
        await self.store_memory("metric_history", dict(hist))
        return hist

    async def optimize_parameters(self, task: Dict[str, Any]) -> Dict[str, Any]:
        hist = await self._metric_history()
        recs = []
        for k, vs in hist.items():
            if len(vs) < MIN_DATA_POINTS:
                continue
            avg, peak = sum(vs) / len(vs), max(vs)
            if "percent" in k or k in ("cpu.usage", "gpu.utilization"):
                if avg > 80:
                    recs.append({"metric": k, "avg": avg, "suggestion": "sustained high load: scale out or throttle"})
                elif peak < 20:
                    recs.append({"metric": k, "avg": avg, "suggestion": "resource mostly idle: consolidate work"})
        # the model's parameter changes from the same data (reference learning.py:268)
        perf = {k: {"current": vs[-1], "mean": sum(vs) / len(vs), "min": min(vs), "max": max(vs)}
                for k, vs in hist.items() if vs}
        suggestions = []
        if perf:
            sug = await self.think_json(
                "System parameter optimization analysis.\n\nPerformance data:\n" +
                "\n".join(f"- {k}: current={v['current']:.1f}, mean={v['mean']:.1f}, "
                          f"range=[{v['min']:.1f}, {v['max']:.1f}]" for k, v in perf.items()) +
                "\n\nSuggest specific parameter changes to improve performance. JSON: {\"suggestions\": "
                "[{\"parameter\": \"...\", \"current\": \"...\", \"suggested\": \"...\", \"impact\": \"...\"}]}",
                IntelligenceLevel.STRATEGIC)
            if isinstance(sug, dict) and isinstance(sug.get("suggestions"), list):
                suggestions = [x for x in sug["suggestions"] if isinstance(x, dict)][:10]
            elif isinstance(sug, list):
                suggestions = [x for x in sug if isinstance(x, dict)][:10]
        return {"success": True, "recommendations": recs, "ai_suggestions": suggestions,
                "metrics_considered": len(hist)}

    async def tool_effectiveness(self, task: Dict[str, Any]) -> Dict[str, Any]:
        events = await self.get_recent_events(500)
        stats: Dict[str, Counter] = defaultdict(Counter)
        for e in events:
            tool = e["data"].get("tool") if isinstance(e["data"], dict) else None
            if tool:
                stats[tool]["ok" if e["data"].get("success", True) else "fail"] += 1
        report = {t: {"calls": c["ok"] + c["fail"], "success_rate": c["ok"] / max(c["ok"] + c["fail"], 1)}
                  for t, c in stats.items()}
        return {"success": True, "tools": report}

    async def performance_analysis(self, task: Dict[str, Any]) -> Dict[str, Any]:
        status = await self.client.get_system_status()
        goals = await self.client.list_goals(limit=200)
        st = Counter(g["status"] for g in goals["goals"])
        done = st.get("completed", 0) + st.get("failed", 0)
        return {"success": True, "system": status, "goal_status": dict(st),
                "goal_success_rate": st.get("completed", 0) / done if done else None}

    async def suggest_improvements(self, task: Dict[str, Any]) -> Dict[str, Any]:
        perf = await self.performance_analysis(task)
        opt = await self.optimize_parameters(task)
        ana = await self.analyze_patterns(task)
        ideas = await self.think_json(
            f"System performance: {perf['goal_status']}, success rate {perf['goal_success_rate']}; "
            f"recommendations {opt['recommendations'][:5]}; frequent events {ana.get('patterns', [])[:5]}. "
            "Propose improvements. JSON: {\"improvements\": [{\"goal\": \"...\", \"confidence\": 0.0-1.0}]}",
            IntelligenceLevel.STRATEGIC)
        items = ideas.get("improvements", []) if isinstance(ideas, dict) else []
        for r in opt["recommendations"]:
            items.append({"goal": f"{r['suggestion']} ({r['metric']} avg {r['avg']:.0f})", "confidence": 0.75})
        return {"success": True, "improvements": items}

    async def learning_cycle(self):
        await self.update_patterns({})
        sug = await self.suggest_improvements({})
        for it in sug["improvements"]:
            goal = str(it.get("goal", "")).strip()
            if goal and float(it.get("confidence", 0)) >= IMPROVEMENT_CONFIDENCE_THRESHOLD and goal not in self.proposed:
                self.proposed.add(goal)
                await self.client.submit_goal(goal, priority=7, source="learning-agent")

    async def background(self):
        return [self.periodic(LEARNING_CYCLE_INTERVAL_S, self.learning_cycle)]


if __name__ == "__main__":
    main_for(LearningAgent)

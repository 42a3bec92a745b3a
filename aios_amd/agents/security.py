"""SecurityAgent: vulnerability scan, integrity, permissions, audit log review, intrusion checks,
threat analysis (reference `aios_agent/agents/security.py:29-600`; 45 s IDS loop, 120 s audit
loop, severity weights critical 10 / high 7 / medium 4 / low 1)."""
from __future__ import annotations

from typing import Any, Dict, List

from .base import BaseAgent, IntelligenceLevel, main_for

IDS_CHECK_INTERVAL_S = 45.0
AUDIT_CHECK_INTERVAL_S = 120.0
SEVERITY_WEIGHTS = {"critical": 10, "high": 7, "medium": 4, "low": 1, "info": 0}
SENSITIVE_PATHS = ("/etc/passwd", "/etc/shadow", "/etc/sudoers", "/etc/ssh/sshd_config")
SUSPICIOUS_PROCS = ("nc", "ncat", "socat", "cryptominer", "xmrig", "minerd")
EXPECTED_PORTS = {22, 80, 443, 9090, 50051, 50052, 50053, 50054, 50055, 8082}


def risk_score(findings: List[Dict[str, Any]]) -> int:
    return min(100, sum(SEVERITY_WEIGHTS.get(str(f.get("severity", "info")).lower(), 0) for f in findings))


class SecurityAgent(BaseAgent):
    AGENT_TYPE = "security"
    CAPABILITIES = ("sec.scan", "sec.check_perms", "sec.file_integrity", "sec.scan_rootkits", "sec.audit",
                    "sec.audit_query", "monitor.logs", "net.port_scan", "process.list")
    ACTIONS = ((("vulnerab", "security scan", "scan"), "scan_vulnerabilities"),
               (("integrity", "tamper", "checksum"), "check_integrity"),
               (("permission", "perms", "chmod"), "check_permissions"),
               (("audit", "log review"), "audit_logs"),
               (("intrusion", "breach", "rootkit"), "intrusion_check"),
               (("threat", "analy"), "threat_analysis"))

    async def scan_vulnerabilities(self, task: Dict[str, Any]) -> Dict[str, Any]:
        scan = await self.call_tool("sec.scan", {})
        perms = await self.call_tools([("sec.check_perms", {"path": p}) for p in SENSITIVE_PATHS])
        findings = list(scan.get("output", {}).get("findings", [])) if scan["success"] else []
        for p, r in zip(SENSITIVE_PATHS, perms):
            if r["success"] and r["output"].get("writable_by_others"):
                findings.append({"severity": "high", "issue": f"{p} is world-writable"})
        score = risk_score(findings)
        # the model's remediation plan for the critical / high findings (reference security.py:175)
        severe = [f for f in findings if str(f.get("severity", "")).lower() in ("critical", "high")]
        recommendations: List[str] = []
        if severe:
            recommendations = self.advice_lines(await self.analyze(
                f"Security scan found {len(severe)} critical/high issues:\n" +
                "\n".join(f"- [{f.get('severity')}] {str(f.get('issue', f.get('description', '')))[:100]}"
                          for f in severe[:10]) +
                "\n\nProvide prioritised remediation steps (one per line, max 5).", IntelligenceLevel.TACTICAL))
        try:
            await self.push_event("security.scan_complete", {"findings": len(findings), "risk_score": score},
                                  critical=score >= 50)
        except Exception:
            pass
        return {"success": True, "findings": findings, "risk_score": score, "recommendations": recommendations}

    async def check_integrity(self, task: Dict[str, Any]) -> Dict[str, Any]:
        mode = task.get("input", {}).get("mode", "check")
        r = await self.call_tool("sec.file_integrity", {"mode": mode, "paths": list(SENSITIVE_PATHS)})
        changed = r.get("output", {}).get("changed", []) if r["success"] else []
        if changed:
            # is any change suspicious? (reference security.py:273)
            analysis = await self.analyze(
                f"File integrity check found {len(changed)} changes:\n" +
                "\n".join(f"- {c if isinstance(c, str) else c.get('path', c)}" for c in changed[:20]) +
                "\n\nAre any of these suspicious? Which need investigation? Reply with a brief risk assessment.",
                IntelligenceLevel.TACTICAL)
            try:
                await self.push_event("security.integrity_changes", {"changed": changed}, critical=True)
            except Exception:
                pass
            return {**r, "analysis": analysis}
        return {**r, "analysis": "No changes detected. All files match baseline."} if r["success"] else r

    async def check_permissions(self, task: Dict[str, Any]) -> Dict[str, Any]:
        path = task.get("input", {}).get("path")
        paths = [path] if path else list(SENSITIVE_PATHS)
        res = await self.call_tools([("sec.check_perms", {"path": p}) for p in paths])
        return {"success": True, "results": {p: r.get("output", r.get("error")) for p, r in zip(paths, res)}}

    async def audit_logs(self, task: Dict[str, Any]) -> Dict[str, Any]:
        logs = await self.call_tool("monitor.logs", {"lines": 200})
        entries = logs.get("output", {}).get("entries", []) if logs["success"] else []
        alerts = [e for e in entries if any(k in str(e).lower() for k in ("failed password", "authentication failure",
                                                                            "invalid user", "segfault", "denied"))]
        chain = await self.call_tool("sec.audit", {"limit": 50})
        analysis = ""
        if alerts:
            # security assessment of the suspicious entries (reference security.py:382)
            failed = sum("failed password" in str(e).lower() or "authentication failure" in str(e).lower()
                         for e in alerts)
            analysis = await self.analyze(
                f"Audit log analysis:\n- Total entries: {len(entries)}\n- Failed logins: {failed}\n"
                f"- Suspicious events: {len(alerts)}\n\nSample suspicious events:\n" +
                "\n".join(f"  - {str(e)[:150]}" for e in alerts[:5]) +
                "\n\nProvide a security assessment. Is immediate action needed?", IntelligenceLevel.TACTICAL)
            try:
                await self.push_event("security.audit_alerts", {"count": len(alerts), "sample": alerts[:5]})
            except Exception:
                pass
        return {"success": True, "alerts": alerts[:50], "alert_count": len(alerts), "analysis": analysis,
                "tool_audit": chain.get("output", {})}

    async def intrusion_check(self, task: Dict[str, Any]) -> Dict[str, Any]:
        procs, rk = await self.call_tools([("process.list", {}), ("sec.scan_rootkits", {})])
        ports = await self.call_tools([("net.port_scan", {"host": "127.0.0.1", "port": p})
                                       for p in (4444, 5555, 6667, 31337, 1337)])
        sus = [p for p in procs.get("output", {}).get("processes", []) if p.get("name") in SUSPICIOUS_PROCS]
        odd_ports = [p for p, r in zip((4444, 5555, 6667, 31337, 1337), ports)
                     if r["success"] and r.get("output", {}).get("open")]
        detected = bool(sus or odd_ports or (rk["success"] and rk["output"].get("suspicious")))
        analysis = "No threats detected. System appears clean."
        if detected:
            # threat assessment and immediate actions (reference security.py:464)
            analysis = await self.analyze(
                f"IDS check results:\n- Suspicious processes: {sus[:10]}\n- Unexpected open ports: {odd_ports}\n"
                f"- Rootkit scan: {rk.get('output', rk.get('error'))}\n\n"
                "Assess the threat and recommend immediate actions.", IntelligenceLevel.TACTICAL)
            try:
                await self.push_event("security.intrusion_detected", {"processes": sus, "ports": odd_ports},
                                      critical=True)
            except Exception:
                pass
        return {"success": True, "intrusion_detected": detected, "analysis": analysis, "suspicious_processes": sus,
                "unexpected_open_ports": odd_ports, "rootkit_scan": rk.get("output", rk.get("error"))}

    async def threat_analysis(self, task: Dict[str, Any]) -> Dict[str, Any]:
        scan = await self.scan_vulnerabilities(task)
        intr = await self.intrusion_check(task)
        verdict = await self.think_json(
            f"Security findings: {scan['findings'][:20]}; intrusion: {intr['intrusion_detected']}. JSON: "
            "{\"threat_level\": \"low|medium|high|critical\", \"summary\": \"...\", \"actions\": []}",
            IntelligenceLevel.TACTICAL)
        return {"success": True, "risk_score": scan["risk_score"], "intrusion": intr["intrusion_detected"],
                "analysis": verdict}

    async def background(self):
        return [self.periodic(IDS_CHECK_INTERVAL_S, lambda: self.intrusion_check({})),
                self.periodic(AUDIT_CHECK_INTERVAL_S, lambda: self.audit_logs({}))]


if __name__ == "__main__":
    main_for(SecurityAgent)

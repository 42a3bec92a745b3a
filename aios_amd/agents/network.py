"""NetworkAgent: connectivity, DNS, interfaces, port scans, firewall (reference
`aios_agent/agents/network.py:28-419`; 60 s connectivity loop, ping targets 8.8.8.8 / 1.1.1.1 /
9.9.9.9, DNS test domains google.com / cloudflare.com)."""
from __future__ import annotations

import re
from typing import Any, Dict

from .base import BaseAgent, IntelligenceLevel, main_for

CONNECTIVITY_CHECK_INTERVAL_S = 60.0
PING_TARGETS = ("8.8.8.8", "1.1.1.1", "9.9.9.9")
DNS_TEST_DOMAINS = ("google.com", "cloudflare.com")
_HOST = re.compile(r"\b((?:\d{1,3}\.){3}\d{1,3}|(?:[a-z0-9-]+\.)+[a-z]{2,})\b", re.I)


def host_in(text: str, default: str = "") -> str:
    m = _HOST.search(text)
    return m.group(1) if m else default


class NetworkAgent(BaseAgent):
    AGENT_TYPE = "network"
    CAPABILITIES = ("net.interfaces", "net.ping", "net.dns", "net.port_scan", "net.http_get", "firewall.rules",
                    "firewall.add_rule", "firewall.delete_rule")
    ACTIONS = ((("diagnos", "troubleshoot"), "diagnose"),
               (("connectivity", "internet", "online"), "check_connectivity"),
               (("dns", "resolve", "lookup"), "dns_lookup"),
               (("interface", "ip address", "nic"), "list_interfaces"),
               (("port scan", "open port", "ports"), "port_scan"),
               (("firewall", "nft", "iptables"), "manage_firewall"),
               (("ping",), "ping"))

    async def ping(self, task: Dict[str, Any]) -> Dict[str, Any]:
        host = task.get("input", {}).get("host") or host_in(task.get("description", ""), "1.1.1.1")
        return await self.call_tool("net.ping", {"host": host, "count": 3})

    async def check_connectivity(self, task: Dict[str, Any]) -> Dict[str, Any]:
        pings = await self.call_tools([("net.ping", {"host": h, "count": 1}) for h in PING_TARGETS])
        dns = await self.call_tools([("net.dns", {"hostname": d, "host": d}) for d in DNS_TEST_DOMAINS])
        ping_ok = sum(1 for p in pings if p["success"] and p.get("output", {}).get("reachable", True))
        dns_ok = sum(1 for d in dns if d["success"])
        healthy = ping_ok > 0 and dns_ok > 0
        try:
            await self.update_metric("network.connectivity_healthy", 1.0 if healthy else 0.0)
            if not healthy:
                await self.push_event("network.connectivity_issue", {"ping_ok": ping_ok, "dns_ok": dns_ok},
                                      critical=True)
        except Exception:
            pass
        return {"success": True, "healthy": healthy, "ping_reachable": ping_ok, "ping_targets": len(PING_TARGETS),
                "dns_resolved": dns_ok, "dns_domains": len(DNS_TEST_DOMAINS)}

    async def dns_lookup(self, task: Dict[str, Any]) -> Dict[str, Any]:
        h = task.get("input", {}).get("hostname") or host_in(task.get("description", ""), "localhost")
        return await self.call_tool("net.dns", {"hostname": h, "host": h})

    async def list_interfaces(self, task: Dict[str, Any]) -> Dict[str, Any]:
        return await self.call_tool("net.interfaces", {})

    async def port_scan(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp = task.get("input", {})
        host = inp.get("host") or host_in(task.get("description", ""), "127.0.0.1")
        ports = inp.get("ports") or [22, 80, 443, 9090, 50051, 50052, 50053, 50054, 50055]
        res = await self.call_tools([("net.port_scan", {"host": host, "port": int(p)}) for p in ports])
        open_ports = [p for p, r in zip(ports, res) if r["success"] and r.get("output", {}).get("open")]
        return {"success": True, "host": host, "open_ports": open_ports, "scanned": len(ports)}

    async def diagnose(self, task: Dict[str, Any]) -> Dict[str, Any]:
        target = host_in(task.get("description", ""), "1.1.1.1")
        ping, dns, ifs = await self.call_tools([("net.ping", {"host": target, "count": 3}),
                                                ("net.dns", {"hostname": "google.com", "host": "google.com"}),
                                                ("net.interfaces", {})])
        findings = {"ping": ping.get("output", ping.get("error")), "dns": dns.get("output", dns.get("error")),
                    "interfaces_up": [i["name"] for i in ifs.get("output", {}).get("interfaces", [])
                                      if i.get("status") == "up"]}
        advice = await self.think_json(f"Network diagnosis data: {findings}. JSON: {{\"problem\": \"...\", "
                                       "\"likely_cause\": \"...\", \"fix\": \"...\"}}", IntelligenceLevel.OPERATIONAL)
        return {"success": True, "findings": findings, "analysis": advice}

    async def manage_firewall(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp, d = task.get("input", {}), task.get("description", "").lower()
        if inp.get("rule") or "add" in d or "allow" in d or "block" in d:
            rule = inp.get("rule")
            if not rule:
                m = re.search(r"port\s+(\d+)", d)
                if not m:
                    return {"success": False, "error": "no rule / port in task"}
                rule = f"tcp dport {m.group(1)} {'drop' if 'block' in d else 'accept'}"
            # lock-out check by the model before the rule goes in (reference network.py:329)
            safety = await self.safety_check(f"A firewall rule is being added: {rule}. Is this safe? Could it lock "
                                             "us out of the system? Answer YES or NO.", IntelligenceLevel.OPERATIONAL)
            if safety is None:
                return self.safety_unavailable("adding the firewall rule", rule=rule)
            if safety.lower().lstrip(" *\"'").startswith("no"):
                return {"success": False, "error": f"Firewall rule rejected by safety check: {safety}", "rule": rule}
            return await self.call_tool("firewall.add_rule", {"chain": inp.get("chain", "input"), "rule": rule})
        if "delete" in d or "remove" in d:
            return await self.call_tool("firewall.delete_rule", {"chain": inp.get("chain", "input"),
                                                                 "index": int(inp.get("index", 0))})
        return await self.call_tool("firewall.rules", {})

    async def background(self):
        return [self.periodic(CONNECTIVITY_CHECK_INTERVAL_S, lambda: self.check_connectivity({}))]


if __name__ == "__main__":
    main_for(NetworkAgent)

"""PackageAgent: install / remove / update / search / info / list / vulnerability check
(reference `aios_agent/agents/package.py:24-553`).  The reference called a non-existent
`package.cve_check` tool (App. A); here the vulnerability check uses `sec.scan` findings and the
package list."""
from __future__ import annotations

import re
from typing import Any, Dict

from .base import BaseAgent, IntelligenceLevel, main_for

_PKG = re.compile(r"(?:install|remove|uninstall|purge|search(?: for)?|info(?:rmation)? (?:about|on)|package)\s+"
                  r"([a-z0-9][a-z0-9+._-]*)", re.I)


def package_name(text: str) -> str:
    m = _PKG.search(text)
    return m.group(1) if m else ""


class PackageAgent(BaseAgent):
    AGENT_TYPE = "package"
    CAPABILITIES = ("pkg.install", "pkg.remove", "pkg.update", "pkg.search", "pkg.list_installed", "sec.scan")
    ACTIONS = ((("uninstall", "remove", "purge"), "remove_package"),
               (("list installed", "installed packages", "list packages"), "list_installed"),
               (("install",), "install_package"),
               (("upgrade", "update"), "update_all"),
               (("cve", "vulnerab"), "check_vulnerabilities"),
               (("search", "find package"), "search_packages"),
               (("info", "details"), "package_info"),
               (("installed", "list"), "list_installed"))

    def _name(self, task):
        return task.get("input", {}).get("name") or package_name(task.get("description", ""))

    async def install_package(self, task: Dict[str, Any]) -> Dict[str, Any]:
        name = self._name(task)
        if not name:
            return {"success": False, "error": "no package name in task"}
        found, scan = await self.call_tools([("pkg.search", {"query": name}), ("sec.scan", {})])
        if found["success"] and not found["output"].get("results", found["output"].get("packages", [1])):
            return {"success": False, "error": f"package {name} not found"}
        # known critical / high advisories for this package: ask before installing (reference
        # package.py:139); `force` skips the question
        cves = [f for f in (scan.get("output", {}).get("findings", []) if scan["success"] else [])
                if name in str(f.get("package", f.get("issue", ""))).lower()
                and str(f.get("severity", "")).lower() in ("critical", "high")]
        if cves and not (task.get("input") or {}).get("force"):
            decision = await self.safety_check(
                f"Package '{name}' has {len(cves)} critical/high advisories:\n" +
                "\n".join(f"- {c.get('cve', 'N/A')}: {str(c.get('description', c.get('issue', '')))[:100]}"
                          for c in cves[:5]) +
                "\n\nShould I still install it? Consider the risk vs. necessity. Answer INSTALL or SKIP with "
                "brief reason.", IntelligenceLevel.TACTICAL)
            if decision is None:
                return self.safety_unavailable(f"installing {name}", advisories=cves)
            if "skip" in decision.lower()[:10]:
                return {"success": False, "error": f"skipped {name}: {decision}", "advisories": cves}
        r = await self.call_tool("pkg.install", {"name": name}, reason=f"install {name}")
        try:
            await self.push_event("package.installed" if r["success"] else "package.install_failed", {"name": name})
        except Exception:
            pass
        return r

    async def remove_package(self, task: Dict[str, Any]) -> Dict[str, Any]:
        name = self._name(task)
        if not name:
            return {"success": False, "error": "no package name in task"}
        if name in ("libc6", "systemd", "bash", "coreutils", "apt", "dpkg", "python3", "rocm-core"):
            return {"success": False, "error": f"refusing to remove essential package {name}"}
        # installed packages that name it as a dependency: ask whether removal is safe (reference
        # package.py:243); `force` skips the question
        inst = await self.call_tool("pkg.list_installed", {"filter": ""})
        dependents = [p.get("name") for p in (inst.get("output", {}).get("packages", []) if inst["success"] else [])
                      if isinstance(p, dict) and p.get("name") != name
                      and name in " ".join(map(str, p.get("depends", [])))][:10]
        if dependents and not (task.get("input") or {}).get("force"):
            check = await self.safety_check(
                f"Package '{name}' is required by: {dependents}. Is it safe to remove? Could it break the system? "
                "Answer REMOVE or KEEP with reason.", IntelligenceLevel.OPERATIONAL)
            if check is None:
                return self.safety_unavailable(f"removing {name}", dependents=dependents)
            if "keep" in check.lower()[:10]:
                return {"success": False, "error": f"kept {name}: {check}", "dependents": dependents}
        return await self.call_tool("pkg.remove", {"name": name}, reason=f"remove {name}")

    async def update_all(self, task: Dict[str, Any]) -> Dict[str, Any]:
        r = await self.call_tool("pkg.update", {}, reason="system update")
        try:
            await self.push_event("package.system_update", {"success": r["success"]})
        except Exception:
            pass
        return r

    async def check_vulnerabilities(self, task: Dict[str, Any]) -> Dict[str, Any]:
        scan, inst = await self.call_tools([("sec.scan", {}), ("pkg.list_installed", {})])
        findings = scan.get("output", {}).get("findings", []) if scan["success"] else []
        by_sev: Dict[str, list] = {"critical": [], "high": [], "medium": [], "low": []}
        for f in findings:
            by_sev.setdefault(str(f.get("severity", "low")).lower(), []).append(f)
        try:
            await self.update_metric("package.cve_total", float(len(findings)))
            await self.update_metric("package.cve_critical", float(len(by_sev["critical"])))
        except Exception:
            pass
        n_pkgs = len(inst.get("output", {}).get("packages", [])) if inst["success"] else 0
        recommendations = []
        if by_sev["critical"] or by_sev["high"]:
            # prioritised fixes (reference package.py:430)
            recommendations = self.advice_lines(await self.analyze(
                f"CVE scan results: {len(by_sev['critical'])} critical, {len(by_sev['high'])} high, "
                f"{len(by_sev['medium'])} medium, {len(by_sev['low'])} low vulnerabilities.\n\nCritical / high:\n" +
                "\n".join(f"- {v.get('cve', '')}: {v.get('package', '')} - "
                          f"{str(v.get('description', v.get('issue', '')))[:80]}"
                          for v in (by_sev["critical"] + by_sev["high"])[:5]) +
                "\n\nProvide prioritised fix recommendations (max 5, one per line).", IntelligenceLevel.TACTICAL))
        return {"success": True, "installed_packages": n_pkgs, "vulnerabilities": findings,
                "by_severity": {k: len(v) for k, v in by_sev.items()}, "recommendations": recommendations}

    async def search_packages(self, task: Dict[str, Any]) -> Dict[str, Any]:
        q = task.get("input", {}).get("query") or self._name(task) or task.get("description", "").split()[-1]
        return await self.call_tool("pkg.search", {"query": q})

    async def package_info(self, task: Dict[str, Any]) -> Dict[str, Any]:
        name = self._name(task)
        inst = await self.call_tool("pkg.list_installed", {"filter": name})
        found = await self.call_tool("pkg.search", {"query": name})
        return {"success": True, "name": name, "installed": inst.get("output", {}).get("packages", []),
                "available": found.get("output", {})}

    async def list_installed(self, task: Dict[str, Any]) -> Dict[str, Any]:
        return await self.call_tool("pkg.list_installed", {"filter": task.get("input", {}).get("filter", "")})

    async def fallback(self, task: Dict[str, Any]) -> Dict[str, Any]:
        plan = await self.think_json(f"Package management task: {task.get('description')}. JSON: {{\"action\": "
                                     "\"install|remove|update|search|list\", \"name\": \"...\"}",
                                     IntelligenceLevel.OPERATIONAL)
        if isinstance(plan, dict) and plan.get("action"):
            t = dict(task, input={**task.get("input", {}), "name": plan.get("name", "")})
            m = {"install": "install_package", "remove": "remove_package", "update": "update_all",
                 "search": "search_packages", "list": "list_installed"}.get(plan["action"])
            if m:
                return await getattr(self, m)(t)
        return {"success": False, "error": f"package agent cannot handle: {task.get('description')}"}


if __name__ == "__main__":
    main_for(PackageAgent)

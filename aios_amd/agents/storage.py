"""StorageAgent: disk health, backup / restore, mounts, fsck, capacity planning (reference
`aios_agent/agents/storage.py:28-637`; 5 min disk loop, warn 85 % / crit 95 %)."""
from __future__ import annotations

import os
import re
import time
from typing import Any, Dict

from .base import BaseAgent, IntelligenceLevel, main_for

DISK_CHECK_INTERVAL_S = 300.0
DISK_WARN, DISK_CRIT = 85.0, 95.0
BACKUP_ROOT = os.environ.get("AIOS_BACKUP_ROOT", "/var/lib/aios/backups")
_PATH = re.compile(r"(/[\w./-]+)")


class StorageAgent(BaseAgent):
    AGENT_TYPE = "storage"
    CAPABILITIES = ("monitor.disk", "fs.list", "fs.stat", "fs.disk_usage", "fs.read", "fs.write", "fs.copy",
                    "fs.mkdir", "process.spawn")
    ACTIONS = ((("restore",), "restore_backup"),
               (("backup", "snapshot"), "create_backup"),
               (("mount",), "manage_mounts"),
               (("fsck", "filesystem check"), "fsck"),
               (("capacity", "forecast", "grow"), "capacity_planning"),
               (("disk", "storage", "space", "health"), "check_disk_health"))

    async def check_disk_health(self, task: Dict[str, Any]) -> Dict[str, Any]:
        path = (task.get("input") or {}).get("path", "/")
        r = await self.call_tool("monitor.disk", {"path": path})
        if not r["success"]:
            return r
        pct = float(r["output"].get("percent", 0.0))
        status = "critical" if pct >= DISK_CRIT else "warning" if pct >= DISK_WARN else "ok"
        warnings = []
        if status != "ok":
            # what to do about an unhealthy disk, is data at risk (reference storage.py:166)
            warnings = self.advice_lines(await self.analyze(
                f"Disk health check: {path} is {pct:.1f}% full ({status}); usage {r['output']}.\n"
                "What actions should be taken? Is data at risk?", IntelligenceLevel.TACTICAL), 8)
        try:
            await self.update_metric("storage.disk_percent", pct)
            if status != "ok":
                await self.push_event("storage.disk_unhealthy", {"path": path, "percent": pct, "status": status},
                                      critical=status == "critical")
        except Exception:
            pass
        return {"success": True, "path": path, "percent": pct, "status": status, "usage": r["output"],
                "warnings": warnings}

    async def create_backup(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp = task.get("input") or {}
        src = inp.get("source") or (_PATH.findall(task.get("description", "")) or ["/etc/aios"])[0]
        dst = inp.get("destination") or os.path.join(BACKUP_ROOT, time.strftime("%Y%m%d-%H%M%S"),
                                                     os.path.basename(src.rstrip("/")) or "root")
        du_src = await self.call_tool("fs.disk_usage", {"path": src})
        du_dst = await self.call_tool("fs.disk_usage", {"path": os.path.dirname(BACKUP_ROOT) or "/"})
        need = du_src.get("output", {}).get("used_bytes", 0) if du_src["success"] else 0
        avail = du_dst.get("output", {}).get("available_bytes", 1 << 62) if du_dst["success"] else 1 << 62
        if need and need > avail:
            return {"success": False, "error": f"not enough space for backup of {src}"}
        if need and need > 0.9 * avail:
            # tight on space: let the model decide between proceeding and aborting (reference
            # storage.py:244); an unavailable runtime aborts (fail closed, as the reference's think())
            decision = await self.safety_check(
                f"Backup of {src} estimated at {need / 1e9:.1f}GB but only {avail / 1e9:.1f}GB available. "
                "Should I proceed, skip some paths, or abort?", IntelligenceLevel.OPERATIONAL)
            if decision is None:
                return self.safety_unavailable(f"backing up {src} into a nearly full disk")
            if "abort" in decision.lower():
                return {"success": False, "error": f"aborted: backup of {src} would not fit",
                        "ai_decision": decision}
        await self.call_tool("fs.mkdir", {"path": os.path.dirname(dst), "recursive": True})
        r = await self.call_tool("fs.copy", {"source": src, "destination": dst, "recursive": True})
        try:
            await self.push_event("storage.backup_created" if r["success"] else "storage.backup_failed",
                                  {"source": src, "destination": dst})
            if r["success"]:
                await self.store_memory("last_backup", {"source": src, "destination": dst, "ts": int(time.time())})
        except Exception:
            pass
        return {"success": r["success"], "source": src, "destination": dst, "error": r.get("error")} \
            if not r["success"] else {"success": True, "source": src, "destination": dst}

    async def restore_backup(self, task: Dict[str, Any]) -> Dict[str, Any]:
        inp = task.get("input") or {}
        last = None
        try:
            last = await self.recall_memory("last_backup")
        except Exception:
            pass
        src = inp.get("backup") or (last or {}).get("destination")
        dst = inp.get("destination") or (last or {}).get("source")
        if not src or not dst:
            return {"success": False, "error": "no backup to restore"}
        st = await self.call_tool("fs.stat", {"path": src})
        if not st["success"]:
            return {"success": False, "error": f"backup {src} missing"}
        # safety review before overwriting (reference storage.py:359)
        safety = await self.safety_check(f"About to restore backup {src} to {dst}. Is this safe? What could go "
                                         "wrong?", IntelligenceLevel.TACTICAL)
        if safety is None and not inp.get("dry_run"):
            return self.safety_unavailable(f"restoring {src} over {dst}")
        if inp.get("dry_run"):
            return {"success": True, "dry_run": True, "restored": None, "from": src, "to": dst, "safety": safety}
        r = await self.call_tool("fs.copy", {"source": src, "destination": dst, "recursive": True})
        return {"success": r["success"], "restored": dst, "from": src, "safety": safety,
                **({} if r["success"] else {"error": r["error"]})}

    async def manage_mounts(self, task: Dict[str, Any]) -> Dict[str, Any]:
        r = await self.call_tool("fs.read", {"path": "/proc/mounts"})
        if not r["success"]:
            return r
        mounts = []
        for ln in r["output"].get("content", "").splitlines():
            p = ln.split()
            if len(p) >= 4 and p[0].startswith("/dev"):
                mounts.append({"device": p[0], "mountpoint": p[1], "fstype": p[2], "options": p[3]})
        return {"success": True, "mounts": mounts}

    async def fsck(self, task: Dict[str, Any]) -> Dict[str, Any]:
        dev = (task.get("input") or {}).get("device")
        if not dev:
            return {"success": False, "error": "fsck needs an explicit unmounted device"}
        return await self.call_tool("process.spawn", {"command": "fsck", "args": ["-n", dev], "wait": True})

    async def capacity_planning(self, task: Dict[str, Any]) -> Dict[str, Any]:
        now = await self.check_disk_health(task)
        hist = []
        try:
            hist = (await self.recall_memory("disk_history")) or []
        except Exception:
            pass
        hist = (hist + [[int(time.time()), now.get("percent", 0.0)]])[-100:]
        try:
            await self.store_memory("disk_history", hist)
        except Exception:
            pass
        eta_days = None
        if len(hist) >= 2 and hist[-1][1] > hist[0][1]:
            rate = (hist[-1][1] - hist[0][1]) / max(hist[-1][0] - hist[0][0], 1)  # %/s
            eta_days = (100.0 - hist[-1][1]) / rate / 86400.0
        recommendations = []
        pct = now.get("percent") or 0.0
        if pct >= DISK_WARN or (eta_days is not None and eta_days < 30):
            # free space / plan expansion (reference storage.py:569)
            recommendations = self.advice_lines(await self.analyze(
                f"Storage capacity warning: {pct:.1f}% used"
                + (f", full in {eta_days:.1f} days at the current rate" if eta_days is not None else "")
                + ".\nRecommend actions to free space or plan expansion.", IntelligenceLevel.OPERATIONAL))
        return {"success": True, "percent": now.get("percent"), "samples": len(hist), "days_until_full": eta_days,
                "recommendations": recommendations}

    async def background(self):
        return [self.periodic(DISK_CHECK_INTERVAL_S, lambda: self.capacity_planning({}))]


if __name__ == "__main__":
    main_for(StorageAgent)

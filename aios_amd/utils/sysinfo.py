"""Host / GPU telemetry read straight from procfs and the amdgpu sysfs nodes.

Used by the orchestrator's GetSystemStatus, the memory service's GetSystemSnapshot, the
proactive goal generator and the management console (reference: `agent-core/src/main.rs:
103-133` read /proc/stat + /proc/meminfo; `memory/src/operational.rs:63-82` mapped metric keys).
GPU utilisation comes from `/sys/class/drm/card*/device/gpu_busy_percent` (amdgpu), VRAM from
`mem_info_vram_{used,total}` -- no rocm-smi subprocess on the hot path.
"""
from __future__ import annotations

import glob
import os
import shutil
import time
from typing import Dict, List, Optional, Tuple

_last_cpu: Optional[Tuple[int, int]] = None


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


def cpu_percent() -> float:
    """Busy % since the previous call (first call: since boot)."""
    global _last_cpu
    line = _read("/proc/stat").split("\n", 1)[0].split()
    if not line or line[0] != "cpu":
        return 0.0
    vals = [int(x) for x in line[1:]]
    idle = vals[3] + (vals[4] if len(vals) > 4 else 0)
    total = sum(vals)
    prev = _last_cpu
    _last_cpu = (idle, total)
    if prev is None:
        return 100.0 * (total - idle) / total if total else 0.0
    di, dt = idle - prev[0], total - prev[1]
    return max(0.0, min(100.0, 100.0 * (dt - di) / dt)) if dt > 0 else 0.0


def memory_mb() -> Tuple[float, float]:
    """(used_mb, total_mb) with used = total - available."""
    info: Dict[str, int] = {}
    for ln in _read("/proc/meminfo").splitlines():
        k, _, v = ln.partition(":")
        parts = v.split()
        if parts:
            info[k] = int(parts[0])
    total = info.get("MemTotal", 0) / 1024.0
    avail = info.get("MemAvailable", info.get("MemFree", 0)) / 1024.0
    return total - avail, total


def disk_gb(path: str = "/") -> Tuple[float, float]:
    try:
        u = shutil.disk_usage(path)
        return u.used / 1e9, u.total / 1e9
    except OSError:
        return 0.0, 0.0


def disk_percent(path: str = "/") -> float:
    used, total = disk_gb(path)
    return 100.0 * used / total if total else 0.0


def uptime_s() -> float:
    s = _read("/proc/uptime").split()
    return float(s[0]) if s else 0.0


def load_avg() -> List[float]:
    try:
        return list(os.getloadavg())
    except OSError:
        return [0.0, 0.0, 0.0]


def amd_gpus() -> List[dict]:
    """amdgpu devices visible through sysfs: busy %, VRAM used/total (MB)."""
    out = []
    for dev in sorted(glob.glob("/sys/class/drm/card[0-9]*/device")):
        if _read(os.path.join(dev, "vendor")).strip() != "0x1002":
            continue
        busy = _read(os.path.join(dev, "gpu_busy_percent")).strip()
        vu = _read(os.path.join(dev, "mem_info_vram_used")).strip()
        vt = _read(os.path.join(dev, "mem_info_vram_total")).strip()
        out.append({
            "card": dev.split("/")[-2],
            "device_id": _read(os.path.join(dev, "device")).strip(),
            "busy_percent": float(busy) if busy.isdigit() else 0.0,
            "vram_used_mb": int(vu) / 2**20 if vu.isdigit() else 0.0,
            "vram_total_mb": int(vt) / 2**20 if vt.isdigit() else 0.0,
        })
    return out


def gpu_utilization() -> float:
    g = amd_gpus()
    return sum(x["busy_percent"] for x in g) / len(g) if g else 0.0


def snapshot() -> dict:
    used, total = memory_mb()
    du, dt = disk_gb("/")
    return {"cpu_percent": cpu_percent(), "memory_used_mb": used, "memory_total_mb": total,
            "disk_used_gb": du, "disk_total_gb": dt, "gpu_utilization": gpu_utilization(),
            "load_avg": load_avg(), "uptime_s": uptime_s(), "timestamp": int(time.time())}


def metric_snapshot() -> dict:
    """Flat metric map for plugin metric_threshold triggers (operational-memory metric keys)."""
    used, total = memory_mb()
    out = {"cpu.usage": cpu_percent(), "memory.used_mb": used, "memory.total_mb": total,
           "memory.percent": 100.0 * used / total if total else 0.0, "disk.percent": disk_percent("/"),
           "load.1m": (load_avg() or [0.0])[0], "uptime.seconds": uptime_s()}
    try:
        out["gpu.utilization"] = gpu_utilization()
    except Exception:  # pragma: no cover - no GPU sysfs
        pass
    return out

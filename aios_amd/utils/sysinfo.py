"""Host / GPU telemetry read straight from procfs and the amdgpu sysfs nodes.

Used by the orchestrator's GetSystemStatus, the memory service's GetSystemSnapshot, the
proactive goal generator and the management console (reference: `agent-core/src/main.rs:
103-133` read /proc/stat + /proc/meminfo; `memory/src/operational.rs:63-82` mapped metric keys).
GPU utilisation comes from `/sys/class/drm/card*/device/gpu_busy_percent` (amdgpu), VRAM from
`mem_info_vram_{used,total}` -- no rocm-smi subprocess on the hot path.  GPU health (SURVEY §5
"amd-smi ECC/xGMI counters feed health"): the amdgpu RAS counters `device/ras/*_err_count`
(`ue: N` / `ce: M` per block -- umc = HBM ECC, xgmi_wafl = the xGMI links, gfx, sdma, ...),
`device/pcie_replay_count`, and hwmon temperatures (edge / junction / mem, millidegrees) and
average socket power (microwatts).  `root` re-targets every read for tests.
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


def _ras(dev: str) -> Dict[str, Dict[str, int]]:
    """RAS error counts per block: {"umc": {"ue": 0, "ce": 3}, "xgmi_wafl": {...}, ...}."""
    out: Dict[str, Dict[str, int]] = {}
    for f in sorted(glob.glob(os.path.join(dev, "ras", "*_err_count"))):
        block = os.path.basename(f)[: -len("_err_count")]
        counts = {}
        for ln in _read(f).splitlines():
            k, _, v = ln.partition(":")
            if v.strip().isdigit():
                counts[k.strip()] = int(v.strip())
        if counts:
            out[block] = counts
    return out


def _hwmon(dev: str) -> dict:
    out: Dict[str, float] = {}
    for hw in sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*"))):
        for t in sorted(glob.glob(os.path.join(hw, "temp*_input"))):
            label = _read(t.replace("_input", "_label")).strip() or os.path.basename(t)[:-6]
            v = _read(t).strip()
            if v.lstrip("-").isdigit():
                out[f"temp_{label}_c"] = int(v) / 1000.0
        for name in ("power1_average", "power1_input"):
            v = _read(os.path.join(hw, name)).strip()
            if v.isdigit():
                out["power_w"] = int(v) / 1e6
                break
    return out


def amd_gpus(root: str = "/") -> List[dict]:
    """amdgpu devices visible through sysfs: busy %, VRAM used/total (MB), RAS error counts,
    PCIe replays, temperatures and power."""
    out = []
    for dev in sorted(glob.glob(os.path.join(root, "sys/class/drm/card[0-9]*/device"))):
        if _read(os.path.join(dev, "vendor")).strip() != "0x1002":
            continue
        busy = _read(os.path.join(dev, "gpu_busy_percent")).strip()
        vu = _read(os.path.join(dev, "mem_info_vram_used")).strip()
        vt = _read(os.path.join(dev, "mem_info_vram_total")).strip()
        rp = _read(os.path.join(dev, "pcie_replay_count")).strip()
        ras = _ras(dev)
        out.append({
            "card": dev.split("/")[-2],
            "device_id": _read(os.path.join(dev, "device")).strip(),
            "busy_percent": float(busy) if busy.isdigit() else 0.0,
            "vram_used_mb": int(vu) / 2**20 if vu.isdigit() else 0.0,
            "vram_total_mb": int(vt) / 2**20 if vt.isdigit() else 0.0,
            "ras": ras,
            "ecc_ue": sum(c.get("ue", 0) for c in ras.values()),
            "ecc_ce": sum(c.get("ce", 0) for c in ras.values()),
            "xgmi_ue": ras.get("xgmi_wafl", {}).get("ue", 0),
            "pcie_replays": int(rp) if rp.isdigit() else 0,
            **_hwmon(dev),
        })
    return out


def gpu_health(root: str = "/", hot_c: float = 95.0) -> dict:
    """Node GPU health from the RAS / thermal counters: per-card problems and a verdict."""
    cards, problems = amd_gpus(root), []
    for g in cards:
        if g["ecc_ue"]:
            problems.append({"card": g["card"], "kind": "uncorrectable_ecc", "count": g["ecc_ue"],
                             "blocks": sorted(b for b, c in g["ras"].items() if c.get("ue"))})
        if g["xgmi_ue"]:
            problems.append({"card": g["card"], "kind": "xgmi_link_errors", "count": g["xgmi_ue"]})
        hot = max([v for k, v in g.items() if k.startswith("temp_") and isinstance(v, float)] or [0.0])
        if hot >= hot_c:
            problems.append({"card": g["card"], "kind": "overtemperature", "temp_c": hot})
    return {"gpus": len(cards), "healthy": not problems, "problems": problems,
            "ecc_ce_total": sum(g["ecc_ce"] for g in cards), "ecc_ue_total": sum(g["ecc_ue"] for g in cards)}


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

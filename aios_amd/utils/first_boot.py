"""One-time node initialisation, run by aios-init (phase 3.5) when <data_dir>/.first-boot exists
(`scripts/first-boot.sh` -> `python3 -m aios_amd.utils.first_boot`).

Reference: scripts/first-boot.sh (656 lines of bash: identity keys, SQLite schemas, directory
layout, permissions, network + API probes, model download, hardware detection, system-agent
state, flag removal).  Same steps here, through the native cores so every schema is the one the
services open, plus what an MI355X node needs: the KFD topology (gfx target, CUs, HBM, xGMI links
between GPUs) in hardware.json, and the node's mTLS certificates generated ONCE before any
service starts (services then only verify them; ADVICE r1: concurrent generation raced).

Every step is recorded in <data_dir>/first-boot.json; a failed step does not stop the others,
and the exit status is 1 only when a step the node cannot run without fails (directories,
databases, identity).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import time
import uuid
from typing import Callable, Dict, List, Tuple

DIRS = ("data", "memory", "ledger", "models", "plugins", "cache/backups", "certs", "workspace", "downloads", "keys")


def _read(path: str, default: str = "") -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def _kv(path: str) -> Dict[str, int]:
    out = {}
    for line in _read(path).splitlines():
        p = line.split()
        if len(p) == 2 and p[1].lstrip("-").isdigit():
            out[p[0]] = int(p[1])
    return out


def kfd_topology(root: str = "/sys/class/kfd/kfd/topology/nodes") -> List[Dict]:
    """GPU agents of the KFD topology: gfx target, CUs, HBM bytes, xGMI / PCIe links."""
    gpus = []
    for node in sorted(glob.glob(os.path.join(root, "*")), key=lambda p: int(os.path.basename(p) or 0)):
        props = _kv(os.path.join(node, "properties"))
        if not props.get("simd_count"):
            continue  # CPU node
        gfx = props.get("gfx_target_version", 0)
        mem = sum(_kv(b + "/properties").get("size_in_bytes", 0)
                  for b in glob.glob(os.path.join(node, "mem_banks", "*")))
        links = []
        for l in sorted(glob.glob(os.path.join(node, "io_links", "*"))):
            lp = _kv(os.path.join(l, "properties"))
            # io_link type 11 = xGMI, 2 = PCIe (KFD CRAT)
            links.append({"to_node": lp.get("node_to"), "type": {11: "xgmi", 2: "pcie"}.get(lp.get("type"), lp.get("type")),
                          "weight": lp.get("weight"), "max_bandwidth_mbs": lp.get("max_bandwidth")})
        gpus.append({"node": int(os.path.basename(node)), "gfx_target_version": gfx,
                     "gfx": f"gfx{gfx // 10000}{(gfx // 100) % 100:x}{gfx % 100:x}" if gfx else "",
                     "simd_count": props.get("simd_count"), "cu_count": props.get("simd_count", 0) // 4,
                     "max_waves_per_simd": props.get("max_waves_per_simd"), "hbm_bytes": mem,
                     "unique_id": props.get("unique_id"), "links": links})
    return gpus


def hardware_inventory() -> Dict:
    mem_kb = 0
    for line in _read("/proc/meminfo").splitlines():
        if line.startswith("MemTotal:"):
            mem_kb = int(line.split()[1])
    model = next((l.split(":", 1)[1].strip() for l in _read("/proc/cpuinfo").splitlines() if l.startswith("model name")),
                 "")
    cards = []
    for c in sorted(glob.glob("/sys/class/drm/card[0-9]*")):
        if os.path.basename(c).count("-"):
            continue  # connectors
        if _read(os.path.join(c, "device", "vendor")) == "0x1002":
            cards.append({"card": os.path.basename(c), "device": _read(os.path.join(c, "device", "device"))})
    gpus = kfd_topology()
    return {"hostname": socket.gethostname(), "cpus": os.cpu_count(), "cpu_model": model, "mem_kb": mem_kb,
            "kfd": os.path.exists("/dev/kfd"), "amd_drm_cards": cards, "amd_gpus": gpus,
            "mi355x": sum(1 for g in gpus if g["gfx"] == "gfx950"),
            "xgmi_links": sum(1 for g in gpus for l in g["links"] if l["type"] == "xgmi")}


def _valid_key(path: str) -> bool:
    """an existing private key openssl can parse (an empty or truncated file is not one)"""
    if not os.path.exists(path) or os.path.getsize(path) == 0:
        return False
    if not shutil.which("openssl"):
        return True
    r = subprocess.run(["openssl", "pkey", "-in", path, "-noout"], capture_output=True, timeout=30)
    return r.returncode == 0


class FirstBoot:
    def __init__(self, data: str, etc: str, log: str, probe_network: bool = True, download_models: bool = False):
        self.data, self.etc, self.log = data, etc, log
        self.probe_network, self.download_models = probe_network, download_models
        self.report: Dict[str, Dict] = {}

    def p(self, *parts: str) -> str:
        return os.path.join(self.data, *parts)

    # -- steps ----------------------------------------------------------------------------------
    def directories(self):
        for d in DIRS:
            os.makedirs(self.p(d), exist_ok=True)
        os.makedirs(self.log, exist_ok=True)
        return {"created": list(DIRS)}

    def identity(self):
        node_id_file = self.p("node_id")
        if not os.path.exists(node_id_file):
            with open(node_id_file, "w") as f:
                f.write(str(uuid.uuid4()) + "\n")
        keys = {}
        for name in ("node", "ledger-signing"):
            key = self.p("keys", f"{name}.key")
            if not _valid_key(key):
                # generated into a private temp file and renamed into place: a crash mid-way
                # leaves no empty key behind that later runs would mistake for an identity
                # (ADVICE r2); an empty or unparsable key is regenerated
                if not shutil.which("openssl"):
                    raise RuntimeError("openssl not found: cannot create the Ed25519 identity")
                tmp = f"{key}.tmp.{os.getpid()}"
                fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
                os.close(fd)
                r = subprocess.run(["openssl", "genpkey", "-algorithm", "ed25519", "-out", tmp],
                                   capture_output=True, text=True, timeout=30)
                if r.returncode:
                    os.unlink(tmp)
                    raise RuntimeError(f"openssl genpkey failed: {r.stderr.strip()}")
                os.chmod(tmp, 0o600)
                os.replace(tmp, key)
                pub = subprocess.run(["openssl", "pkey", "-in", key, "-pubout"], capture_output=True, text=True,
                                     timeout=30)
                with open(key[:-4] + ".pub", "w") as f:
                    f.write(pub.stdout)
            keys[name] = key
        return {"node_id": _read(node_id_file), "keys": keys}

    def databases(self):
        from ..core import load as load_core

        c = load_core()
        c.ToolService(self.data, os.environ.get("AIOS_SOURCE_DIR", ""))  # audit ledger, capability grants, backups
        m = c.MemoryStore(self.p("memory", "working.db"), self.p("memory", "longterm.db"),
                          self.p("memory", "knowledge.db"))
        c.GoalEngine(self.p("data", "goals.db"))
        c.gateway.BudgetLedger(100.0, 50.0, self.p("data", "gateway_usage.db"))
        m.store_agent_state("system-agent", json.dumps({"initialized_at": int(time.time()), "first_boot": True,
                                                        "node_id": _read(self.p("node_id"))}))
        dbs = sorted(glob.glob(self.p("**", "*.db"), recursive=True))
        return {"databases": [os.path.relpath(d, self.data) for d in dbs]}

    def permissions(self):
        for d in ("ledger", "certs", "keys"):
            os.chmod(self.p(d), 0o700)
        n = 0
        for f in glob.glob(self.p("**", "*.db"), recursive=True) + glob.glob(self.p("keys", "*.key")):
            os.chmod(f, 0o600)
            n += 1
        return {"restricted_files": n}

    def tls(self):
        from ..core import load as load_core

        mgr = load_core().TlsManager(self.p("certs"))
        mgr.generate_self_signed("aios")
        return {"verify": mgr.verify(), "paths": mgr.paths()}

    def hardware(self):
        inv = hardware_inventory()
        with open(self.p("hardware.json"), "w") as f:
            json.dump(inv, f, indent=2)
        return {"amd_gpus": len(inv["amd_gpus"]), "mi355x": inv["mi355x"], "xgmi_links": inv["xgmi_links"],
                "kfd": inv["kfd"]}

    def network(self):
        if not self.probe_network:
            return {"skipped": True}
        ok = []
        for host, port in (("1.1.1.1", 53), ("8.8.8.8", 53)):
            try:
                socket.create_connection((host, port), timeout=2).close()
                ok.append(host)
            except OSError:
                pass
        return {"reachable": ok, "online": bool(ok)}

    def api_keys(self):
        keys = {k: bool(os.environ.get(k)) for k in ("CLAUDE_API_KEY", "OPENAI_API_KEY", "QWEN3_API_KEY")}
        secrets = os.environ.get("AIOS_SECRETS", os.path.join(self.etc, "secrets.toml"))
        return {"env_keys": keys, "secrets_file": os.path.exists(secrets),
                "note": "cloud providers optional: the local strategic tier serves the api-gateway"}

    def models(self):
        from .config import load as load_config

        cfg = load_config()
        model_dir = cfg.models.model_dir
        have, missing = [], []
        for name, t in cfg.models.tiers.items():
            path = t.file if os.path.isabs(t.file) else os.path.join(model_dir, t.file)
            (have if t.file and os.path.exists(path) else missing).append(name)
        out = {"model_dir": model_dir, "present": have, "missing": missing}
        if missing and self.download_models:
            script = os.path.join(os.path.dirname(__file__), "..", "..", "scripts", "download-models.sh")
            r = subprocess.run(["bash", script], capture_output=True, text=True, timeout=3600)
            out["download_rc"] = r.returncode
        return out

    def finalize(self):
        with open(self.p(".first-boot-done"), "w") as f:
            f.write(str(int(time.time())) + "\n")
        try:
            os.unlink(self.p(".first-boot"))
        except FileNotFoundError:
            pass
        return {"done": True}

    # -- driver ---------------------------------------------------------------------------------
    def run(self) -> int:
        steps: List[Tuple[str, Callable[[], Dict], bool]] = [
            ("directories", self.directories, True), ("identity", self.identity, True),
            ("databases", self.databases, True), ("permissions", self.permissions, False),
            ("tls", self.tls, False), ("hardware", self.hardware, False), ("network", self.network, False),
            ("api_keys", self.api_keys, False), ("models", self.models, False)]
        fatal = False
        for i, (name, fn, critical) in enumerate(steps, 1):
            t0 = time.time()
            try:
                res = fn()
                self.report[name] = {"ok": True, **res}
            except Exception as e:  # a step failing is recorded, the rest still run
                self.report[name] = {"ok": False, "error": f"{type(e).__name__}: {e}"}
                fatal |= critical
            self.report[name]["seconds"] = round(time.time() - t0, 3)
            print(f"[first-boot] {i}/{len(steps) + 1} {name}: {'ok' if self.report[name]['ok'] else 'FAILED'}",
                  flush=True)
        if not fatal:
            self.report["finalize"] = {"ok": True, **self.finalize()}
            print(f"[first-boot] {len(steps) + 1}/{len(steps) + 1} finalize: ok", flush=True)
        with open(self.p("first-boot.json"), "w") as f:
            json.dump(self.report, f, indent=2, default=str)
        return 1 if fatal else 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="aiOS first-boot initialisation")
    ap.add_argument("--data-dir", default=os.environ.get("AIOS_DATA_DIR", "/var/lib/aios"))
    ap.add_argument("--etc", default=os.environ.get("AIOS_ETC", "/etc/aios"))
    ap.add_argument("--log-dir", default=os.environ.get("AIOS_LOG_DIR", "/var/log/aios"))
    ap.add_argument("--no-network", action="store_true", help="skip the connectivity probe")
    ap.add_argument("--download-models", action="store_true", help="fetch missing GGUF files")
    a = ap.parse_args(argv)
    return FirstBoot(a.data_dir, a.etc, a.log_dir, not a.no_network, a.download_models).run()


if __name__ == "__main__":
    sys.exit(main())

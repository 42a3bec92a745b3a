#!/usr/bin/env bash
# One-time node initialisation (run by aios-init when <data_dir>/.first-boot exists).
# Steps: directory layout, node identity key, databases, permissions, hardware inventory
# (incl. MI355X / amdgpu detection), firewall baseline, connectivity probe, finalize.
set -uo pipefail
DATA=${AIOS_DATA_DIR:-/var/lib/aios}
ETC=${AIOS_ETC:-/etc/aios}
LOG=${AIOS_LOG_DIR:-/var/log/aios}
say() { echo "[first-boot] $*"; }
say "1/8 directories"
for d in data memory ledger models plugins cache/backups certs workspace downloads; do mkdir -p "$DATA/$d"; done
mkdir -p "$LOG"
say "2/8 node identity"
if [ ! -f "$DATA/certs/node.key" ]; then
  if command -v openssl >/dev/null; then
    openssl genpkey -algorithm ed25519 -out "$DATA/certs/node.key" 2>/dev/null && chmod 600 "$DATA/certs/node.key"
  fi
fi
say "3/8 databases (created on first open by the services; touch to fix ownership)"
for f in data/goals.db data/scheduler.db memory/working.db memory/longterm.db memory/knowledge.db ledger/audit.db; do
  touch "$DATA/$f"
done
say "4/8 permissions"
chmod 700 "$DATA/ledger" "$DATA/certs" 2>/dev/null || true
say "5/8 hardware inventory"
{
  echo "{"
  echo "  \"cpus\": $(nproc),"
  echo "  \"mem_kb\": $(awk '/MemTotal/ {print $2}' /proc/meminfo),"
  printf '  "amd_gpus": ['
  first=1
  for c in /sys/class/drm/card[0-9]*; do
    [ -f "$c/device/vendor" ] || continue
    [ "$(cat "$c/device/vendor")" = "0x1002" ] || continue
    [ $first = 1 ] || printf ', '
    first=0
    printf '{"card": "%s", "device": "%s"}' "$(basename "$c")" "$(cat "$c/device/device")"
  done
  echo "],"
  echo "  \"kfd\": $([ -e /dev/kfd ] && echo true || echo false)"
  echo "}"
} > "$DATA/hardware.json"
say "6/8 firewall baseline"
if command -v nft >/dev/null && [ -f "$ETC/security/firewall-rules.toml" ]; then
  nft list tables >/dev/null 2>&1 && say "nftables available (rules applied by the network agent)"
fi
say "7/8 connectivity probe"
(ping -c1 -W2 1.1.1.1 >/dev/null 2>&1 && say "network ok") || say "network unreachable (offline node)"
say "8/8 finalize"
date -u +%s > "$DATA/.first-boot-done"
rm -f "$DATA/.first-boot"

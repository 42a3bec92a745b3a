#!/usr/bin/env bash
# Install aiOS onto an MI355X host (ROCm + PyTorch-ROCm already present):
#   sudo scripts/install.sh [--prefix /opt/aios] [--no-systemd]
# Copies the built package, config and agent definitions, creates the data layout, installs the
# aios-init systemd unit (aios-init supervises runtime, memory, tools, api-gateway, orchestrator).
set -euo pipefail
SRC="$(cd "$(dirname "$0")/.." && pwd)"
PREFIX=/opt/aios; SYSTEMD=1
while [ $# -gt 0 ]; do
  case "$1" in --prefix) PREFIX="$2"; shift ;; --no-systemd) SYSTEMD=0 ;; *) echo "unknown $1"; exit 2 ;; esac
  shift
done
[ -f "$SRC/aios_amd/bin/aios-init" ] || { echo "run scripts/build-all.sh first"; exit 1; }
echo "[install] package -> $PREFIX"
mkdir -p "$PREFIX"
cp -a "$SRC/aios_amd" "$SRC/tools" "$SRC/config" "$SRC/scripts" "$PREFIX/"
echo "[install] config -> /etc/aios"
mkdir -p /etc/aios/agents /etc/aios/security
[ -f /etc/aios/config.toml ] || cp "$SRC/config/default-config.toml" /etc/aios/config.toml
cp -n "$SRC"/deploy/etc/aios/agents/*.toml /etc/aios/agents/ || true
cp -n "$SRC"/deploy/etc/aios/security/*.toml /etc/aios/security/ || true
mkdir -p /usr/lib/aios && cp "$SRC/scripts/first-boot.sh" /usr/lib/aios/first-boot.sh
mkdir -p /var/lib/aios /var/log/aios && touch /var/lib/aios/.first-boot
if [ "$SYSTEMD" = 1 ] && command -v systemctl >/dev/null; then
  sed "s#@PREFIX@#$PREFIX#g" "$SRC/deploy/systemd/aios.service" > /etc/systemd/system/aios.service
  systemctl daemon-reload
  echo "[install] enable with: systemctl enable --now aios"
fi
echo "[install] done"

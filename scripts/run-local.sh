#!/usr/bin/env bash
# Run the whole stack on this machine without root (development / demo): a private data dir,
# synthetic models unless AIOS_MODEL_DIR holds GGUF files, console on :9090.
#   scripts/run-local.sh [--data DIR] [--synthetic "mistral-7b=synthetic:mistral-7b"] [--seconds N]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
DATA="${TMPDIR:-/tmp}/aios-local"; SYN="tinyllama-1.1b=synthetic:tinyllama-1.1b,mistral-7b=synthetic:mistral-7b"; SECS=0
while [ $# -gt 0 ]; do
  case "$1" in --data) DATA="$2"; shift ;; --synthetic) SYN="$2"; shift ;; --seconds) SECS="$2"; shift ;; *) exit 2 ;; esac
  shift
done
mkdir -p "$DATA/log"
CFG="$DATA/config.toml"
cat > "$CFG" <<TOML
[system]
data_dir = "$DATA"
log_dir = "$DATA/log"
[boot]
clean_shutdown_flag = "$DATA/.clean-shutdown"
[services.aios-runtime.env]
AIOS_SYNTHETIC_MODELS = "$SYN"
AIOS_MODEL_DIR = "${AIOS_MODEL_DIR:-$DATA/models}"
[services.aios-tools.env]
AIOS_DATA_DIR = "$DATA"
[services.aios-memory.env]
AIOS_DATA_DIR = "$DATA"
[services.aios-orchestrator.env]
AIOS_DATA_DIR = "$DATA"
AIOS_AGENTS_DIR = "$ROOT/deploy/etc/aios/agents"
TOML
export PYTHONPATH="$ROOT${PYTHONPATH:+:$PYTHONPATH}" AIOS_DATA_DIR="$DATA" HSA_ENABLE_IPC_MODE_LEGACY=0
ARGS=(--config "$CFG" --no-mount)
[ "$SECS" != 0 ] && ARGS+=(--run-for "$SECS")
exec "$ROOT/aios_amd/bin/aios-init" "${ARGS[@]}"

#!/usr/bin/env bash
# One-time node initialisation, run by aios-init (phase 3.5) when <data_dir>/.first-boot exists.
# Steps (aios_amd/utils/first_boot.py, report in <data_dir>/first-boot.json):
#   1 directories  2 Ed25519 node identity + ledger signing key  3 SQLite schemas through the
#   native cores (audit ledger, memory tiers, goals, gateway usage) + system-agent state
#   4 permissions  5 node mTLS certificates (generated once, before any service)
#   6 hardware inventory (KFD topology: gfx950 agents, CUs, HBM, xGMI links)  7 connectivity
#   8 API keys  9 model files (optional download)  10 finalize (flag removed, timestamp)
# Exit status 1 only when a step the node cannot run without failed.
set -uo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=${AIOS_SOURCE_DIR:-$(cd "$HERE/.." && pwd)}
PY=${AIOS_PYTHON:-python3}
export PYTHONPATH="$ROOT${PYTHONPATH:+:$PYTHONPATH}"
exec "$PY" -m aios_amd.utils.first_boot "$@"

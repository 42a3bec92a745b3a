#!/usr/bin/env bash
# In-situ sweep of the decode GEMV knobs (AIOS_GEMV_{U,GRID}_{QKV,O,GU,DOWN,LM}) on the captured
# Mistral decode step: one short bench.py run per setting, tok/s per line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CONFIGS=${CONFIGS:-"base"}
for c in $CONFIGS; do
  envs=()
  if [ "$c" != base ]; then
    if [[ "$c" == *:* ]]; then
      kind=${c%%:*}; kv=${c#*:}; knob=${kv%%=*}; val=${kv#*=}
      envs=("AIOS_GEMV_${knob}_${kind}=${val}")
    else
      envs=(${c//,/ })   # raw VAR=VAL[,VAR=VAL]
    fi
  fi
  out=$(env "${envs[@]}" timeout -k 10 120 python bench.py --steps 96 --warmup 8 --no-secondary 2>/dev/null | tail -1) || { echo "$c FAILED"; exit 1; }
  v=$(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
  echo "$c $v"
done

#!/usr/bin/env bash
# batch-1 ring depth per format: Q4_K RSUB 1 with Q6_K RSUB 1 / 2 / 0, interleaved
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
for r in 0 1; do
  for x in 1 2 0; do
    echo -n "B1 RSUB_Q6=$x "; AIOS_LDS_B1_RSUB_Q6=$x timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j || exit 1
  done
done

#!/usr/bin/env bash
# batched decode step times after the ring split-norm fix (B = 5 / 32)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
for b in 5 32 5 32; do
  echo -n "B$b "; timeout -k 10 300 python bench.py --batch $b --steps 128 --warmup 16 --no-secondary 2>/dev/null | j || exit 1
done

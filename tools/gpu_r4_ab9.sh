#!/usr/bin/env bash
# confirmation: ring one slot shallower (this tree) vs cmp_r4c at B = 5 / 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
md5sum aios_amd/_engine*.so cmp_r4c/aios_amd/_engine*.so | cut -c1-12
for b in 5 8; do
  for d in . cmp_r4c; do
    echo -n "B$b $d "; (cd $d && timeout -k 10 300 python bench.py --batch $b --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
  done
done

#!/usr/bin/env bash
# ring GEMM one slot shallower (RG_RSUB 1) vs cmp_r4c (full depth), B = 5 / 8 / 16 / 32; ring tests first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "ring or skinny" > gpurun_out/t_ab8.log 2>&1 || { tail -40 gpurun_out/t_ab8.log; exit 1; }
tail -1 gpurun_out/t_ab8.log
for b in 5 8 16 32; do
  for d in cmp_r4c . cmp_r4c .; do
    echo -n "B$b $d "; (cd $d && timeout -k 10 300 python bench.py --batch $b --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
  done
done

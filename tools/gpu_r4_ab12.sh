#!/usr/bin/env bash
# same box: cmp_r4c vs this tree (attention phase stamps compiled out + the row-GEMV / engine stamp
# changes), B=1 at 128 and 4000-token prompts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn or attention" > gpurun_out/t_ab12.log 2>&1 || { tail -40 gpurun_out/t_ab12.log; exit 1; }
tail -1 gpurun_out/t_ab12.log
for r in 0 1; do
  for d in cmp_r4c .; do
    echo -n "B1 $d "; (cd $d && timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
    echo -n "p4000 $d "; (cd $d && timeout -k 10 300 python bench.py --prompt 4000 --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
  done
done

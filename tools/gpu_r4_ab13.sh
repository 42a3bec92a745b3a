#!/usr/bin/env bash
# same box: cmp_r4c vs this tree with the row-GEMV / CU-kernel phase stamps compiled out as well
# (previous build measured 663.3 -> 671.2 against cmp_r4c, tools/gpu_r4_final.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemv" > gpurun_out/t_ab13.log 2>&1 || { tail -40 gpurun_out/t_ab13.log; exit 1; }
tail -1 gpurun_out/t_ab13.log
for r in 0 1; do
  for d in cmp_r4c .; do
    echo -n "B1 $d "; (cd $d && timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
  done
done
for d in cmp_r4c .; do
  echo -n "tinyllama $d "; (cd $d && timeout -k 10 300 python bench.py --model tinyllama-1.1b --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
done

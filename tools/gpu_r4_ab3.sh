#!/usr/bin/env bash
# same box: previous build (cmp_r4a) vs this tree -- B=1 (row GEMV probe branches compiled out) and
# B = 5 / 8 / 16 / 32 (ring GEMM with the resident X slice at M <= 8); kernel tests first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_engine_gpu.py -k "ring or skinny or batched or gemv or short_prompt" > gpurun_out/t_ab3.log 2>&1 \
  || { tail -40 gpurun_out/t_ab3.log; exit 1; }
tail -1 gpurun_out/t_ab3.log
for r in 0 1; do
  for d in cmp_r4a .; do
    echo -n "B1 $d "; (cd $d && timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
  done
done
for d in cmp_r4a .; do
  echo -n "tinyllama $d "; (cd $d && timeout -k 10 300 python bench.py --model tinyllama-1.1b --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
done
for b in 5 8 16 32; do
  for d in cmp_r4a .; do
    echo -n "B$b $d "; (cd $d && timeout -k 10 300 python bench.py --batch $b --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
  done
done

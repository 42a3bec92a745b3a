#!/usr/bin/env bash
# same box: cmp_r4c vs this tree (GEMV phase stamps stored as taken: SGPR spills of the row GEMVs
# 69-190 -> 20-112), B=1 Mistral / TinyLlama / B=4; GEMV tests first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_engine_gpu.py -k "gemv or decode or skinny" > gpurun_out/t_ab10.log 2>&1 || { tail -40 gpurun_out/t_ab10.log; exit 1; }
tail -1 gpurun_out/t_ab10.log
for r in 0 1; do
  for d in cmp_r4c .; do
    echo -n "B1 $d "; (cd $d && timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
  done
done
for d in cmp_r4c . cmp_r4c .; do
  echo -n "tinyllama $d "; (cd $d && timeout -k 10 300 python bench.py --model tinyllama-1.1b --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
done
for d in cmp_r4c .; do
  echo -n "B4 $d "; (cd $d && timeout -k 10 300 python bench.py --batch 4 --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
done

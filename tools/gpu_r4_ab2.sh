#!/usr/bin/env bash
# same-box: the previous build (cmp_r4a) vs this tree, TinyLlama + Mistral B=1 + 4k context; kernel tests first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn or attention or gemv" > gpurun_out/t_k.log 2>&1 || { tail -40 gpurun_out/t_k.log; exit 1; }
tail -1 gpurun_out/t_k.log
for r in 0 1; do
  for d in cmp_r4a .; do
    echo -n "$d tinyllama "; (cd $d && timeout -k 10 300 python bench.py --model tinyllama-1.1b --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
  done
done
for d in cmp_r4a .; do
  echo -n "$d mistral "; (cd $d && timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
  echo -n "$d p4000 "; (cd $d && timeout -k 10 300 python bench.py --prompt 4000 --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
done

#!/usr/bin/env bash
# batch-1 ring depth: AIOS_LDS_B1_RSUB 0 / 1 / 2, interleaved, Mistral + TinyLlama; GEMV tests first
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_engine_gpu.py -k "gemv or lds or decode" > gpurun_out/t_ab6.log 2>&1 || { tail -40 gpurun_out/t_ab6.log; exit 1; }
tail -1 gpurun_out/t_ab6.log
for r in 0 1; do
  for x in 0 1 2; do
    echo -n "B1 RSUB=$x "; AIOS_LDS_B1_RSUB=$x timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j || exit 1
  done
done
for x in 0 1 2; do
  echo -n "tinyllama RSUB=$x "; AIOS_LDS_B1_RSUB=$x timeout -k 10 300 python bench.py --model tinyllama-1.1b --steps 256 --warmup 16 --no-secondary 2>/dev/null | j || exit 1
done
for x in 0 1; do
  echo -n "p4000 RSUB=$x "; AIOS_LDS_B1_RSUB=$x timeout -k 10 300 python bench.py --prompt 4000 --steps 128 --warmup 8 --no-secondary 2>/dev/null | j || exit 1
done

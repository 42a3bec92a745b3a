#!/usr/bin/env bash
# TP tests (fused epilogue on the row kernel only), B=1 ring depth knob, B = 2..4 vs cmp_r4a
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_tp.py \
  tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "tp or gemv or batched" > gpurun_out/t_ab5.log 2>&1 \
  || { tail -40 gpurun_out/t_ab5.log; exit 1; }
tail -1 gpurun_out/t_ab5.log
for r in 0 1; do
  for x in 0 1; do
    echo -n "B1 RSUB=$x "; AIOS_LDS_B1_RSUB=$x timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j || exit 1
  done
done
for b in 2 3 4; do
  for d in cmp_r4a .; do
    echo -n "B$b $d "; (cd $d && timeout -k 10 300 python bench.py --batch $b --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
  done
done

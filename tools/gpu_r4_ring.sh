#!/usr/bin/env bash
# round-4 check: ring GEMM numerics, then same-box decode (round-3 tree vs this one) and the
# batched-decode GEMM arms (ring on/off).  Every GPU step under its own limit; stop at first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="--steps 128 --warmup 8 --no-secondary"
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "ring or skinny" > gpurun_out/t_ring.log 2>&1 || { tail -40 gpurun_out/t_ring.log; exit 1; }
tail -2 gpurun_out/t_ring.log
for b in 1 4; do
  for d in cmp_r3 .; do
    echo -n "$d B$b "; (cd $d && timeout -k 10 300 python bench.py --batch $b $B 2>/dev/null | j) || exit 1
  done
done
for b in 5 8 16 32; do
  for ring in 0 1; do
    echo -n "ring=$ring B$b "; AIOS_GEMM_RING=$ring timeout -k 10 300 python bench.py --batch $b $B 2>/dev/null | j || exit 1
  done
done

#!/usr/bin/env bash
# ring GEMM, LDS reads hoisted per slot: numerics, anatomy at B = 8, decode B = 5 / 8 / 16 / 32 vs the
# previous build (cmp_r4a: first ring version)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_engine_gpu.py -k "ring or skinny or batched or short_prompt" > gpurun_out/t_xr.log 2>&1 \
  || { tail -40 gpurun_out/t_xr.log; exit 1; }
tail -1 gpurun_out/t_xr.log
for x in 1 0; do
  echo "AIOS_RING_XR=$x"
  AIOS_RING_XR=$x timeout -k 10 300 python tools/skinny_probe.py --batch 8 > gpurun_out/xrprobe_$x.log 2>&1 \
    || { tail -20 gpurun_out/xrprobe_$x.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/xrprobe_$x.log | cut -c1-120
done
for b in 5 8 16 32; do
  for d in cmp_r4a .; do
    echo -n "B$b $d "; (cd $d && timeout -k 10 300 python bench.py --batch $b --steps 128 --warmup 8 --no-secondary 2>/dev/null | j) || exit 1
  done
done

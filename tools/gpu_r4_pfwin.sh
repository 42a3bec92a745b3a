#!/usr/bin/env bash
# hipBLASLt window for 48..160-row prefill chunks (AIOS_PREFILL_BLAS_WINDOW "0" vs default "33,128"),
# same box, ms per prompt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py \
  -k "prefill" > gpurun_out/t_pfwin.log 2>&1 || { tail -40 gpurun_out/t_pfwin.log; exit 1; }
tail -1 gpurun_out/t_pfwin.log
for r in 0 1; do
  for w in 0 33,128; do
    echo "AIOS_PREFILL_BLAS_WINDOW=$w"
    AIOS_PREFILL_BLAS_WINDOW=$w timeout -k 10 300 python tools/bench_prefill.py --lens 32,33,40,48,64,96,128 \
      > gpurun_out/pfw.log 2>&1 || { tail -20 gpurun_out/pfw.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/pfw.log | python -c 'import sys,json; print(" ".join("%d:%.2f" % (d["prompt_tokens"], d["ms"]) for d in map(json.loads, sys.stdin)))'
  done
done

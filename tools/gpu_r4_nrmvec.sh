#!/usr/bin/env bash
# ring GEMM split-norm consumer: the row's partial sums loaded at once (was one dependent load per part)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py \
  -k "ring or gemm or prefill or batched" > gpurun_out/t_nrmvec.log 2>&1 || { tail -40 gpurun_out/t_nrmvec.log; exit 1; }
tail -1 gpurun_out/t_nrmvec.log
for r in 0 1; do
  for b in 8 16; do
    echo -n "B$b "; timeout -k 10 300 python bench.py --batch $b --steps 128 --warmup 16 --no-secondary 2>/dev/null | j || exit 1
  done
done
timeout -k 10 300 python tools/bench_prefill.py --lens 5,8,15,32 2>/dev/null | grep prompt_tokens | cut -c1-120

#!/usr/bin/env bash
# round-4 attention / short-prompt check: attention tests, combine stamps, long-context bench arms,
# short-prompt prefill.  Every GPU step under its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attn or attention" > gpurun_out/t_attn.log 2>&1 || { tail -40 gpurun_out/t_attn.log; exit 1; }
tail -1 gpurun_out/t_attn.log
timeout -k 10 300 python tools/attn_probe.py --stamps > gpurun_out/attn_stamps.log 2>&1 || { tail -20 gpurun_out/attn_stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/attn_stamps.log | cut -c1-400
for p in 4000 16000; do
  for arm in "AIOS_ATTN_COMBINE=2 AIOS_ATTN_NT=0" "AIOS_ATTN_COMBINE=1 AIOS_ATTN_NT=0" "AIOS_ATTN_COMBINE=1 AIOS_ATTN_NT=1"; do
    echo -n "p$p $arm: "; env $arm timeout -k 10 300 python bench.py --prompt $p --steps 128 --warmup 8 --no-secondary 2>/dev/null | j || exit 1
  done
done
timeout -k 10 300 python tools/bench_prefill.py --lens 2,4,5,8,12,15,32 > gpurun_out/prefill_short.log 2>&1 || { tail -20 gpurun_out/prefill_short.log; exit 1; }
grep -v amdgpu.ids gpurun_out/prefill_short.log | tail -12

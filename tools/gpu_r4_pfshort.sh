#!/usr/bin/env bash
# short-chunk prefill fusions (QKV epilogue RoPE + KV write, split RMSNorm): numerics, then
# AIOS_PREFILL_SHORT_FUSE 0 vs 1 on 5..64-token prompts, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py \
  -k "prefill" > gpurun_out/t_pfshort.log 2>&1 || { tail -40 gpurun_out/t_pfshort.log; exit 1; }
tail -1 gpurun_out/t_pfshort.log
for r in 0 1; do
  for f in 0 1; do
    echo "AIOS_PREFILL_SHORT_FUSE=$f"
    AIOS_PREFILL_SHORT_FUSE=$f timeout -k 10 300 python tools/bench_prefill.py --lens 5,8,15,32,64 > gpurun_out/pfs_$f.log 2>&1 \
      || { tail -20 gpurun_out/pfs_$f.log; exit 1; }
    grep -v amdgpu.ids gpurun_out/pfs_$f.log | cut -c1-160
  done
done

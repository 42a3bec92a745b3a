#!/usr/bin/env bash
# hipBLASLt prefill threshold: AIOS_PREFILL_BLAS_MIN 32 vs 256 (default) on 32..256-token prompts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in 256 32; do
  echo "AIOS_PREFILL_BLAS_MIN=$m"
  AIOS_PREFILL_BLAS_MIN=$m timeout -k 10 300 python tools/bench_prefill.py --lens 16,32,64,128,192,256 > gpurun_out/pfmin_$m.log 2>&1 \
    || { tail -20 gpurun_out/pfmin_$m.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/pfmin_$m.log | cut -c1-160
done

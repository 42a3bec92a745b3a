#!/usr/bin/env bash
# ring GEMM anatomy at B = 8: full kernel vs no dequant (bit 0) vs no MFMA (bit 1) vs bare ring (bit 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for d in 0 1 2 3 4; do
  echo "AIOS_RING_DBG=$d"
  AIOS_RING_DBG=$d timeout -k 10 300 python tools/skinny_probe.py --batch 8 > gpurun_out/ringprobe_$d.log 2>&1 \
    || { tail -20 gpurun_out/ringprobe_$d.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ringprobe_$d.log | cut -c1-200
done

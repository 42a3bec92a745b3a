#!/bin/bash
# batch-1 LDS-DMA ring depth A/B: default RSUB 1, Q6_K matrices at RSUB 2, every matrix at RSUB 2
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do for v in "X=0" "AIOS_LDS_B1_RSUB_Q6=2" "AIOS_LDS_B1_RSUB=2" "AIOS_LDS_B1_RSUB_Q6=0"; do
  env $v timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary > gpurun_out/rs.json 2> gpurun_out/rs.err || { tail -20 gpurun_out/rs.err; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/rs.json | head -1)"
done; done

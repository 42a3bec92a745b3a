#!/bin/bash
# TinyLlama Q4_K_M B=1: LDS-DMA engine threshold A/B (small GEMVs on the engine)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do for kb in 40 16 8; do
  AIOS_GEMV_LDS_MIN_KB=$kb timeout -k 10 300 python bench.py --model tinyllama-1.1b --steps 256 --warmup 16 --no-secondary > gpurun_out/tl.json 2> gpurun_out/tl.err || { tail -20 gpurun_out/tl.err; exit 1; }
  echo "min_kb $kb: $(grep -o '"value": [0-9.]*' gpurun_out/tl.json | head -1)"
done; done

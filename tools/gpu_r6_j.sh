#!/bin/bash
# fp8 long-mode attention: numerics of both schedules at 32k keys, then kernel traces (32k) of each
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
AIOS_ATTN_NB=0 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "attention_decode_fp8_kv and 32768" > gpurun_out/attn0.log 2>&1 || { tail -40 gpurun_out/attn0.log; exit 1; }
tail -n 1 gpurun_out/attn0.log
for nb in 1 0; do
  AIOS_ATTN_NB=$nb BENCH_ARGS="--prompt 32000 --kv-dtype fp8_e4m3" bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  echo "== nb $nb"; head -12 gpurun_out/prof_summary.txt; grep -o '"value": [0-9.]*' gpurun_out/prof.log
done

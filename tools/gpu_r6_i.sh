#!/bin/bash
# fp8 long-mode decode attention with 4 passes in flight: numerics, then 16k / 32k decode NB=4 vs NB=2
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "attention_decode" > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -n 1 gpurun_out/attn_tests.log
for p in 32000 16000 4000; do for nb in 1 0; do
  AIOS_ATTN_NB=$nb timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p --kv-dtype fp8_e4m3 > gpurun_out/nb.json 2> gpurun_out/nb.err || { tail -20 gpurun_out/nb.err; exit 1; }
  echo "fp8 nb $nb prompt $p: $(grep -o '"value": [0-9.]*' gpurun_out/nb.json)"
done; done

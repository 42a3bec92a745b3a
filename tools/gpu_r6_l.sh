#!/bin/bash
# decode attention with per-key-group softmax state: numerics, then long-context decode bf16 / fp8
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "attention_decode or attn" > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -n 1 gpurun_out/attn_tests.log
for p in 32000 16000 4000 128; do for kv in fp8_e4m3 bf16; do
  timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p --kv-dtype $kv > gpurun_out/lc.json 2> gpurun_out/lc.err || { tail -20 gpurun_out/lc.err; exit 1; }
  echo "$kv prompt $p: $(grep -o '"value": [0-9.]*' gpurun_out/lc.json)"
done; done

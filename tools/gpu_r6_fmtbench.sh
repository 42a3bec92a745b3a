#!/bin/bash
# batch-1 decode of Mistral-7B in the load-time-expanded GGUF recipes (bf16 matrices in HBM, the mixes'
# native K-quant tensors kept)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in Q3_K_M Q2_K IQ4_XS; do
  timeout -k 10 300 python bench.py --recipe $r --steps 128 --warmup 8 --no-secondary > gpurun_out/fb.json 2> gpurun_out/fb.err || { tail -20 gpurun_out/fb.err; exit 1; }
  echo "$r: $(grep -o '"value": [0-9.]*' gpurun_out/fb.json | head -1) $(grep -o '"weight_gb": [0-9.]*' gpurun_out/fb.json | head -1)"
done

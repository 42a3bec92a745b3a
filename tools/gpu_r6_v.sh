#!/bin/bash
# batch-1 short-context decode attention knobs (Mistral, 128-token prompt)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do for v in "X=0" "AIOS_ATTN_GROUPED_MIN=1" "AIOS_ATTN_SHORT_P=2" "AIOS_ATTN_XCD=0"; do
  env $v timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary > gpurun_out/ak.json 2> gpurun_out/ak.err || { tail -20 gpurun_out/ak.err; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/ak.json | head -1)"
done; done

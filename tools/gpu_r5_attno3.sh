#!/bin/bash
# fused attention -> O: kernel time with the dependency wait off (1) / the attention role off (2)
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2; do
  AIOS_ATTN_O_DBG=$d AIOS_ATTN_O=1 timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  echo "DBG=$d $(grep 'attn_o_kernel' gpurun_out/prof_summary.txt | head -1)"
done
for v in 0 1 0 1; do
  AIOS_ATTN_O=$v timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-secondary > gpurun_out/attno_b$v.json 2>gpurun_out/attno_b$v.err || { tail -20 gpurun_out/attno_b$v.err; exit 1; }
  echo "ATTN_O=$v $(cat gpurun_out/attno_b$v.json | tail -1 | cut -c60-100)"
done

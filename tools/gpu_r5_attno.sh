#!/bin/bash
# fused attention -> O launch: numerics, then the headline bench with the fusion off / on
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  -k "attention_o_one_launch or greedy_decode or graph_loop" > gpurun_out/attno_tests.log 2>&1 || { tail -40 gpurun_out/attno_tests.log; exit 1; }
tail -3 gpurun_out/attno_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "attn or gemv" > gpurun_out/attno_k.log 2>&1 || { tail -40 gpurun_out/attno_k.log; exit 1; }
tail -2 gpurun_out/attno_k.log
for v in 0 1 0 1; do
  AIOS_ATTN_O=$v timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-secondary > gpurun_out/attno_b$v.json 2>gpurun_out/attno_b$v.err || { tail -20 gpurun_out/attno_b$v.err; exit 1; }
  echo "ATTN_O=$v $(cat gpurun_out/attno_b$v.json | tail -1 | cut -c1-120)"
done
export AIOS_ATTN_O=1
timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
head -16 gpurun_out/prof_summary.txt

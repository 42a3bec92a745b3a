#!/bin/bash
# Q2_K / Q3_K_M / Q4_1 / Q5_0 / Q5_1 GGUFs through the GPU loader (bf16 expansion) vs the fp32 reference
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_engine_gpu.py \
  -k "expanded_formats or prefill_logits_match or greedy_decode_token_exact" > gpurun_out/t_fmt.log 2>&1 || { tail -40 gpurun_out/t_fmt.log; exit 1; }
tail -n 3 gpurun_out/t_fmt.log

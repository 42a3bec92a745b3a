#!/bin/bash
# fused attention -> O launch (kernels/attn_o.hip): numerics, then A/B with profiles
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
  -k "attention_o_one_launch or greedy_decode or graph_loop" > gpurun_out/attno_tests.log 2>&1 || { tail -40 gpurun_out/attno_tests.log; exit 1; }
tail -1 gpurun_out/attno_tests.log
bash tools/ab.sh -n 2 -p -b "--steps 64 --warmup 8 --no-secondary" off="AIOS_ATTN_O=0" on="AIOS_ATTN_O=1" || exit 1
grep -h "attn_o_kernel\|attn_decode_kernel\|gemv_q8_rows<12, 12, 1, 2, 1>" gpurun_out/prof_off.txt gpurun_out/prof_on.txt | head -6
bash tools/ab.sh -n 1 -b "--steps 64 --warmup 8 --no-secondary --prompt 1500" loff="AIOS_ATTN_O=0" lon="AIOS_ATTN_O=1" || exit 1

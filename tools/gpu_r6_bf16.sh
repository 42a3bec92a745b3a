#!/bin/bash
# BF16 LDS-DMA engine: numerics, TP fused self-test, decode profile
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "bf16 or BF16 or norm_resid_swiglu" > gpurun_out/t_bf16.log 2>&1 || { tail -40 gpurun_out/t_bf16.log; exit 1; }
tail -3 gpurun_out/t_bf16.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_tp.py \
  -k "fused_epilogue_int8 and 2" > gpurun_out/t_tp.log 2>&1 || { tail -40 gpurun_out/t_tp.log; exit 1; }
tail -3 gpurun_out/t_tp.log
MODEL=tinyllama-1.1b BENCH_ARGS="--recipe BF16" timeout -k 10 600 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/prof_tinyllama_bf16.txt
head -16 gpurun_out/prof_tinyllama_bf16.txt
timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary --model tinyllama-1.1b --recipe BF16 > gpurun_out/bf16.json 2>gpurun_out/bf16.err || { tail -20 gpurun_out/bf16.err; exit 1; }
cat gpurun_out/bf16.json

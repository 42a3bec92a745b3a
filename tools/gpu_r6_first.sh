#!/bin/bash
# round-6 first contact: BF16 TinyLlama decode profile (config 2's engine path), fixed-length goal->plan
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODEL=tinyllama-1.1b BENCH_ARGS="--recipe BF16" timeout -k 10 600 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/prof_tinyllama_bf16.txt
head -24 gpurun_out/prof_tinyllama_bf16.txt
timeout -k 10 300 python -u tools/bench_goal_plan.py --goals 8 --burst 3 > gpurun_out/goal_plan.json 2> gpurun_out/goal_plan.err || { tail -20 gpurun_out/goal_plan.err; exit 1; }
cat gpurun_out/goal_plan.json
timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary > gpurun_out/b1.json 2> gpurun_out/b1.err || { tail -20 gpurun_out/b1.err; exit 1; }
cat gpurun_out/b1.json

#!/bin/bash
# round-5 decode profiles + long-context bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/prof_mistral.txt
MODEL=tinyllama-1.1b timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/prof_tinyllama.txt
for p in 4000 16000 32000; do
  timeout -k 10 600 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p > gpurun_out/lc_$p.json 2> gpurun_out/lc_$p.err || { tail -20 gpurun_out/lc_$p.err; exit 1; }
  echo "prompt $p: $(grep -o '"value": [0-9.]*, "unit": "tokens/s", "n_gpus": 1, "steps": 128, "warmup": 8, "ms_per_step": [0-9.]*' gpurun_out/lc_$p.json)"
done
BENCH_ARGS="--prompt 4000" timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/prof_mistral_4k.txt
head -12 gpurun_out/prof_mistral_4k.txt

#!/bin/bash
# round-6 profiles: Mistral B=1 decode kernel trace; 512-token prefill per-projection table
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/decode_mistral_r6.txt; grep -o '"value": [0-9.]*' gpurun_out/prof.log >> gpurun_out/decode_mistral_r6.txt
head -14 gpurun_out/decode_mistral_r6.txt
rm -rf gpurun_out/prof
BENCH_ARGS="--lens 512" bash tools/prof_prefill.sh > /dev/null 2>&1 || { tail -20 gpurun_out/pf/log; exit 1; }
python3 tools/prof_prefill_table.py gpurun_out/pf/run_kernel_trace.csv --tokens 512 > gpurun_out/pf512_table.txt 2>&1
grep '^{' gpurun_out/pf/log | tail -1 >> gpurun_out/pf512_table.txt
cat gpurun_out/pf512_table.txt
rm -rf gpurun_out/pf

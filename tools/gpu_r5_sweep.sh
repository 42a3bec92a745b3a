#!/bin/bash
# round 5: prefill GEMM tile x split sweep + prefill kernel profile (Mistral-7B Q4_K_M)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/prof_pf
export TMPDIR=/tmp
timeout -k 10 400 python tools/bench_gemm.py --pf-sweep --ms 64,128,256,512,1024,2048 --json gpurun_out/r5_sweep.jsonl > gpurun_out/r5_sweep.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pf -o pf --output-format csv -- python3 tools/bench_prefill.py --lens 512,2048 > gpurun_out/prof_pf/bench.log 2>&1
echo rc=$?

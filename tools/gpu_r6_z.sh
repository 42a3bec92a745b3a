#!/bin/bash
# 50-token response latency over gRPC, TinyLlama and Mistral-7B (reference targets 200 / 100 ms)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python tools/bench_response.py --json gpurun_out/response_r6.json > gpurun_out/response.log 2>&1 || { tail -30 gpurun_out/response.log; exit 1; }
tail -n 1 gpurun_out/response.log

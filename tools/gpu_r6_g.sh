#!/bin/bash
# Q5_K / Q4_0 / Q8_0 on the prefill GEMM: numerics tests, prefill bench per recipe; copy-engine A/B on the
# pipelined service decode (goal -> plan, gRPC stream)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_pf" > gpurun_out/pf_tests.log 2>&1 || { tail -40 gpurun_out/pf_tests.log; exit 1; }
tail -3 gpurun_out/pf_tests.log
for r in Q5_K_M Q8_0 Q4_0; do
  timeout -k 10 300 python tools/bench_prefill.py --recipe $r --lens 128,512,2048 > gpurun_out/pf_$r.jsonl 2> gpurun_out/pf.err || { tail -20 gpurun_out/pf.err; exit 1; }
  cat gpurun_out/pf_$r.jsonl
done

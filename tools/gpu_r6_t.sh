#!/bin/bash
# prefill GEMM ring depth (AIOS_PF4_NS build): GEMM tests, prefill per recipe
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm_pf" > gpurun_out/pf_tests.log 2>&1 || { tail -40 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
for r in Q4_K_M Q4_K_M Q5_K_M BF16; do
  timeout -k 10 300 python tools/bench_prefill.py --recipe $r --lens 128,512,2048 > gpurun_out/pfn.jsonl 2> gpurun_out/pfn.err || { tail -20 gpurun_out/pfn.err; exit 1; }
  echo "$r: $(grep -o '"prompt_tokens": [0-9]*, "ms": [0-9.]*' gpurun_out/pfn.jsonl | tr '\n' ' ')"
done

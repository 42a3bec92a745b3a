#!/bin/bash
# round 5: prefill GEMM (gemm_pf.hip) numerics + per-shape timing on one MI355X
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_pf" > gpurun_out/r5_pf_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r5_pf_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/bench_gemm.py --ms 64,128,512,2048 --json gpurun_out/r5_pf_gemm.jsonl > gpurun_out/r5_pf_gemm.log 2>&1

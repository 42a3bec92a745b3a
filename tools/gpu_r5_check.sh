#!/bin/bash
# round 5: GEMM + engine GPU tests, then the prefill bench
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py > gpurun_out/r5_check_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r5_check_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/bench_prefill.py --lens 64,128,512,2048 > gpurun_out/r5_check_prefill.log 2>&1

#!/bin/bash
# engine + TP GPU tests after the ADVICE r4 fixes (fused-epilogue launch reporting, comm self-test)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py > gpurun_out/eng_tests.log 2>&1 || { tail -40 gpurun_out/eng_tests.log; exit 1; }
tail -1 gpurun_out/eng_tests.log
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_tp.py > gpurun_out/tp_tests.log 2>&1 || { tail -60 gpurun_out/tp_tests.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED|passed|failed" gpurun_out/tp_tests.log | tail -20

#!/bin/bash
# prefill GEMM: numerics (kernel + engine prefill tests), the M = 512 plan sweep, prefill tok/s
set -o pipefail
mkdir -p gpurun_out/pfc
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_pf" > gpurun_out/pfc/tests.log 2>&1 || { tail -30 gpurun_out/pfc/tests.log; exit 1; }
tail -1 gpurun_out/pfc/tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "prefill" > gpurun_out/pfc/tests2.log 2>&1 || { tail -30 gpurun_out/pfc/tests2.log; exit 1; }
tail -1 gpurun_out/pfc/tests2.log
[ -n "$NOSWEEP" ] || timeout -k 10 300 python tools/bench_gemm.py --pf-sweep --ms ${SWEEP_MS:-512} --shapes qkv,o,down_q6k --no-torch > gpurun_out/pfc/sweep.log 2>&1 || { tail -20 gpurun_out/pfc/sweep.log; exit 1; }
timeout -k 10 300 python tools/bench_prefill.py --lens 64,128,512,2048 > gpurun_out/pfc/bench.log 2>&1 || { tail -20 gpurun_out/pfc/bench.log; exit 1; }
grep '^{' gpurun_out/pfc/bench.log

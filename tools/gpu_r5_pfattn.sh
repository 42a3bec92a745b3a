#!/bin/bash
# prefill attention: numerics, prefill tok/s, kernel-time profile at 2048 tokens
set -o pipefail
ROOT=$PWD
mkdir -p gpurun_out/pfa
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "prefill" > gpurun_out/pfa_tests.log 2>&1 || { tail -30 gpurun_out/pfa_tests.log; exit 1; }
tail -1 gpurun_out/pfa_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py -k "prefill" > gpurun_out/pfa_tests2.log 2>&1 || { tail -30 gpurun_out/pfa_tests2.log; exit 1; }
tail -1 gpurun_out/pfa_tests2.log
timeout -k 10 300 python tools/bench_prefill.py --lens 64,128,512,2048 > gpurun_out/pfa_bench.log 2>&1 || { tail -20 gpurun_out/pfa_bench.log; exit 1; }
grep '^{' gpurun_out/pfa_bench.log | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/pfa -o run --output-format csv -- \
  python3 $ROOT/tools/bench_prefill.py --lens 2048 > $ROOT/gpurun_out/pfa/log 2>&1 || { echo prof failed; tail -5 $ROOT/gpurun_out/pfa/log; exit 1; }
head -12 $ROOT/gpurun_out/pfa/run_kernel_stats.csv | cut -c1-160

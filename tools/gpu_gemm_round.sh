#!/bin/bash
# GPU session: GEMM kernel tests + GEMM bench.  Stops at the first fault / timeout / abort.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 420 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" > gpurun_out/t_gemm.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/t_gemm.log
ok $rc || exit $rc
timeout -k 10 300 python -u tools/bench_gemm.py ${BENCH_ARGS} --json gpurun_out/bench_gemm.jsonl > gpurun_out/bench_gemm.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_gemm.log
exit $rc

#!/usr/bin/env bash
# One GPU iteration: GPU tests (optional filter), the headline bench, optionally a rocprof decode
# profile.  Every step runs under its own limit and the script stops at the first failure.
#   TESTS="tests/test_kernels_gpu.py -k qkv" BENCH="--steps 256 --no-secondary" PROF=1 tools/gpu_check.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-3} | cut -c1-700; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
if [ -n "${TESTS:-}" ]; then
  eval "run tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $TESTS"
fi
if [ -n "${BENCH:-}" ]; then
  eval "TAILN=1 run bench 400 python bench.py $BENCH"
fi
if [ -n "${PROF:-}" ]; then
  TAILN=12 run prof 700 bash tools/prof_decode.sh
fi

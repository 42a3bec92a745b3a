#!/usr/bin/env bash
# GPU iteration for the persistent decode kernel: its tests, then the B=1 bench with it off / on
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-3}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
[ -n "${NOTEST:-}" ] || run t_mk 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_decode_mk_gpu.py
[ -z "${EXTRA_K:-}" ] || run t_extra 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "$EXTRA_K"
TAILN=1 run bench_off 240 python bench.py --steps 128 --warmup 8 --no-secondary ${BENCH_ARGS:-}
TAILN=1 AIOS_MK=1 run bench_on 240 python bench.py --steps 128 --warmup 8 --no-secondary ${BENCH_ARGS:-}
[ -z "${PROF:-}" ] || bash tools/prof_decode.sh > /dev/null

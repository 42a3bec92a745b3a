#!/usr/bin/env bash
# GPU validation run used with gpurun: smoke -> pytest -m gpu -> bench (-> optional rocprof).
# Each GPU step has its own time limit; a crash/abort/timeout ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "[gpu_check] $name start $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_check] $name rc=$rc $(date +%T)"
  tail -n 5 "gpurun_out/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
MODE=${1:-all}
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 1200 python -m pytest tests -m gpu -q --maxfail=30 -p no:cacheprovider
  rc=$?; if fatal $rc; then exit $rc; fi
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 900 python bench.py ${BENCH_ARGS:-} || exit 1
fi
if [ "${PROFILE:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
  step rocprof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python bench.py --steps 64 --warmup 8 --no-secondary || exit 1
fi
echo "[gpu_check] done"

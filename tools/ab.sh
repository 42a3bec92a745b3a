#!/usr/bin/env bash
# Same-box A/B runner (replaces the round-1/2 one-off tools/gpu_*_ab.sh scripts; git history keeps
# them and the profiles/ summaries they produced).  Runs optional tests once, then every arm of the
# experiment back to back, REPS times interleaved, and prints one bench.py JSON line per run.
#
#   tools/ab.sh [-n REPS] [-t "pytest args"] [-b "bench.py args"] [-c "command"] [-p]
#               NAME='ENV=VAL ...' [NAME='...' ...]
#
#   -c  run this command per arm instead of `python bench.py ARGS` (e.g. "python tools/bench_prefill.py
#       --lens 512,2048", "python tools/bench_gemm.py --pf-sweep")
#   -p  also take a rocprofv3 kernel trace of the decode loop per arm (tools/prof_decode.sh; summary in
#       gpurun_out/prof_<name>.txt)
#
# e.g. through gpurun:
#   gpurun -- 'tools/ab.sh -n 2 -b "--batch 32 --steps 32 --warmup 4 --no-secondary" \
#              s8="AIOS_SKINNY_SMAX=8" s16="AIOS_SKINNY_SMAX=16"'
# Logs land in gpurun_out/ab_<name>_<rep>.log; every step runs under its own time limit and the
# script stops at the first failure (no GPU step is retried).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
REPS=1; TESTS=""; BARGS="--steps 128 --warmup 8 --no-secondary"; T=${AB_TIMEOUT:-300}; CMD=""; PROF=0
while getopts "n:t:b:c:p" o; do
  case $o in n) REPS=$OPTARG ;; t) TESTS=$OPTARG ;; b) BARGS=$OPTARG ;; c) CMD=$OPTARG ;; p) PROF=1 ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
run() {
  local name=$1; shift
  timeout -k 10 "$T" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -1 | cut -c1-400
  [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 "gpurun_out/$name.log"; exit 1; }
}
if [ -n "$TESTS" ]; then
  eval "run ab_tests python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS"
fi
for ((r = 0; r < REPS; r++)); do
  for arm in "$@"; do
    name=${arm%%=*}; envs=${arm#*=}
    echo "== $name ($envs) rep $r"
    if [ -n "$CMD" ]; then eval "run ab_${name}_$r env $envs $CMD"; else eval "run ab_${name}_$r env $envs python bench.py $BARGS"; fi
    if [ $PROF -eq 1 ] && [ $r -eq 0 ]; then
      eval "env $envs timeout -k 10 700 bash tools/prof_decode.sh" > /dev/null 2>&1 || { echo "[$name] profile failed"; exit 1; }
      cp gpurun_out/prof_summary.txt "gpurun_out/prof_$name.txt" && head -3 "gpurun_out/prof_$name.txt"
    fi
  done
done

#!/usr/bin/env bash
# rocprofv3 kernel trace of the Mistral decode loop; summary -> gpurun_out/prof_summary.txt
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODEL=${MODEL:-mistral-7b}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 32 --warmup 4 --no-secondary --model "$MODEL" ${BENCH_ARGS:-} > "$ROOT/gpurun_out/prof.log" 2>&1
cd "$ROOT"
python3 tools/prof_step.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/prof_summary.txt
head -40 gpurun_out/prof/run_kernel_stats.csv >> gpurun_out/prof_summary.txt
cat gpurun_out/prof_summary.txt | head -30

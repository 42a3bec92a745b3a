#!/bin/bash
# where the pipelined service decode spends the time between forward graphs (goal -> plan path)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $ROOT/gpurun_out/gp -o run --output-format csv -- \
  python3 $ROOT/tools/bench_goal_plan.py --goals 2 --burst 1 --warmup 1 > $ROOT/gpurun_out/gp_prof.log 2>&1 || { tail -20 $ROOT/gpurun_out/gp_prof.log; exit 1; }
cd $ROOT
python3 tools/step_gaps.py gpurun_out/gp/run_kernel_trace.csv gpurun_out/gp/run_memory_copy_trace.csv > gpurun_out/gp_gaps.txt; rm -rf gpurun_out/gp; cat gpurun_out/gp_gaps.txt
grep -o '"ms_per_token": [0-9.]*' gpurun_out/gp_prof.log

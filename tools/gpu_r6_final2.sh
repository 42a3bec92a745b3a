#!/bin/bash
# round-6 end validation, part 1: every GPU test and smoke() (bench.py: tools/gpu_r6_final3.sh)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests > gpurun_out/t_final.log 2>&1 || { tail -40 gpurun_out/t_final.log; exit 1; }
tail -n 1 gpurun_out/t_final.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log

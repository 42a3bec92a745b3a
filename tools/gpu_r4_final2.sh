#!/usr/bin/env bash
# round-4 closing validation of the committed tree: every GPU test, smoke(), the driver's default bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_final2.log 2>&1 \
  || { tail -40 gpurun_out/t_final2.log; exit 1; }
tail -1 gpurun_out/t_final2.log
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' 2>&1 | grep -v amdgpu.ids | tail -2
timeout -k 10 900 python bench.py > gpurun_out/bench_final2.log 2>&1 || { tail -20 gpurun_out/bench_final2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_final2.log | tail -1 > gpurun_out/bench_final2.json
cut -c1-600 gpurun_out/bench_final2.json

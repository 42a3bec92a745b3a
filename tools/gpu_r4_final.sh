#!/usr/bin/env bash
# round-4 validation: every GPU test, the driver's default bench (all secondaries), B=1 against the
# cmp_r4c build on the same box, and the B=1 rocprof decode profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
j() { python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_final.log 2>&1 \
  || { tail -40 gpurun_out/t_final.log; exit 1; }
tail -1 gpurun_out/t_final.log
timeout -k 10 900 python bench.py > gpurun_out/bench_final.log 2>&1 || { tail -20 gpurun_out/bench_final.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_final.log | tail -1 | cut -c1-400
for r in 0 1; do
  for d in cmp_r4c .; do
    echo -n "B1 $d "; (cd $d && timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary 2>/dev/null | j) || exit 1
  done
done
timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 && head -12 gpurun_out/prof_summary.txt
